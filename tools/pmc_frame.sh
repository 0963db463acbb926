#!/bin/bash
# SQ counters per kernel, one frame per dispatch (bench --inflight 1), for several env settings
# (e.g. RT_LIB=... for an A/B build).  One rocprofv3 pass per counter group.
#   bash tools/pmc_frame.sh "ENV=.." ...   ("-" = default env)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmcf
mkdir -p $OUT
i=0
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg="RT_NONE=1"
  i=$((i+1))
  g=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY" \
             "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"; do
    g=$((g+1))
    env $cfg timeout -k 5 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/c${i}g$g -o run --output-format csv -- python3 bench.py --steps ${STEPS:-8} --warmup 2 --inflight ${INFLIGHT:-1} --no-cpu-baseline > $OUT/c${i}g$g.log 2>&1
    rc=$?
    echo "[$cfg] pass $g rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 $OUT/c${i}g$g.log; exit $rc; fi
  done
  python3 - "$OUT" "$i" "$cfg" <<'PY'
import csv, collections, glob, sys, os, re
out, i, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "c%sg1" % i, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_]+)(<[^>]*>)?", r["Kernel_Name"])
        if m and "true" not in (m.group(2) or ""):
            dur[m.group(1)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for f in glob.glob(os.path.join(out, "c%sg*" % i, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_]+)(<[^>]*>)?", r["Kernel_Name"])
        if not m or "true" in (m.group(2) or ""): continue
        agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("==", cfg)
for k, d in sorted(agg.items()):
    v = {c: sum(x) / len(x) for c, x in d.items()}
    valu = v.get("SQ_INSTS_VALU", 0)
    lanes = v.get("SQ_THREAD_CYCLES_VALU", 0) / valu if valu else 0
    print("  %-12s VALU %8.2fM SALU %7.2fM VMEM %6.2fM LDS %5.2fM BR %6.2fM cvt %6.2fM fma %6.2fM mul %6.2fM add %6.2fM  thr/valu %5.1f  "
          "wave_cyc %7.1fM active %4.2f wait %4.2f waitinst %4.2f waves %d" % (
          k, valu / 1e6, v.get("SQ_INSTS_SALU", 0) / 1e6, v.get("SQ_INSTS_VMEM_RD", 0) / 1e6, v.get("SQ_INSTS_LDS", 0) / 1e6,
          v.get("SQ_INSTS_BRANCH", 0) / 1e6, v.get("SQ_INSTS_VALU_CVT", 0) / 1e6, v.get("SQ_INSTS_VALU_FMA_F32", 0) / 1e6,
          v.get("SQ_INSTS_VALU_MUL_F32", 0) / 1e6, v.get("SQ_INSTS_VALU_ADD_F32", 0) / 1e6, lanes,
          v.get("SQ_WAVE_CYCLES", 0) / 1e6, v.get("SQ_ACTIVE_INST_ANY", 0) / max(1, v.get("SQ_WAVE_CYCLES", 1)),
          v.get("SQ_WAIT_ANY", 0) / max(1, v.get("SQ_WAVE_CYCLES", 1)), v.get("SQ_WAIT_INST_ANY", 0) / max(1, v.get("SQ_WAVE_CYCLES", 1)),
          v.get("SQ_WAVES", 0)))
    if dur.get(k):
        us = sum(dur[k]) / len(dur[k])
        print("  %-12s avg dispatch %8.1f us   VALU issue util (2 cyc/VALU, 1024 SIMDs, 2.1 GHz) %.2f" % (
              k, us, valu * 2 / (us * 1e-6 * 1024 * 2.1e9)))
PY
done
exit 0
