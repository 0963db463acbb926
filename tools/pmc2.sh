#!/bin/bash
# Counter list + per-kernel SQ counters for the chain path (one rocprofv3 pass per group).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc2
mkdir -p $OUT
timeout -k 5 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
echo "list rc=$?"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timeout: stopping"; break; fi
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys, os, re
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_]+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:30]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print("==", k)
    for c, v in sorted(d.items()):
        print("   %-36s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
PY
