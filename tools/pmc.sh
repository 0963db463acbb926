#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the bench.
#   bash tools/pmc.sh TAG "ENV=.." "group1 counters" "group2 counters" ...
# A group that rocprofv3 rejects is skipped (short timeout), the rest continue.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
ENVS=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  env $ENVS timeout -k 5 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timeout: stopping"; break; fi
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys, os, re
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"::(k_[a-z_]+(<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:30]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print("==", k)
    for c, v in sorted(d.items()):
        print("   %-36s %16.1f" % (c, sum(v) / len(v)))
PY
