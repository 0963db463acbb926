#!/bin/bash
# Per-kernel average durations of the bench under several env settings (rocprofv3 --kernel-trace --stats).
#   bash tools/kt_quick.sh "ENV=.." "ENV=.." ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ktq$i -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ktq$i.log 2>&1
  rc=$?
  echo "[$cfg] rc=$rc $(grep '^{' gpurun_out/ktq$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  f=$(find gpurun_out/ktq$i -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    n = re.search(r"(k_[a-z_0-9]+)(<[^>]*>)?", r["Name"])
    if n and int(r["Calls"]) > 1:   # the counting pass launches its kernels once
        print("   %-22s calls=%-4s avg_us=%.1f" % (n.group(1) + (n.group(2) or ""), r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  [ $rc -ne 0 ] && exit 1
done
