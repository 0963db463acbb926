#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of the bench, one frame at a time
# and batched, under several env settings.   bash tools/kt_cmp.sh "ENV=.." ...   ("-" = default env)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg="RT_NONE=1"
  for inflight in 1 96; do
    i=$((i+1))
    env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ktc$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --inflight $inflight --no-cpu-baseline > gpurun_out/ktc$i.log 2>&1
    rc=$?
    echo "[$cfg inflight=$inflight] rc=$rc $(grep '^{' gpurun_out/ktc$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
    f=$(find gpurun_out/ktc$i -name '*kernel_stats.csv' | head -1)
    python3 - "$f" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    n = re.search(r"(k_[a-z_0-9]+)(<[^>]*>)?", r["Name"])
    if n and int(r["Calls"]) > 2 and "true" not in (n.group(2) or ""):
        print("   %-22s calls=%-4s avg_us=%.1f" % (n.group(1) + (n.group(2) or ""), r["Calls"], float(r["AverageNs"]) / 1e3))
PY
    [ $rc -ne 0 ] && exit 1
  done
done
exit 0
