#!/bin/bash
# Per-rank shard time (tools/exp_shard.py) under several env settings, on one GPU.
#   bash tools/sweep_shard.sh "WORLDS" "ENV=.." "ENV=.." ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
W=$1; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg EXP_REPS=5 timeout -k 10 120 python3 tools/exp_shard.py $W > gpurun_out/sw$i.log 2>&1
  rc=$?
  echo "[$cfg] rc=$rc"
  grep '^{' gpurun_out/sw$i.log | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); print("   N=%d S=%d max=%.4f min=%.4f" % (d["N"], d["S"], d["max_ms"], d["min_ms"]))'
  [ $rc -ne 0 ] && exit 1
done
exit 0
