#!/bin/bash
# Batched bench (ms/frame) and single-frame time (exp_shard F=1, N=1) under several env settings.
#   bash tools/sweep_both.sh "ENV=.." ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --steps ${SB_STEPS:-64} --warmup 3 --no-cpu-baseline $SB_ARGS > gpurun_out/sb_$i.log 2>&1 || exit 1
  b=$(grep '^{' gpurun_out/sb_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['config']['frame_latency_ms'])")
  env $cfg EXP_F=32 timeout -k 10 100 python3 tools/exp_shard.py 8 > gpurun_out/sb8_$i.log 2>&1 || exit 1
  n8=$(grep '^{' gpurun_out/sb8_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['max_ms'])")
  echo "[$cfg] batched ms/Mray/latency: $b  N8-shard: $n8"
done
