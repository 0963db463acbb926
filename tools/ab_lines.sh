#!/bin/bash
# GPU A/B of full bench lines (frame batches): stdin lines "ENV=a,ENV2=b" ("-" = default env); prints the
# line's ms/frame, latency and the one-slot per-kernel times (kernel_ms_one_slot.batched)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r envs args; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  [ "$envs" = "-" ] && envs="RT_NONE=1"
  env ${envs//,/ } timeout -k 10 240 python bench.py --steps 96 --warmup 5 --no-cpu-baseline $args > gpurun_out/abl_$i.log 2>&1 || { echo "fail $envs $args"; tail -3 gpurun_out/abl_$i.log; exit 1; }
  echo "[$envs | $args] $(grep '^{' gpurun_out/abl_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); k=d["kernel_ms_one_slot"]["batched"]; print(d["ms_per_step"], "lat", d["single_frame"]["ms"], "one-slot", {n: v for n, v in k.items() if n.startswith("k_")})')"
done
exit 0
