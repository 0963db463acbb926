#!/bin/bash
# GPU A/B of bench configurations with bench arguments:  stdin lines "ENV=a,ENV2=b ARGS..." ("-" = default env)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r envs args; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  [ "$envs" = "-" ] && envs="RT_NONE=1"
  env ${envs//,/ } timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline $args > gpurun_out/ab2_$i.log 2>&1 || { echo "fail $envs $args"; tail -3 gpurun_out/ab2_$i.log; exit 1; }
  echo "[$envs | $args] $(grep '^{' gpurun_out/ab2_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], "lat", d["config"]["frame_latency_ms"], "slots", d["config"]["workspace_slots"])')"
done
exit 0
