#!/bin/bash
# A/B of bench lines at the driver's command (--steps 20 --warmup 5), REPS rounds interleaved:
#   stdin lines "ENV=a,ENV2=b [extra bench args]" ("-" = default env)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
REPS=${REPS:-2}
mapfile -t CFG
for r in $(seq 1 $REPS); do
  i=0
  for line in "${CFG[@]}"; do
    read -r envs args <<< "$line"
    [ -z "$envs" ] && continue
    i=$((i+1))
    [ "$envs" = "-" ] && envs="RT_NONE=1"
    env ${envs//,/ } timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline $args > gpurun_out/ab/$r.$i.log 2>&1 \
      || { echo "fail $envs $args"; tail -3 gpurun_out/ab/$r.$i.log; exit 1; }
    echo "[$envs | $args] $(grep '^{' gpurun_out/ab/$r.$i.log | python3 tools/line_summary.py)"
  done
done
exit 0
