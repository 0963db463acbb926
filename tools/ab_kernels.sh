#!/bin/bash
# GPU A/B of per-kernel one-slot times (bench.py's RT_KTIME pass, roofline.per_kernel) for env configs:
#   bash tools/ab_kernels.sh "ENV=a,ENV2=b" ...   ("-" = default env)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for envs in "$@"; do
  i=$((i+1))
  [ "$envs" = "-" ] && envs="RT_NONE=1"
  env ${envs//,/ } timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/abk_$i.log 2>&1 || { echo "fail $envs"; tail -3 gpurun_out/abk_$i.log; exit 1; }
  echo "[$envs] $(grep '^{' gpurun_out/abk_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); pk=d["roofline"]["per_kernel"]; print(d["ms_per_step"], " ".join("%s=%.4f" % (k, v["ms_one_slot"]) for k, v in pk.items()))')"
done
exit 0
