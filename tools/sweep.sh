#!/bin/bash
# Parity tests for one path (-k expr) + bench under several env settings.
#   bash tools/sweep.sh "<pytest -k expr>" "ENV=a ENV2=b" "ENV=c" ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
K=$1; shift
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 -k "$K" > gpurun_out/sweep_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc"; tail -4 gpurun_out/sweep_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps ${SWEEP_STEPS:-64} --warmup 3 --no-cpu-baseline > gpurun_out/sweep_$i.log 2>&1
  rc=$?
  ms=$(grep '^{' gpurun_out/sweep_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")
  echo "[$cfg] rc=$rc ms/Mray: $ms"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep_$i.log; exit $rc; fi
done
