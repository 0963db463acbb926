#!/bin/bash
# GPU session: smoke, parity tests, bench for every render path.
#   bash tools/gpu_session.sh [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -k "$K" > gpurun_out/gpu_tests.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/gpu_tests.log 2>&1
fi
rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
for P in mega wave; do
  RT_PATH=$P timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$P.log 2>&1
  rc=$?
  echo "bench $P rc=$rc"; grep '^{' gpurun_out/bench_$P.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
