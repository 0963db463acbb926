#!/bin/bash
# GPU A/B: parity tests (optional), then the bench under several env settings.
#   bash tools/ab.sh [--tests] "ENV=a" "ENV=b" ...     ("-" = default env)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" = "--tests" ]; then
  shift
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc"; tail -4 gpurun_out/ab_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for cfg in "$@"; do
  i=$((i+1))
  [ "$cfg" = "-" ] && cfg="RT_NONE=1"
  env $cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$i.log 2>&1
  rc=$?
  echo "[$cfg] rc=$rc $(grep '^{' gpurun_out/ab_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], "lat", d["config"]["frame_latency_ms"])')"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$i.log; exit $rc; }
done
exit 0
