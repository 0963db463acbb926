#!/bin/bash
# One GPU call: the GPU test suite, then (if green) the bench line at the driver's command and optional
# extras.   bash tools/gpu_check.sh TAG [extra command...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-chk}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench20.jsonl 2> gpurun_out/$TAG/bench20.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/line_summary.py gpurun_out/$TAG/bench20.jsonl
if [ $# -gt 0 ]; then "$@"; fi
