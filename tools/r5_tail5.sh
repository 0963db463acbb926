#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t5
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t5/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5t5/tests.log; [ $rc -ne 0 ] && exit $rc
export EXP_REPS=21 RT_KTIME=1
timeout -k 10 900 python3 tools/exp_lone.py RT_TAIL=0 RT_TAIL=500 RT_TAIL=1000 RT_TAIL=2000 RT_TAIL=4000 RT_TAIL=8000 \
  RT_TAIL=2000,RT_TAIL_GRID=2048 RT_TAIL=0 2>&1 | tee gpurun_out/r5t5/lone.txt
