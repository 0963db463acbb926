#!/bin/bash
# k_tail: parity, then lone-frame medians over the hand-off threshold and per-kernel times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t/tests.log 2>&1
rc=$?; echo "tail tests rc=$rc"; tail -3 gpurun_out/r5t/tests.log; [ $rc -ne 0 ] && exit $rc
export EXP_REPS=31
timeout -k 10 600 python3 tools/exp_lone.py RT_TAIL=0 RT_TAIL=1 RT_TAIL=4 RT_TAIL=8 RT_TAIL=16 RT_TAIL=32 RT_TAIL=64 \
   RT_TAIL=0,RT_KTIME=1 RT_TAIL=8,RT_KTIME=1 RT_TAIL=32,RT_KTIME=1 RT_TAIL=0 RT_TAIL=8 2>&1 | tee gpurun_out/r5t/lone.txt
