#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t3
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_fallback.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t3/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5t3/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/exp_walk_latency.py > gpurun_out/r5t3/walk.json 2> gpurun_out/r5t3/walk.err || exit 1
python3 -c "
import json
d = json.load(open('gpurun_out/r5t3/walk.json'))
for k in ('mode0_lanes64', 'mode5_lanes64'):
    print(k, [(x['steps'], x['cyc_per_step']) for x in d[k]])"
export EXP_REPS=21 RT_KTIME=1
timeout -k 10 900 python3 tools/exp_lone.py RT_TAIL=0,RT_DCHUNK=0 RT_TAIL=0 RT_TAIL=64,RT_TAIL_AFTER=900 RT_TAIL=64,RT_TAIL_AFTER=950 \
  RT_TAIL=64,RT_TAIL_AFTER=980 RT_TAIL=64,RT_TAIL_AFTER=800 RT_TAIL=64,RT_TAIL_AFTER=950,RT_GB=384 RT_TAIL=64,RT_TAIL_AFTER=950,RT_GB=256 \
  RT_TAIL=65 RT_TAIL=0,RT_DCHUNK=0 2>&1 | tee gpurun_out/r5t3/lone.txt
