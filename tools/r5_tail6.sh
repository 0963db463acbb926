#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t6
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t6/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5t6/tests.log; [ $rc -ne 0 ] && exit $rc
export EXP_REPS=21 RT_KTIME=1
timeout -k 10 900 python3 tools/exp_lone.py RT_TAIL=0 RT_TAIL=1000 RT_TAIL=2000 RT_TAIL=4000 RT_TAIL=8000 \
  RT_TAIL=2000,RT_FIN_SPLIT=0 RT_TAIL=4000,RT_FIN_SPLIT=0 RT_TAIL=2000,RT_DCHUNK=1024 \
  RT_TAIL_A=2000 RT_TAIL_A=5000 RT_TAIL_A=20000 RT_TAIL_A=5000,RT_TAIL=2000 RT_TAIL=0 2>&1 | tee gpurun_out/r5t6/lone.txt
timeout -k 10 300 python3 tools/exp_cli.py --phases --reps 7 2>&1 | tee gpurun_out/r5t6/cli_phases.jsonl
for F in 6 96; do for S in 4 8; do
  EXP_F=$F EXP_S=$S EXP_REPS=5 timeout -k 10 300 python3 tools/exp_shard.py 1 8 2>/dev/null | tail -2 | sed "s/^/F=$F S=$S /"
done; done | tee gpurun_out/r5t6/shard.txt
