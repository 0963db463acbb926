#!/bin/bash
# GPU check after a change: all GPU tests, the default bench, C5, per-rank shard scaling.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 64 --warmup 3 > gpurun_out/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['frame_latency_ms'])"
timeout -k 10 300 python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_c5.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
EXP_F=${EXP_F:-32} timeout -k 10 200 python3 tools/exp_shard.py 1 2 4 8 > gpurun_out/shard.log 2>&1 || exit 1
grep '^{' gpurun_out/shard.log
