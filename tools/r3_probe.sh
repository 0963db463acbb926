#!/bin/bash
# Round-3 probes in one GPU call: occupancy A/B (ab3_cfg.txt), the cooperative-fetch microbenchmark,
# single-walk step latency, and the TA busy counter per kernel (one workspace slot).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab2.sh < tools/ab3_cfg.txt || exit $?
timeout -k 5 120 ./tools/ubench_coop > gpurun_out/ub_coop.txt 2>&1 || { echo "ubench_coop failed"; exit 1; }
echo "ubench_coop ok"
timeout -k 5 120 python3 tools/exp_walk_latency.py > gpurun_out/walk_latency.json 2>&1 || { echo "walk latency failed"; exit 1; }
echo "walk latency ok"
RT_SLOTS=1 timeout -k 5 150 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE -d gpurun_out/pmc_ta -o run --output-format csv -- python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_ta.log 2>&1
echo "pmc rc=$?"
