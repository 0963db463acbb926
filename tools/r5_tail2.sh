#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t2
timeout -k 10 300 python3 tools/exp_walk_latency.py > gpurun_out/r5t2/walk.json 2> gpurun_out/r5t2/walk.err || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5t2/walk.json"))
for k, v in d.items():
    print(k, [(x["steps"], x["cyc_per_step"]) for x in v])
PY
export EXP_REPS=21 RT_KTIME=1
timeout -k 10 600 python3 tools/exp_lone.py RT_TAIL=0 RT_TAIL=8 RT_TAIL=2 RT_TAIL=8,RT_GB=256 RT_TAIL=8,RT_GB=128 \
   RT_TAIL=8,RT_TAIL_GRID=1024 RT_TAIL=0,RT_GB=256 2>&1 | tee gpurun_out/r5t2/lone.txt
