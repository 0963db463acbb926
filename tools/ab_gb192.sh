#!/bin/bash
# 96-frame-call bench lines (192 steps) per env config, REPS interleaved rounds
cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq 1 ${REPS:-2}); do for c in "$@"; do
  e="RT_NONE=1"; [ "$c" != "-" ] && e="${c//,/ }"
  env $e timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/ab1/g.jsonl 2>/dev/null || { echo "fail $c"; exit 1; }
  echo "$c: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab1/g.jsonl') if l.startswith('{')][-1]); print(d['ms_per_step'])")"
done; done
