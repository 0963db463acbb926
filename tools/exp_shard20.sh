#!/bin/bash
# The driver's multi-GPU command rehearsed on one GPU: a 20-frame call per rank (4-row stripes), N = 1..8,
# ranks one after another (tools/exp_shard.py), by batch dealing (env configs as arguments, "-" default).
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=8
for v in "${@:--}"; do
  e="RT_NONE=1"; [ "$v" != "-" ] && e="${v//,/ }"
  env $e EXP_F=20 EXP_S=4 EXP_REPS=7 timeout -k 10 300 python3 tools/exp_shard.py ${NS:-1 2 4 8} 2>/dev/null | sed "s/^/$v /"
done
