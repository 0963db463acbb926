#!/bin/bash
# The multi-GPU row-stripe shards rehearsed on one GPU: per-rank render time, ranks rendered one
# after another (tools/exp_shard.py, max over ranks, no gather), N = 1, 2, 4, 8, 4-row stripes, with the
# bench's and the CLI's 8 hardware queues, by frames per call (env FRAMES, default "1 6 20 96": a lone frame,
# a 6-camera call, the driver's --steps 20 call, the bench's 96-frame calls).  Arguments: env configs
# ("-" = defaults, "K=V,K2=W" otherwise).
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=8
for v in "${@:--}"; do
  e="RT_NONE=1"; [ "$v" != "-" ] && e="${v//,/ }"
  for F in ${FRAMES:-1 6 20 96}; do
    env $e EXP_F=$F EXP_S=${STRIPE:-4} EXP_REPS=7 timeout -k 10 300 python3 tools/exp_shard.py ${NS:-1 2 4 8} 2>/dev/null \
      | sed "s/^/$v F=$F /"
  done
done
