#!/bin/bash
# The group rehearsal of DESIGN §6: frames per call x stripe rows, N = 1 and 8 (tools/exp_shard.py), with the
# bench's and the CLI's 8 hardware queues.
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=8
for F in 1 6 96; do for S in 4 8; do
  EXP_F=$F EXP_S=$S EXP_REPS=7 timeout -k 10 300 python3 tools/exp_shard.py 1 2 4 8 2>/dev/null | sed "s/^/F=$F /"
done; done
