#!/bin/bash
# ms per frame of one rt_render_frames_device call of F frames (C3, one rank, 4-row stripes) by the
# minimum batch size (RT_BATCH_MIN), tools/exp_shard.py at N = 1.   bash tools/exp_callsize.sh "F..." "B..."
cd "$GRAFT_REPO_ROOT" || exit 1
for F in ${1:-2 4 6 12 20 32 96}; do for B in ${2:-1 2 3 4 6 8}; do
  r=$(EXP_F=$F EXP_S=4 EXP_REPS=7 RT_BATCH_MIN=$B timeout -k 10 120 python3 tools/exp_shard.py 1 2>/dev/null | tail -1)
  echo "F=$F BATCH_MIN=$B $r"
done; done
