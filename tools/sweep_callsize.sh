#!/bin/bash
# Call-size sweep of the batch defaults: ms per frame by frames per call (1, 2, 3, 6, 20,
# 96) for C3 AA1, C3 AA2, mirror_spheres and marbles, the current defaults against round 4's rules
# (RT_COMPACT=1: compact phase-A records in every frame batch; RT_BATCH_SAMPLES=1: no minimum batch size),
# interleaved rounds (tools/ab_quick.py).  Output: gpurun_out/sweep/<scene>.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for sc in "C3_hm_1080p_d6 1" "C3_hm_1080p_d6 2" "mirror_spheres.xml 1" "marbles.xml 1"; do
  read -r scene aa <<< "$sc"
  AB_SCENE=$scene AB_AA=$aa AB_CALLS=1,2,3,6,20,96 AB_ROUNDS=${ROUNDS:-2} AB_REPS=5 AB_LONE=21 \
    timeout -k 10 900 python3 tools/ab_quick.py - RT_COMPACT=1 RT_BATCH_SAMPLES=1 \
    > "gpurun_out/sweep/${scene%.xml}_aa$aa.jsonl" 2>&1 || { echo "fail $scene $aa"; tail -3 "gpurun_out/sweep/${scene%.xml}_aa$aa.jsonl"; exit 1; }
  echo "$scene aa$aa:"; grep summary "gpurun_out/sweep/${scene%.xml}_aa$aa.jsonl"
done
