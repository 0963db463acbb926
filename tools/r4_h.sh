#!/bin/bash
# k_fallback on the lone-frame critical path: C3 with the phase-B record space below the
# continuation count, the wide trees off, and an axis-aligned odd-resolution camera (eye rays with a
# direction component of exactly 0); mirror-heavy scenes one frame at a time.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/h_${1:-a}
mkdir -p $OUT
RT_KTIME=1 EXP_REPS=31 timeout -k 10 400 python3 tools/exp_lone.py - RT_CONT_CB=150000 RT_CONT_CB=100000 RT_WIDE_WALK=0 - > $OUT/lone_fb.jsonl 2> $OUT/lone_fb.err; echo "lone_fb rc=$?"; cat $OUT/lone_fb.jsonl
EXP_SCENE=X_cornell_801_axis RT_KTIME=1 EXP_REPS=31 timeout -k 10 200 python3 tools/exp_lone.py - RT_WIDE_WALK=0 > $OUT/lone_axis.jsonl 2> $OUT/lone_axis.err; echo "lone_axis rc=$?"; cat $OUT/lone_axis.jsonl
for sc in mirror_spheres.xml marbles.xml; do
  EXP_SCENE=$sc RT_KTIME=1 EXP_REPS=31 timeout -k 10 200 python3 tools/exp_lone.py - > $OUT/lone_$sc.jsonl 2> $OUT/lone_$sc.err; echo "lone $sc rc=$?"; cat $OUT/lone_$sc.jsonl
done
echo done
