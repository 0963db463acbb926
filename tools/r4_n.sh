#!/bin/bash
# a lone frame's early finish in k_mix (RT_EARLY_FIN) vs off vs the build before phase B's in-place overflow
# (librt_cont2.so); the batched traffic of the spill-free compact k_finish; scene creation; C5
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/n_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
RT_KTIME=1 EXP_REPS=61 timeout -k 10 300 python3 tools/exp_lone.py - RT_EARLY_FIN=0 RT_LIB=$P/librt_cont2.so > $OUT/lone.jsonl 2> $OUT/lone.err; echo "lone rc=$?"; cut -c1-330 $OUT/lone.jsonl
EXP_REPS=61 timeout -k 10 300 python3 tools/exp_dropin.py - RT_EARLY_FIN=0 > $OUT/dropin.jsonl 2> $OUT/dropin.err; echo "dropin rc=$?"; cat $OUT/dropin.jsonl
EXP_SCENE=marbles.xml RT_KTIME=1 EXP_REPS=31 timeout -k 10 300 python3 tools/exp_lone.py - RT_EARLY_FIN=0 > $OUT/lone_mb.jsonl 2> $OUT/lone_mb.err; echo "lone mb rc=$?"; cut -c1-330 $OUT/lone_mb.jsonl
RT_SLOTS=1 bash tools/profile_round.sh r04b_b96s1 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
timeout -k 10 300 python3 bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5.jsonl 2> $OUT/c5.err; echo "c5 rc=$?"; cut -c1-400 $OUT/c5.jsonl
echo done
