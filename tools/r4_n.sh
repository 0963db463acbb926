#!/bin/bash
# compact-record k_finish at 3 waves (no spills) vs 4 (spilled): parity, batched lines, batched traffic;
# scene creation with the early upload
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/n_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
printf -- "- \nRT_LIB=$P/librt_prev.so \n- \nRT_LIB=$P/librt_prev.so \n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cat $OUT/lines.txt
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
RT_SLOTS=1 bash tools/profile_round.sh r04b_b96s1 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
echo done
