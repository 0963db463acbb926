#!/bin/bash
# parity of the round-4 build; batched lines with one-slot kernel times (compact records, in-place tasks,
# the early-round build); lone frames (hot units); scene creation
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/k_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
printf -- "- \nRT_COMPACT=0 \nRT_OCC_INPLACE=0 \nRT_LIB=$P/librt_base.so \n- \nRT_COMPACT=0 \n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cat $OUT/lines.txt
RT_KTIME=1 EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_HOT_UNITS=0 RT_LIB=$P/librt_base.so - RT_HOT_UNITS=0 > $OUT/lone.jsonl 2> $OUT/lone.err; echo "lone rc=$?"; cat $OUT/lone.jsonl
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16,1 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
RT_BUILD_TRACE=1 timeout -k 10 100 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > /dev/null 2> $OUT/build_trace.err; echo "build trace rc=$?"; grep -m3 "build:" $OUT/build_trace.err
echo done
