#!/bin/bash
# parity; lone frames with the class-ranked unit order; frame batches with the measured continuation
# share sizing phase B's record space (C3 and marbles); scene creation
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/l_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
RT_KTIME=1 EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_HOT_UNITS=0 RT_LIB=$P/librt_base.so - RT_HOT_UNITS=0 > $OUT/lone.jsonl 2> $OUT/lone.err; echo "lone rc=$?"; cat $OUT/lone.jsonl
printf -- "- --config MB\nRT_LIB=$P/librt_base.so --config MB\n- \nRT_LIB=$P/librt_base.so \n- \n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cat $OUT/lines.txt
for i in 1 5; do grep '^{' gpurun_out/abl_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["config"]["workload"], d["ms_per_step"], d["fallback"])'; done
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16,1 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
RT_BUILD_TRACE=1 timeout -k 10 100 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > /dev/null 2> $OUT/build_trace.err; echo "build trace rc=$?"; grep -m3 "build:" $OUT/build_trace.err
echo done
