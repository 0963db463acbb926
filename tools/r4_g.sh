#!/bin/bash
# compact phase-A records: parity, batched / lone A/B against the previous build and a 3-wave k_finish;
# scene creation phases (early SAH); lone-frame stripe shards
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/g_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
RT_KTIME=1 EXP_REPS=61 timeout -k 10 500 python3 tools/exp_lone.py - RT_LIB=$P/librt_base.so RT_LIB=$P/librt_fw3.so RT_COMPACT=0 RT_HOT_UNITS=0 - RT_LIB=$P/librt_base.so > $OUT/lone.jsonl 2> $OUT/lone.err; echo "lone rc=$?"; cat $OUT/lone.jsonl
printf -- "- \nRT_LIB=$P/librt_base.so \nRT_LIB=$P/librt_fw3.so \nRT_OCC_INPLACE=0 \nRT_COMPACT=0 \n- \nRT_LIB=$P/librt_base.so \nRT_LIB=$P/librt_fw3.so \n" | bash tools/ab2.sh > $OUT/batched.txt 2>&1; echo "batched rc=$?"; cat $OUT/batched.txt
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16,8,1 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
RT_BUILD_TRACE=1 timeout -k 10 100 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > /dev/null 2> $OUT/stree_trace.err; echo "stree trace rc=$?"
EXP_F=1 EXP_S="1 2 4 8" timeout -k 10 500 python3 tools/exp_shard.py 1 2 4 8 > $OUT/shard_f1.jsonl 2> $OUT/shard_f1.err; echo "shard rc=$?"; cat $OUT/shard_f1.jsonl
echo done
