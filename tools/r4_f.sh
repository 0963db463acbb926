#!/bin/bash
# scene creation phases after the build changes; lone-frame stripe shards (item 5)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/f_${1:-a}
mkdir -p $OUT
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16,8,1 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
RT_BUILD_TRACE=1 timeout -k 10 100 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > /dev/null 2> $OUT/stree_trace.err; echo "stree trace rc=$?"
EXP_F=1 EXP_S="1 2 4 8" timeout -k 10 500 python3 tools/exp_shard.py 1 2 4 8 > $OUT/shard_f1.jsonl 2> $OUT/shard_f1.err; echo "shard rc=$?"; cat $OUT/shard_f1.jsonl
