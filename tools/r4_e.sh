#!/bin/bash
# scene creation phases, drop-in CLI end-to-end vs the reference executable
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/e_${1:-a}
mkdir -p $OUT
make -C oracle ref_stock > /dev/null 2>&1 || true
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16,12,8,1 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
RT_BUILD_TRACE=1 timeout -k 10 100 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16 > /dev/null 2> $OUT/stree_trace.err; echo "stree trace rc=$?"
timeout -k 10 600 python3 tools/exp_cli.py --reps 3 > $OUT/cli.jsonl 2> $OUT/cli.err; echo "cli rc=$?"; cat $OUT/cli.jsonl | cut -c1-400
