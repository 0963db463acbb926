#!/bin/bash
# Walk-step latency: per-lane vs cooperative (librt_coop.so), then the round check.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/lat_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
RT_LIB=$P/librt_coop.so timeout -k 10 200 python3 tools/exp_walk_latency.py > $OUT/walk_latency.json 2> $OUT/walk_latency.err; echo "lat rc=$?"
EXP_REPS=61 timeout -k 10 300 python3 tools/exp_lone.py - RT_LIB=$P/librt_r3.so - RT_LIB=$P/librt_r3.so > $OUT/lone.jsonl 2> $OUT/lone.err
rc=$?; echo "lone rc=$rc"; cat $OUT/lone.jsonl; [ $rc -ne 0 ] && exit $rc
bash tools/r4_check.sh ${1:-a}
