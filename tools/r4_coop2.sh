#!/bin/bash
# Coop A/B against builds without it (librt_nocoop.so: RT_COOP_BUILD=0; librt_r3.so: round 3), traces.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/coop2_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_COOP=0 RT_LIB=$P/librt_nocoop.so RT_LIB=$P/librt_r3.so - RT_COOP=0 > $OUT/lone.jsonl 2> $OUT/lone.err
rc=$?; echo "lone rc=$rc"; cat $OUT/lone.jsonl; [ $rc -ne 0 ] && exit $rc
EXP_REPS=21 RT_KTIME=1 timeout -k 10 300 python3 tools/exp_lone.py - RT_COOP=0 > $OUT/lone_kt.jsonl 2> $OUT/lone_kt.err
rc=$?; echo "lone_kt rc=$rc"; cat $OUT/lone_kt.jsonl; [ $rc -ne 0 ] && exit $rc
RT_COOP=1 timeout -k 10 200 python3 tools/trace_report.py chain > $OUT/trace_coop.json 2> $OUT/trace_coop.err; echo "trace rc=$?"
RT_COOP=0 timeout -k 10 200 python3 tools/trace_report.py chain > $OUT/trace_nocoop.json 2> $OUT/trace_nocoop.err; echo "trace0 rc=$?"
bash tools/r4_check.sh ${1:-a}
