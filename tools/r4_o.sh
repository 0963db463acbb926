#!/bin/bash
# a lone frame's early finish in k_mix with striped pixel counters (RT_EARLY_FIN) vs off; phase B's overflow
# walked in place vs packed (RT_OCC_INPLACE=0) on marbles; the build before both (librt_cont2.so)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/o_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
RT_KTIME=1 EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_EARLY_FIN=0 RT_LIB=$P/librt_cont2.so - RT_EARLY_FIN=0 > $OUT/lone.jsonl 2> $OUT/lone.err; echo "lone rc=$?"; cut -c1-330 $OUT/lone.jsonl
EXP_REPS=61 timeout -k 10 300 python3 tools/exp_dropin.py - RT_EARLY_FIN=0 > $OUT/dropin.jsonl 2> $OUT/dropin.err; echo "dropin rc=$?"; cat $OUT/dropin.jsonl
EXP_SCENE=marbles.xml RT_KTIME=1 EXP_REPS=31 timeout -k 10 400 python3 tools/exp_lone.py - RT_EARLY_FIN=0 RT_EARLY_FIN=0,RT_OCC_INPLACE=0 RT_LIB=$P/librt_cont2.so > $OUT/lone_mb.jsonl 2> $OUT/lone_mb.err; echo "lone mb rc=$?"; cut -c1-330 $OUT/lone_mb.jsonl
echo done
