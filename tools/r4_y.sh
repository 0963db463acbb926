#!/bin/bash
# a lone frame's k_mix shadow role walks A's shadow tasks where k_chain left them (k_pack_a copies none):
# parity; lone-frame medians '-' vs RT_OCC_INPLACE=2 (packed, the build before) on C3 and marbles; drop-in
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/y_${1:-a}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
RT_KTIME=1 EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_OCC_INPLACE=2 - RT_OCC_INPLACE=2 > $OUT/lone.jsonl 2> $OUT/lone.err; echo "lone rc=$?"; cut -c1-330 $OUT/lone.jsonl
EXP_REPS=61 timeout -k 10 300 python3 tools/exp_dropin.py - RT_OCC_INPLACE=2 > $OUT/dropin.jsonl 2> $OUT/dropin.err; echo "dropin rc=$?"; cat $OUT/dropin.jsonl
EXP_SCENE=marbles.xml RT_KTIME=1 EXP_REPS=31 timeout -k 10 300 python3 tools/exp_lone.py - RT_OCC_INPLACE=2 > $OUT/lone_mb.jsonl 2> $OUT/lone_mb.err; echo "lone mb rc=$?"; cut -c1-330 $OUT/lone_mb.jsonl
EXP_SCENE=C2_cornellbox_800_d0 RT_KTIME=1 EXP_REPS=61 timeout -k 10 300 python3 tools/exp_lone.py - RT_OCC_INPLACE=2 > $OUT/lone_c2.jsonl 2> $OUT/lone_c2.err; echo "lone c2 rc=$?"; cut -c1-330 $OUT/lone_c2.jsonl
echo done
