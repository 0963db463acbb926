#!/bin/bash
# Cooperative tail walks: parity subset, lone-frame A/B, then the round check (all GPU tests, bench lines).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/coop_${1:-a}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "test_render_bit_exact and chain" > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity.log; [ $rc -ne 0 ] && exit $rc
EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_COOP=0 RT_COOP_LIVE=4 RT_COOP_TAIL=64 RT_COOP=0,RT_BTAIL=1 > $OUT/lone.jsonl 2> $OUT/lone.err
rc=$?; echo "lone rc=$rc"; cat $OUT/lone.jsonl; [ $rc -ne 0 ] && exit $rc
EXP_SCENE=mirror_spheres.xml EXP_REPS=61 timeout -k 10 300 python3 tools/exp_lone.py - RT_COOP=0 > $OUT/lone_ms.jsonl 2> $OUT/lone_ms.err
rc=$?; echo "lone_ms rc=$rc"; cat $OUT/lone_ms.jsonl; [ $rc -ne 0 ] && exit $rc
bash tools/r4_check.sh ${1:-a}
