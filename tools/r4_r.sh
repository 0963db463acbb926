#!/bin/bash
# the rest of a scene's first batched call on the next slots in batches of the same size (no workspace
# growth inside later calls), +1/16 workspace headroom: parity, MS / MB / C3 batched lines, growth log
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
RT_LOG_ALLOC=1 timeout -k 10 200 python3 bench.py --config MS --steps 96 --no-cpu-baseline > $OUT/ms_log.jsonl 2> $OUT/ms_log.err; echo "ms_log rc=$?"; grep -E "librt_hip|timed|warmup" $OUT/ms_log.err | head -40
printf -- "- --config MS\nRT_LIB=$P/librt_base.so --config MS\n- --config MS\n- --config MB\n- \nRT_LIB=$P/librt_prev.so \n- \n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cat $OUT/lines.txt
echo done
