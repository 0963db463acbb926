#!/bin/bash
# a frame batch no longer re-polls the continuation share at launch (a larger share split it into chunks
# forked over every slot): mirror_spheres / C3 / MB batched lines against librt_prev, growth log
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/u_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
RT_LOG_ALLOC=1 timeout -k 10 200 python3 bench.py --config MS --steps 96 --no-cpu-baseline > $OUT/ms_log.jsonl 2> $OUT/ms_log.err; echo "ms_log rc=$?"; grep -E "librt_hip|timed|warmup" $OUT/ms_log.err | head -30; cut -c1-200 $OUT/ms_log.jsonl
printf -- "- --config MS\nRT_LIB=$P/librt_prev.so --config MS\n- --config MS\n- \nRT_LIB=$P/librt_prev.so \n- \n- --config MB\nRT_LIB=$P/librt_prev.so --config MB\n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; sed 's/.*librt_\([a-z0-9]*\)\.so/\1/' $OUT/lines.txt | cut -c1-200
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
echo done
