#!/bin/bash
# mirror_spheres in frame batches: 0.102 (r04a) -> 0.177 ms/frame (r04c); workspace growth log, the builds
# before the measured continuation share (librt_base) and the 3-wave compact k_finish (librt_prev); C3 A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/q_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
RT_LOG_ALLOC=1 timeout -k 10 200 python3 bench.py --config MS --steps 96 --no-cpu-baseline > $OUT/ms_log.jsonl 2> $OUT/ms_log.err; echo "ms_log rc=$?"; grep -E "librt_hip|timed|warmup" $OUT/ms_log.err | head -40
printf -- "- --config MS\nRT_LIB=$P/librt_base.so --config MS\nRT_LIB=$P/librt_prev.so --config MS\n- --config MS\n- \nRT_LIB=$P/librt_prev.so \n- \nRT_LIB=$P/librt_prev.so \n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cat $OUT/lines.txt
echo done
