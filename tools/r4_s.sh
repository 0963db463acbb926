#!/bin/bash
# mirror_spheres batched regression (0.10 -> 0.25-0.40 ms/frame): the totals memset back to 12 words in
# default builds ('-'), that with the 4-wave compact k_finish (librt_w4), and librt_prev
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/s_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
printf -- "- --config MS\nRT_LIB=$P/librt_w4.so --config MS\nRT_LIB=$P/librt_prev.so --config MS\n- --config MS\nRT_LIB=$P/librt_w4.so --config MS\nRT_LIB=$P/librt_prev.so --config MS\n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cat $OUT/lines.txt
echo done
