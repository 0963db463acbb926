#!/bin/bash
# mirror_spheres batched: HEAD with a fixed record space (RT_CONT_CB: no share read-backs, no waited first
# batch), HEAD, revision 2bf126a (b2), librt_prev
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/v_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
printf -- "RT_CONT_CB=5531408 --config MS\n- --config MS\nRT_LIB=$P/librt_b2.so --config MS\nRT_LIB=$P/librt_prev.so --config MS\nRT_LIB=$P/librt_c6.so --config MS\nRT_CONT_CB=5531408 --config MS\n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; sed 's/.*librt_\([a-z0-9]*\)\.so/\1/' $OUT/lines.txt | cut -c1-120
echo done
