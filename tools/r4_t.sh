#!/bin/bash
# mirror_spheres batched regression bisect: revisions c609590 (c6), 175a4bb (inb), ebc79ed (cp), 4ab88e4 (eg),
# HEAD ('-'), librt_prev
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/t_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
printf -- "RT_LIB=$P/librt_prev.so --config MS\nRT_LIB=$P/librt_c6.so --config MS\nRT_LIB=$P/librt_inb.so --config MS\nRT_LIB=$P/librt_cp.so --config MS\nRT_LIB=$P/librt_eg.so --config MS\n- --config MS\n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; cut -c1-120 $OUT/lines.txt
echo done
