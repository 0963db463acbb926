#!/bin/bash
# Build the working tree's librt_hip.so into raytracer-ceng477-graphics-hw-1_amd/librt_<name>.so without
# touching the in-tree build (same-box A/B runs with RT_LIB=...):   bash tools/build_wt.sh NAME [make args]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
WT=/tmp/rt_wt_$NAME
rm -rf "$WT"; mkdir -p "$WT"
cp -r "$ROOT/include" "$WT/"
mkdir -p "$WT/raytracer-ceng477-graphics-hw-1_amd"
cp -r "$ROOT/raytracer-ceng477-graphics-hw-1_amd/csrc" "$ROOT/raytracer-ceng477-graphics-hw-1_amd/Makefile" "$WT/raytracer-ceng477-graphics-hw-1_amd/"
make -C "$WT/raytracer-ceng477-graphics-hw-1_amd" -j8 librt_hip.so "$@" > /dev/null
cp "$WT/raytracer-ceng477-graphics-hw-1_amd/librt_hip.so" "$ROOT/raytracer-ceng477-graphics-hw-1_amd/librt_$NAME.so"
echo "built working tree -> librt_$NAME.so"
