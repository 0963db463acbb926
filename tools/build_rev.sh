#!/bin/bash
# Build librt_hip.so of a git revision into raytracer-ceng477-graphics-hw-1_amd/librt_<name>.so
# (for same-box A/B runs with RT_LIB=...):   bash tools/build_rev.sh REV NAME [make args]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2; shift 2
WT=/tmp/rt_rev_$NAME
rm -rf "$WT"; mkdir -p "$WT"
git -C "$ROOT" archive "$REV" | tar -x -C "$WT"
make -C "$WT/raytracer-ceng477-graphics-hw-1_amd" -j8 librt_hip.so "$@" > /dev/null
cp "$WT/raytracer-ceng477-graphics-hw-1_amd/librt_hip.so" "$ROOT/raytracer-ceng477-graphics-hw-1_amd/librt_$NAME.so"
echo "built $REV -> librt_$NAME.so"
