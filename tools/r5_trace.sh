#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp RT_LIB=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd/librt_trace.so
mkdir -p gpurun_out/r5tr
for cfg in "RT_TAIL=0" "RT_TAIL=64 RT_TAIL_AFTER=950" "RT_TAIL=0 RT_DCHUNK=1024" "RT_TAIL=0 RT_GB=256"; do
  echo "== $cfg"
  timeout -k 10 120 python3 tools/trace_mix.py $cfg 2>&1 | tail -60 || exit 1
done
