#!/bin/bash
# every slot stream created up front: mirror_spheres / C3 / MB batched lines against librt_prev; tests
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/w_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
printf -- "- --config MS\nRT_LIB=$P/librt_prev.so --config MS\n- --config MS\n- \nRT_LIB=$P/librt_prev.so \n- --config MB\n" | bash tools/ab_lines.sh > $OUT/lines.txt 2>&1; echo "lines rc=$?"; sed 's/.*librt_\([a-z0-9]*\)\.so/\1/' $OUT/lines.txt | cut -c1-120
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
echo done
