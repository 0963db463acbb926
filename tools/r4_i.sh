#!/bin/bash
# A/B: frame batches' k_occlude walking A's shadow tasks in place (librt_inpl.so) vs packed; parity of
# the in-place build (whole GPU suite under RT_LIB)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/i_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
RT_LIB=$P/librt_inpl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests(inpl) rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
printf -- "- \nRT_LIB=$P/librt_inpl.so \nRT_LIB=$P/librt_inpl.so,RT_OCC_INPLACE=0 \n- \nRT_LIB=$P/librt_inpl.so \nRT_LIB=$P/librt_inpl.so,RT_OCC_INPLACE=0 \n" | bash tools/ab2.sh > $OUT/batched.txt 2>&1; echo "batched rc=$?"; cat $OUT/batched.txt
echo done
