#!/bin/bash
# kernel-trace stats of one bench configuration: bash tools/kt.sh TAG [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/kt_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rc=$rc"
grep '^{' $OUT/bench.log | cut -c1-300
cat $OUT/run_kernel_stats.csv | cut -c1-220
exit $rc
