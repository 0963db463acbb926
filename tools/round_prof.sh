#!/bin/bash
# The round's GPU tests and the two non-overlapping profiles (frame batches on one workspace slot; one
# frame at a time), one GPU call:  bash tools/round_prof.sh TAG    (round_all.sh adds every config's line)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/round_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/round_tests.log; [ $rc -ne 0 ] && exit $rc
RT_SLOTS=1 bash tools/profile_round.sh ${TAG}_b96s1 --steps 20 --warmup 3 || exit $?
bash tools/profile_round.sh ${TAG}_f1 --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline
