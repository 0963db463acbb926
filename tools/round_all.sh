#!/bin/bash
# The round's evidence in one GPU call: GPU tests, the two non-overlapping profiles (frame batches with
# one workspace slot; one frame at a time) and every config's bench line.
#   bash tools/round_all.sh TAG      then locally: summarize_profile.py TAG_b96s1 / TAG_f1, lines -> profiles/
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/round_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/round_tests.log; [ $rc -ne 0 ] && exit $rc
RT_SLOTS=1 bash tools/profile_round.sh ${TAG}_b96s1 --steps 20 --warmup 3 || exit $?
bash tools/profile_round.sh ${TAG}_f1 --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline || exit $?
bash tools/round_lines.sh $TAG
