#!/bin/bash
# Round-4 GPU check: GPU tests, then bench lines (C3 default, C3 one frame, mirror scenes MS / MB in
# batches and one frame at a time).   bash tools/r4_check.sh TAG [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r4}
OUT=gpurun_out/chk_$TAG
mkdir -p $OUT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${K[@]}" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.jsonl 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; return $rc; }
run c3 --no-cpu-baseline && run c3_f1 --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline \
  && run ms --config MS --steps 96 --no-cpu-baseline && run ms_f1 --config MS --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline \
  && run mb --config MB --steps 96 --no-cpu-baseline && run mb_f1 --config MB --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline
timeout -k 10 200 python3 tools/exp_scene_load.py C3_hm_1080p_d6 16,8,4,1 > $OUT/scene_load.json 2> $OUT/scene_load.err; echo "scene_load rc=$?"
