#!/bin/bash
# Round profile of the headline bench on the GPU box (via gpurun):
#   bash tools/profile_round.sh TAG [bench args]
# 1) rocprofv3 --kernel-trace --stats   (per-kernel durations; bench --trace: counting passes, warmup and
#    timed frames only, so the per-frame kernel sums can be checked against the line's kernel_ms)
# 2) rocprofv3 --pmc FETCH_SIZE, 3) --pmc WRITE_SIZE   (separate passes; HBM bytes)
# 4) bench.py --trace (the JSON line of the traced configuration), 5) plain bench.py (with the CPU baseline)
# Frame batches overlap on the workspace slots; pass RT_SLOTS=1 in the environment for per-kernel
# durations that do not overlap.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS=${@:---steps 20 --warmup 3}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS --trace \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run kt --kernel-trace --stats && run fetch --kernel-trace --pmc FETCH_SIZE && run write --kernel-trace --pmc WRITE_SIZE \
  && timeout -k 10 300 python3 bench.py $ARGS --trace > "$OUT/trace.jsonl" 2> "$OUT/trace.err" && echo "trace rc=0" \
  && timeout -k 10 300 python3 bench.py $ARGS > "$OUT/bench.jsonl" 2> "$OUT/bench.err" && echo "bench rc=0"
# afterwards, locally: python tools/summarize_profile.py TAG gpurun_out/prof_TAG
