#!/bin/bash
# rocprofv3 passes over the headline bench (run on the GPU box via gpurun).
#   bash tools/profile.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/{kt,fetch,write,sq}/ ; summaries are copied into
# profiles/ by hand afterwards.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS=${@:---steps 10 --warmup 2 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
ok() { [ "$1" -eq 0 ]; }
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
run kt --kernel-trace --stats || exit 1
run fetch --kernel-trace --pmc FETCH_SIZE || exit 1
run write --kernel-trace --pmc WRITE_SIZE || exit 1
run sq --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM || exit 1
run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
echo done
