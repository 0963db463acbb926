#!/bin/bash
# The round's evidence (bash tools/round6.sh TAG [PART]; PART 1: steps 1-2, 2: step 3, default both), each
# step under its own time limit:
#  1. the GPU suite;
#  2. one-slot profiles of C3 (rocprofv3 --kernel-trace --stats, then FETCH_SIZE and WRITE_SIZE passes, each
#     its own run) of bench.py --trace --one-slot: 96-frame calls (the configuration of the line's
#     kernel_ms_one_slot.batched), AA1 and AA2, and one frame at a time (--inflight 1);
#  3. every config's bench line (C3 at the driver's command and at 192 steps, AA2, one frame, C2, C5, MS, MB).
# Then locally: python tools/summarize_profile.py TAG_<name> gpurun_out/prof_TAG_<name> for b96, aa2, f1.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r06}
OUT=gpurun_out/r6_$TAG
mkdir -p "$OUT"
PART=${2:-all}
if [ "$PART" != 2 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
prof() {   # prof NAME bench-args...
  local name=$1; shift
  local d=gpurun_out/prof_${TAG}_$name
  mkdir -p "$d"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d/kt" -o run --output-format csv -- python3 bench.py "$@" --trace > "$d/kt.log" 2>&1 \
    && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$d/fetch" -o run --output-format csv -- python3 bench.py "$@" --trace > "$d/fetch.log" 2>&1 \
    && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$d/write" -o run --output-format csv -- python3 bench.py "$@" --trace > "$d/write.log" 2>&1 \
    && timeout -k 10 300 python3 bench.py "$@" --trace > "$d/trace.jsonl" 2> "$d/trace.err"
  local rc=$?; echo "prof $name rc=$rc"; return $rc
}
prof b96 --steps 96 --warmup 5 --one-slot && prof aa2 --aa 2 --steps 96 --warmup 5 --one-slot \
  && prof f1 --inflight 1 --steps 32 --warmup 3 || exit 1
fi
[ "$PART" = 1 ] && exit 0
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; local rc=$?; echo "line $name rc=$rc"; return $rc; }
run c3_20 --steps 20 --warmup 5 && run c3 --no-cpu-baseline && run c3_aa2 --aa 2 --steps 20 --warmup 5 --no-cpu-baseline \
  && run c3_f1 --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline && run c2 --config C2 --steps 192 --no-cpu-baseline \
  && run c5 --config C5 --steps 3 --warmup 1 --no-cpu-baseline \
  && run ms --config MS --steps 96 --no-cpu-baseline && run mb --config MB --steps 96 --no-cpu-baseline
