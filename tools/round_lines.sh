#!/bin/bash
# Bench lines of every config at HEAD (C3 default, at the driver's --steps 20 --warmup 5, at AA2, one frame at a time, C2, C5, the mirror-heavy MS / MB
# in batches and one at a time) and the C2 / C5
# rocprof kernel stats, for profiles/:   bash tools/round_lines.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/lines_$TAG
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.jsonl 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; return $rc; }
run c3 && run c3_20 --steps 20 --warmup 5 && run c3_aa2 --aa 2 --steps 20 --warmup 5 --no-cpu-baseline && run c3_f1 --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline && run c2 --config C2 --steps 192 --no-cpu-baseline \
  && run c5 --config C5 --steps 3 --warmup 1 --no-cpu-baseline \
  && run ms --config MS --steps 96 --no-cpu-baseline && run ms_f1 --config MS --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline \
  && run mb --config MB --steps 96 --no-cpu-baseline && run mb_f1 --config MB --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c5 -o run --output-format csv -- python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/kt_c5.log 2>&1 && echo "kt_c5 rc=0" \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c3aa2 -o run --output-format csv -- python3 bench.py --aa 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/kt_c3aa2.log 2>&1 && echo "kt_c3aa2 rc=0" \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c2 -o run --output-format csv -- python3 bench.py --config C2 --steps 64 --no-cpu-baseline > $OUT/kt_c2.log 2>&1 && echo "kt_c2 rc=0"
