#!/bin/bash
# Per-batch host submission time and GPU start/end of the frame batches (RT_DEBUG=4) at the driver's
# command, under env variants: bash tools/exp_submit.sh [ENV=V[,ENV2=W]] ...   ("-": default)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sub
[ $# -eq 0 ] && set -- "-"
for v in "$@"; do
  if [ "$v" = "-" ]; then e="RT_NONE=1"; else e="${v//,/ }"; fi
  env RT_DEBUG=4 $e timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sub/line.jsonl 2> gpurun_out/sub/err.log \
    || { echo "fail $v"; tail -3 gpurun_out/sub/err.log; exit 1; }
  echo "== $v: $(python3 tools/line_summary.py gpurun_out/sub/line.jsonl | cut -c1-100)"
  awk '/warmup done/{w=1} /timed 20/{exit} w && /"submit"/' gpurun_out/sub/err.log
done
