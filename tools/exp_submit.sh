#!/bin/bash
# Host submission time per frame batch at the driver's command (RT_LOG_SUBMIT=1), under env variants.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sub
for v in "-" "HIP_FORCE_DEV_KERNARG=0" "RT_HW_QUEUES=16" "-"; do
  if [ "$v" = "-" ]; then e="RT_NONE=1"; else e="$v"; fi
  env RT_LOG_SUBMIT=1 $e timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sub/line.jsonl 2> gpurun_out/sub/err.log \
    || { echo "fail $v"; tail -3 gpurun_out/sub/err.log; exit 1; }
  echo "== $v: $(python3 tools/line_summary.py gpurun_out/sub/line.jsonl | cut -c1-120)"
  grep '"submit"' gpurun_out/sub/err.log | tail -8
done
