#!/bin/bash
# Bench at the driver's command per env config (REPS interleaved rounds), printing ms/frame and the batched
# one-slot kernel times:   REPS=2 bash tools/ab_oneslot.sh CFG...   (CFG "-" or K=V,K2=W)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab1
for r in $(seq 1 ${REPS:-2}); do for c in "$@"; do
  e="RT_NONE=1"; [ "$c" != "-" ] && e="${c//,/ }"
  env $e timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab1/l.jsonl 2>/dev/null || { echo "fail $c"; exit 1; }
  python3 - "$c" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab1/l.jsonl") if l.startswith("{")][-1])
k = d["kernel_ms_one_slot"]["batched"]
print(f"{sys.argv[1]:28s} {d['ms_per_step']:.4f} ms/frame | one-slot k_chain {k['k_chain']:.4f} k_mix {k['k_mix']:.4f} "
      f"k_occlude_a {k['k_occlude_a']:.4f} k_finish {k['k_finish']:.4f} | lone {d['single_frame']['ms']}")
PY
done; done
