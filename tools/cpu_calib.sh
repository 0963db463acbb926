#!/bin/bash
# The reference CPU renderer (oracle/_ref/ref_harness) on the GPU box's host at 1, 8 and 16 threads
# (C3, render only, median), to relate the box's cpu_baseline to this container's measurements.
cd "$GRAFT_REPO_ROOT" || exit 1
d=$(mktemp -d)
python3 -c "import __graft_entry__ as g; g.import_pkg().scenes.write_config('C3_hm_1080p_d6', '$d')" || exit 1
for t in 1 8 16; do
  timeout -k 5 120 ./oracle/_ref/ref_harness $d/C3_hm_1080p_d6.xml --aa 1 --threads $t --reps 5 | grep '"render"' || exit 1
done
grep -m1 "model name" /proc/cpuinfo
