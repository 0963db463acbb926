#!/bin/bash
# Frame-batch concurrency: per-rank shard time at N=1,2,4,8 for (frames in flight, slots) settings.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for cfg in "$@"; do
  echo "[$cfg]"
  env $cfg timeout -k 10 200 python3 tools/exp_shard.py 1 2 4 8 2>/dev/null | grep "^{" | cut -c1-52 || exit 1
done
