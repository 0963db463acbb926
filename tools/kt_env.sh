#!/bin/bash
# kernel-trace stats of bench under several env settings
#   bash tools/kt_env.sh "ENV=a" "ENV=b" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  OUT=gpurun_out/ktenv_$i
  mkdir -p $OUT
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1
  rc=$?
  echo "== [$cfg] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/bench.log; exit $rc; fi
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/run_kernel_stats.csv')):
    print('%-60s calls=%4s avg_us=%9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
done
