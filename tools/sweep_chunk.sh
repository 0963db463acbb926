cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/sweep_both.sh RT_CHUNK_SAMPLES=16777216 RT_CHUNK_SAMPLES=33554432 || exit 1
for c in 8388608 16777216 33554432; do
  RT_CHUNK_SAMPLES=$c timeout -k 10 300 python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/c5_$c.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('C5 chunk $c', d['ms_per_step'], d['value'])"
done
