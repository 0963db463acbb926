#!/bin/bash
# cb fill (marbles), coop step latency, k_finish grid A/B, parity, bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/d_${1:-a}
mkdir -p $OUT
P=$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
EXP_REPS=61 timeout -k 10 400 python3 tools/exp_lone.py - RT_ABANDON=0 RT_ABANDON=950 RT_ABANDON=990 RT_ABANDON=900 - RT_ABANDON=0 > $OUT/lone_ab.jsonl 2> $OUT/lone_ab.err; echo "lone_ab rc=$?"; cat $OUT/lone_ab.jsonl
timeout -k 10 200 python3 tools/trace_report.py chain > $OUT/trace.json 2> $OUT/trace.err; echo "trace rc=$?"
RT_LIB=$P/librt_coop.so timeout -k 10 200 python3 tools/exp_walk_latency.py > $OUT/walk_latency.json 2> $OUT/walk_latency.err; echo "lat rc=$?"
EXP_SCENE=marbles.xml EXP_REPS=31 timeout -k 10 300 python3 tools/exp_lone.py - > $OUT/lone_mb.jsonl 2> $OUT/lone_mb.err; echo "lone_mb rc=$?"; cat $OUT/lone_mb.jsonl
printf -- "- \nRT_FGRID=1024 \n- \nRT_FGRID=1024 \n- \nRT_FGRID=1024 \n" | bash tools/ab2.sh > $OUT/fgrid.txt 2>&1; echo "fgrid rc=$?"; cat $OUT/fgrid.txt
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.jsonl 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; return $rc; }
run mb --config MB --steps 96 --no-cpu-baseline && run mb_f1 --config MB --inflight 1 --steps 32 --warmup 3 --no-cpu-baseline && run c3 --no-cpu-baseline
