#!/bin/bash
# L2 hit rate per kernel: TCC_HIT/TCC_MISS in frame batches (one slot), L1->L2 reads in one frame.
#   bash tools/pmc_l2.sh   (writes gpurun_out/pmcl2)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmcl2
mkdir -p $OUT
RT_SLOTS=1 timeout -k 5 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/b -o run --output-format csv -- python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
echo pass1 ok
timeout -k 5 150 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $OUT/c -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --inflight 1 --no-cpu-baseline > $OUT/c.log 2>&1 || exit $?
echo pass2 ok
python3 - <<'PY'
import csv, glob, re, collections
for d in ("b", "c"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/pmcl2/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[a-z_]+)(<[^>]*>)?", r["Kernel_Name"])
            if not m or "true" in (m.group(2) or ""): continue
            agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(agg.items()):
        s = {c: round(x / 1e6, 2) for c, x in v.items()}
        if "TCC_HIT_sum" in v:
            s["hit_rate"] = round(v["TCC_HIT_sum"] / max(1, v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 4)
        print(d, k, s)
PY
