#!/usr/bin/env python3
"""Headline benchmark: Mray/s (primary+shadow) and ms/frame, horse_and_mug
1920x1080, MaxRecursionDepth 6 (BASELINE.json configs[2] = SURVEY.md §8d C3),
on N GPUs of one node.

One "step" = one frame: every rank renders its round-robin row stripes of the
frame into an HBM slab, then for N>1 the slabs are gathered to rank 0 with one
RCCL collective over xGMI and un-interleaved by a rank-0 kernel.
Frames are submitted --inflight at a time (default 96) as frame batches
(rt_render_frames_device: one persistent grid walks several frames' samples, so
one frame's serial mirror-chain tail runs beside the others' bulk; one gather
per batch).  Every frame's full work is done and counted.  `value` is that
serving throughput with the scene resident in HBM and frames left in HBM (no
D2H, no write_ppm).  Beside it, first-class: `single_frame` (one frame alone on
the GPU, device time) and `drop_in` -- SURVEY.md §8(d)'s ms/frame, rt_render's
wall time from camera upload to the uint8 frame in host memory (PCIe
included), the drop-in caller's case.  Scaling is strong (the frame is fixed,
split over N).

Roofline: the walks fetch a small, cache-resident scene, so
the memory roofline that bounds them is the L2's (MI355X_MICROARCH.md §L2,
~34.5 TB/s aggregate), not HBM's.  `achieved` = the bytes the TIMED kernels
fetch and move per frame -- traversal bytes counted by a production-fetch
counting pass (RT_DEBUG 0x20: the same walks as the timed kernels, counting
their node, leaf-record and primitive loads) plus the workspace bytes of the
chain path (records, task ids, occlusion bytes, output; a per-ray model of
pathchain.hip) -- divided by the frame's kernel time.  The HBM bytes actually
moved (rocprofv3 FETCH_SIZE / WRITE_SIZE, profiles/) are reported beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--aa F] [--config C3]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent

# Hardware queues per process (read by the HIP runtime at its first use, so set before torch touches
# the GPU): each workspace slot renders on its own stream beside the caller's, and HIP multiplexes
# streams beyond GPU_MAX_HW_QUEUES (4 by default) onto the same queues, which serialises the slots.
# With 8 queues the library runs 6 frame batches in flight (rt_api.cpp tune_slots); RT_HW_QUEUES
# overrides (the box refuses more than 32).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_HW_QUEUES", "8")
sys.path.insert(0, str(ROOT))

import __graft_entry__ as graft  # noqa: E402

HBM_SPEC_GBPS = 8000.0     # MI355X spec (MI355X_MICROARCH.md §HBM); the line prices against MEASURED peaks
                           # (rt_measure_peaks: HBM streaming copy, walk-shaped L2 gather) and shows the spec
# The reference's algorithmic bytes per unit of work, reported for comparison
B_NODE, B_TRI, B_SPH, B_PIX = 32, 36, 16, 3


def kernel_bytes(r: dict, c: dict, out_pixels: int, batched: bool, nlights: int, compact: bool = False) -> dict:
    """Algorithmic bytes of one frame per kernel of the chain path (pathchain.hip), from a
    production-fetch counting pass: `r` = its per-role counter slots (Scene.counters_raw: the bytes
    each role's walks fetch -- wide-node lines, leaf records, primitives -- and its ray / hit counts),
    `c` = the reference's counters.  Workspace traffic per item: a hit writes its record -- 32 B (hit
    point, surface code, direction and material), or 16 B in phase A with compact records (RT_COMPACT,
    pathchain.hpp dbase) -- and reads its 16-B face normal (TriShade); a traced shadow task id
    is written (4 B), read by its walker with the record's first 16 B and the normal, and its 1-B
    result written; a skipped one (light_needed) writes its 1-B result; a continuation id and its
    direction word (16 B, tail) are written in phase A and read in phase B with its record and normal;
    packing reads and writes each task id (in frame batches only the continuations'); k_finish reads every sample's path word (4 B) and every
    hit's record, normal and occlusion dword(s) (4 B when the record's bytes sit in one dword: 1, 2 or
    4 lights; else 8), and writes 3 B per pixel.
    One frame alone, A's shadow rays run in k_mix's shadow role; in frame batches in k_occlude.  Phase-A
    records are 32 B, or 16 B where `compact` (the launches' own report: counter slot compact_launches;
    rt_api.cpp full_records_fit decides by the frames a launch fits)."""
    NRM, TASK, OCC = 16, 4, 1
    REC_B = 32
    REC_A = 16 if compact else 32
    DIRW = 16 if REC_A == 16 else 0
    samples, skipped = c["primary_rays"], c["shadow_rays_skipped"]
    a_sh, bq, bo, conts = r["a_shadow_rays"], r["bq_shadow_rays"], r["bo_shadow_rays"], r["continuations"]
    shadow_ws = TASK + 16 + NRM + OCC
    k = {
        "k_chain": r["a_walk_bytes"] + samples * 4 + r["a_hits"] * (REC_A + NRM) + a_sh * TASK + skipped * OCC
                   + conts * (TASK + DIRW),
        # frame batches: the continuations packed (A's shadow tasks are walked in their regions); a lone frame
        # has no packing pass (round 6): its k_mix reads both lists in their regions and stores each
        # continuation's index (cid) at its grab
        "k_pack_a": conts * 2 * TASK if batched else 0,
        "k_mix": r["b_walk_bytes"] + r["bq_shadow_bytes"] + conts * ((1 if batched else 2) * TASK + 16 + DIRW + (REC_A - 16) + NRM)
                 + r["b_hits"] * (REC_B + NRM) + bq * (16 + NRM + OCC) + bo * TASK,
        "k_occlude_a": r["a_shadow_bytes"] + a_sh * shadow_ws,
        "k_pack_b": bo * 2 * TASK,
        "k_occlude_b": r["bo_shadow_bytes"] + bo * shadow_ws,
        "k_finish": samples * 4 + r["a_hits"] * (REC_A + NRM) + r["b_hits"] * (REC_B + NRM)
                    + (r["a_hits"] + r["b_hits"]) * (4 if nlights in (1, 2, 4) else 8) + out_pixels * 3,
    }
    if not batched:                       # one frame: A's shadow rays are k_mix's shadow role
        k["k_mix"] += k.pop("k_occlude_a")
    return k


def traversal_bytes(r: dict) -> int:
    return r["a_walk_bytes"] + r["b_walk_bytes"] + r["a_shadow_bytes"] + r["bq_shadow_bytes"] + r["bo_shadow_bytes"]


# kernels one frame launches, per render path (the roofline covers all of them)
PATH_KERNELS = {
    "chain": ["k_chain", "k_pack_a", "k_mix", "k_pack_b", "k_occlude", "k_fallback", "k_finish", "k_finish_any"],
}

CONFIGS = {
    "C3": ("C3_hm_1080p_d6", "horse_and_mug.xml 1920x1080, MaxRecursionDepth 6, full BVH + mirror recursion"),
    "C2": ("C2_cornellbox_800_d0", "cornellbox.xml camera 2 800x800, primary+shadow only (depth 0)"),
    "C5": ("C5_hm_8k_d6", "horse_and_mug.xml 7680x4320, depth 6, 16x SSAA (factor 4)"),
    # mirror-heavy reference scenes, verbatim (inputs/, 1024x1024, MaxRecursionDepth 6): deep mirror chains
    # between spheres, where phase B's record space (cb) and k_fallback matter
    "MS": ("mirror_spheres.xml", "mirror_spheres.xml verbatim 1024x1024, depth 6 (all-mirror spheres)"),
    "MB": ("marbles.xml", "marbles.xml verbatim 1024x1024, depth 6 (mirror marbles, 2 lights)"),
}
HBM_GUIDE_GBPS = 6290.0    # MI355X_MICROARCH.md: measured float4 copy (79 % of spec), beside our own measurement
L2_GUIDE_GBPS = 34500.0    # MI355X_MICROARCH.md:316: aggregate L2 streaming bandwidth, beside the measured line gather


def golden_sha(config: str, aa: int) -> str | None:
    """sha256 of the reference's RGB for this workload (tests/golden/goldens.json, made by running the
    compiled reference: tests/golden/make_goldens.py), or None when no golden covers it."""
    gfile = ROOT / "tests" / "golden" / "goldens.json"
    if not gfile.exists():
        return None
    name = config[:-4] if config.endswith(".xml") else config       # (MS / MB: the reference scene files)
    for g in json.loads(gfile.read_text())["goldens"]:
        if g["name"] == f"{name}_aa{aa}" and len(g["cameras"]) >= 1:
            return g["cameras"][0].get("sha256_rgb")
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=192)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--aa", type=int, default=None, help="SSAA factor (default 1; C5: 4)")
    ap.add_argument("--stripe-rows", type=int, default=4,
                    help="output rows per round-robin stripe (4: best rank balance at N=8, tools/exp_shard.py)")
    ap.add_argument("--path", default="chain", choices=sorted(PATH_KERNELS), help="render path (the chain path)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--trace", action="store_true",
                    help="profiling runs (tools/profile_round.sh): only the counting passes, warmup and timed frames "
                         "run, so per-frame kernel sums from rocprofv3 can be checked against kernel_ms")
    ap.add_argument("--one-slot", action="store_true",
                    help="profiling runs: ONE workspace slot with the share of the budget one of the default slots gets "
                         "(the configuration of the line's kernel_ms_one_slot), so rocprofv3's per-kernel times of "
                         "this run check the line's per-kernel ones")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames submitted together (rt_render_frames_device frame batches; 1 = one frame at a "
                         "time; default 96, C5 1: its frames are already 250x larger than one launch's chunk)")
    return ap.parse_args()


def host_cores() -> dict:
    """CPUs this process may use: the affinity set, bounded by a cgroup CPU quota if one is set (the GPU
    boxes give a job a share of a large host: nproc shows the whole machine there)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "usable": min(aff, quota or aff)}


def cpu_baseline(xml: str, aa: int, rays_ps_per_frame: int, budget_s: float) -> dict:
    """Reference CPU renderer timed on this host (rank 0 only), with every usable host core as one thread
    each -- the reference's own default is std::thread::hardware_concurrency() (raytracer.cpp:367).
    Prefers the unmodified reference compiled from its sources (oracle/_ref/ref_harness, kind
    "reference"); falls back to the C restatement (kind "port")."""
    hc = host_cores()
    threads = max(1, min(256, hc["usable"]))
    host = {}        # the reference's own XML load and BVH build times (parser.cpp, bvh.h), for the host rows
    harness = ROOT / "oracle" / "_ref" / "ref_harness"
    if harness.exists():
        def run(reps):
            out = subprocess.run([str(harness), xml, "--aa", str(aa), "--threads", str(threads), "--reps", str(reps)],
                                 check=True, capture_output=True, text=True, cwd=tempfile.gettempdir()).stdout
            evs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
            for e in evs:
                if e.get("event") in ("load", "bvh"):
                    host[f"ref_{e['event']}_ms"] = round(e["seconds"] * 1e3, 3)
            return [e for e in evs if e.get("event") == "render"][0]["median_s"]
        first = run(1)
        reps = int(max(1, min(50, budget_s / max(first, 1e-3))))
        med = run(reps) if reps > 1 else first
        kind = "reference"
    else:
        orc = graft.import_oracle()
        sc = orc.OracleScene(xml)
        t0 = time.perf_counter()
        sc.render(0, aa=aa, threads=threads)
        first = time.perf_counter() - t0
        reps = int(max(1, min(50, budget_s / max(first, 1e-3))))
        ts = [first]
        for _ in range(reps - 1):
            t0 = time.perf_counter()
            sc.render(0, aa=aa, threads=threads)
            ts.append(time.perf_counter() - t0)
        med = sorted(ts)[len(ts) // 2]
        kind = "port"
    return {"value": round(rays_ps_per_frame / med / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": kind,
            "ms_per_frame": round(med * 1e3, 3), **host, "host_cpus": hc,
            "sample": f"{reps} full frames of the same workload (median), render only, {threads} threads "
                      f"(all usable cores; nproc {hc['nproc']})"}


def main() -> int:
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print(f"--gpus {a.gpus} needs torchrun --nproc-per-node {a.gpus}", file=sys.stderr)
            return 2
    # RT_BENCH_BACKEND=gloo: host-staged gather with every rank on GPU local % device_count, to
    # rehearse the N>1 path on a one-GPU box (never for a reported number; RCCL is the product path)
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def all_reduce(t, op=None):
        if world == 1:
            return t
        kw = {} if op is None else {"op": op}
        if backend == "gloo":
            h = t.cpu()
            dist.all_reduce(h, **kw)
            return h.to(t.device)
        dist.all_reduce(t, **kw)
        return t

    pkg = graft.import_pkg()
    config, desc = CONFIGS[a.config]
    aa = a.aa if a.aa is not None else (4 if a.config == "C5" else 1)
    tmpdir = tempfile.mkdtemp(prefix=f"rtbench{rank}_")
    xml = pkg.scenes.write_config(config, tmpdir)

    def one_slot_env():
        """RT_SLOTS=1 and the RT_WS_BUDGET_MB that gives that slot the share one of the default slots gets: the
        scene and the 64 MB staging reserve off the budget, the rest over the slots (rt_api.cpp slot_budget)."""
        nslots = int(os.environ.get("RT_SLOTS", max(1, min(6, int(os.environ["GPU_MAX_HW_QUEUES"]) - 1))))
        budget_mb = int(os.environ.get("RT_WS_BUDGET_MB", "16384"))
        probe = pkg.Scene.from_xml(xml, device=local, render_path=a.path)
        fixed_mb = (probe.memory()["scene_bytes"] >> 20) + 1 + 64
        probe.close()
        return {"RT_SLOTS": "1", "RT_WS_BUDGET_MB": str(max(64, (budget_mb - fixed_mb) // nslots + fixed_mb))}

    if a.one_slot:
        os.environ.update(one_slot_env())
    t0 = time.perf_counter()
    scene = pkg.Scene.from_xml(xml, device=local, render_path=a.path)
    load_s = time.perf_counter() - t0
    binfo = scene.bvh_info()
    cam = scene.camera(0)
    W, H, S = cam.image_width, cam.image_height, a.stripe_rows
    rows = pkg.slab_rows(H, S, world)
    F = max(1, a.inflight if a.inflight is not None else (1 if a.config == "C5" else 96))
    NB = 2 if world > 1 else 1     # N>1: batch b+1 renders while batch b's slabs are gathered (double buffer)
    slab_bufs = [torch.empty((F, rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(NB)]
    slab = slab_bufs[0][0]
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    gbufs = {}
    freed = [None] * NB            # event: the buffer's previous gather has completed
    nxt = [0]
    if world > 1:
        comm = torch.cuda.Stream(dev)     # gather + rank-0 unshuffle, off the render stream
        images = [torch.empty((H, W, 3), dtype=torch.uint8, device=dev) for _ in range(F)] if rank == 0 else None

        def unshuffle_dev(g, img):    # rank-0 kernel: slabs -> row order (rt_unshuffle_stripes), comm stream
            pkg.unshuffle_stripes(g.data_ptr(), img.data_ptr(), W, H, S, world, comm.cuda_stream)

    def note(msg):      # progress on stderr (long configs such as C5)
        print(f"[bench rank {rank}] {msg} t={time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)

    note(f"scene loaded {W}x{H} aa{aa}")
    # measured roofline denominators on this device (rt_measure_peaks, ~1 s): HBM streaming copy and
    # the walks' access shape (random whole 128-B lines shared by every workgroup) from a table inside
    # one XCD's L2 and from a table the size of the scene's walk hot set
    hot_bytes = {k: binfo[k] for k in ("ref_wide_bytes", "occ_wide_bytes", "leaf_record_bytes", "tri_shade_bytes")}
    peaks = pkg.measure_peaks(local, sum(hot_bytes.values()))
    note(f"peaks {({k: round(v) for k, v in peaks.items()})}")
    # Counting passes (not timed).  (1) the reference's exact work (rays, node visits, tests): the
    # metric's ray counts, equal to the reference's counters (parity tests); (2) the production walks'
    # own fetched bytes (RT_DEBUG 0x20: a scene whose counting kernels walk the timed kernels' trees).
    scene.counters_reset(sp)
    scene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world, count=True)
    cnt = scene.counters_read()
    ref_alg_bytes = (cnt["node_visits"] * B_NODE + cnt["tri_tests"] * B_TRI + cnt["sphere_tests"] * B_SPH
                     + rows * W * aa * aa * B_PIX)
    dbg0 = os.environ.get("RT_DEBUG")
    os.environ["RT_DEBUG"] = str(int(dbg0 or "0", 0) | 0x20)
    try:
        pscene = pkg.Scene.from_xml(xml, device=local, render_path=a.path)
    finally:
        if dbg0 is None:
            os.environ.pop("RT_DEBUG", None)
        else:
            os.environ["RT_DEBUG"] = dbg0
    pscene.counters_reset(sp)
    pscene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world, count=True)
    pcnt = pscene.counters_read()
    roles = pscene.counters_raw()
    pscene.close()
    scene.counters_reset(sp)      # from here on the slots count the timed kernels' fallback work (kCntFb*)
    if any(pcnt[k] != cnt[k] for k in ("primary_rays", "shadow_rays", "reflection_rays")):
        raise RuntimeError(f"production counting pass disagrees on ray counts: {pcnt} vs {cnt}")
    if traversal_bytes(roles) != pcnt["node_visits"]:
        raise RuntimeError(f"per-role fetch bytes do not add up: {roles} vs {pcnt['node_visits']}")
    nlights = len(re.findall(r"<PointLight\b", Path(xml).read_text()))
    kbytes = kernel_bytes(roles, cnt, rows * W, batched=F > 1, nlights=nlights)
    kbytes_one = kernel_bytes(roles, cnt, rows * W, batched=False, nlights=nlights)
    alg_bytes = sum(kbytes.values())
    trav_bytes = traversal_bytes(roles)
    ws_bytes = alg_bytes - trav_bytes
    note("counting passes done")
    ps_local = cnt["primary_rays"] + cnt["shadow_rays"]
    tot = torch.tensor([ps_local, cnt["primary_rays"], cnt["shadow_rays"], cnt["reflection_rays"],
                        cnt["shadow_rays_skipped"]], dtype=torch.float64, device=dev)
    tot = all_reduce(tot)
    ps_frame, prim_frame, shadow_frame, refl_frame, skip_frame = (int(x) for x in tot.tolist())

    def step(n, ev_pair=None):
        """n frames (steps) submitted together: this rank's stripes of each, then (N>1) one gather."""
        b = nxt[0]
        nxt[0] = (b + 1) % NB
        sl = slab_bufs[b]
        if freed[b] is not None:
            stream.wait_event(freed[b])       # its previous batch has left for rank 0
        if ev_pair is not None:
            ev_pair[0].record(stream)
        if n == 1:
            scene.render_device(cam, aa, sl[0].data_ptr(), sp, S, rank, world)
        else:
            scene.render_frames_device([cam] * n, aa, [sl[f].data_ptr() for f in range(n)], sp, S, rank, world)
        if ev_pair is not None:
            ev_pair[1].record(stream)
        if world == 1:
            return None
        if backend == "gloo":
            return pkg.frame.assemble_frames(sl[:n].cpu(), H, S)
        if rank == 0 and n not in gbufs:
            gbufs[n] = torch.empty((world, n, rows, W, 3), dtype=torch.uint8, device=dev)
        comm.wait_stream(stream)
        with torch.cuda.stream(comm):
            out = pkg.frame.assemble_frames(sl[:n], H, S, unshuffle=unshuffle_dev, gbuf=gbufs.get(n), images=images)
            ev = torch.cuda.Event()
            ev.record(comm)
        freed[b] = ev
        return out

    def groups(k):
        return [min(F, k - i) for i in range(0, k, F)]

    # at least one full group, twice: every workspace is allocated, and sized by the continuation share
    # the first group's read-backs measured (rt_render_frames_device never waits for them on the host)
    for n in groups(max(a.warmup, F)) + ([F] if F > 1 else []):
        step(n)
    torch.cuda.synchronize(dev)
    note("warmup done")
    gs = groups(a.steps)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in gs]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for n, ev in zip(gs, evs):
        last = step(n, ev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    note(f"timed {a.steps} steps")
    kern_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / a.steps      # render time per frame (batch-amortised)
    # what the timed kernels left to k_fallback, per frame (warmup + timed frames since the reset)
    fbr = scene.counters_raw()
    fb_frames = max(a.warmup, F) + a.steps
    fallback = {k[3:]: round(fbr[k] / fb_frames, 2) for k in scene.FALLBACK_SLOTS if k.startswith("fb_") and k != "fb_launches"}
    fallback["launches_per_frame"] = round(fbr["fb_launches"] / fb_frames, 4)
    # the timed launches' phase-A record size (compact 16-B records where a launch's frames needed them,
    # rt_api.cpp full_records_fit): the per-kernel byte model follows the majority
    compact_frac = fbr["compact_launches"] / max(1, fbr["fb_launches"])
    fallback["compact_record_launches_frac"] = round(compact_frac, 3)
    kbytes = kernel_bytes(roles, cnt, rows * W, batched=F > 1, nlights=nlights, compact=compact_frac >= 0.5)
    alg_bytes = sum(kbytes.values())
    ws_bytes = alg_bytes - trav_bytes
    fallback["note"] = ("per frame, timed kernels: continuations A->B, those beyond the phase-B record space "
                        "(walked whole by k_fallback), deferred closest-hit / shadow rays (outside the wide "
                        "trees' slab-test range), fallback shadow-queue overflows")

    # N=1: the last timed batch's frames, as the timed kernels left them, against the reference's golden
    # RGB (every frame bit-equal to the first, whose sha256 is the golden's)
    golden_ok = None
    if world == 1:
        import hashlib
        want = golden_sha(config, aa)
        n_last = gs[-1]
        frames = slab_bufs[(nxt[0] - 1) % NB][:n_last]
        sha0 = hashlib.sha256(frames[0].cpu().numpy().tobytes()).hexdigest()
        golden_ok = {"frames_checked": n_last, "equal_to_first": all(torch.equal(frames[i], frames[0]) for i in range(n_last)),
                     "sha256_first": sha0, "golden_sha256": want,
                     "equal": (want is not None and sha0 == want)}
    # N>1: the assembled frames equal one GPU's whole-frame render (checked after timing, rank 0)
    frames_ok = None
    if world > 1 and rank == 0:
        full = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        scene.render_device(cam, aa, full.data_ptr(), sp, H, 0, 1)
        torch.cuda.synchronize(dev)
        frames_ok = all(torch.equal(f.to(dev), full) for f in last)

    # single-frame latency (one frame alone on the GPU, this rank's stripes; reported, not `value`)
    # (two untimed frames first: a drop-in caller's repeated camera, whose previous frame ranked the unit
    # deal; the first frame of a view is single_frame_cold's case)
    lat = []
    for _ in range(0 if a.trace else 2):
        scene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world)
    for _ in range(0 if a.trace else 9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        scene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        lat.append(e0.elapsed_time(e1))
    lat_ms = sorted(lat)[len(lat) // 2] if lat else float("nan")

    def dev_ms(fn, reps=5):
        out = []
        for i in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn(i)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            out.append(e0.elapsed_time(e1))
        return out

    # the drop-in caller's other lone frames (reported, not `value`): a moving camera (a different eye every
    # frame: the phase-A unit order comes from the previous, different frame), and cold frames -- a scene
    # whose frames never use a previous frame's unit costs (RT_HOT_UNITS=0: every frame dealt as a first
    # one is), its first call's wall time (workspace allocation included) beside the device time of the rest
    lone_extra = None
    if not a.trace and world == 1:
        import ctypes as _ct

        def moved(i):
            c = pkg.Camera()
            _ct.memmove(_ct.addressof(c), _ct.addressof(cam), _ct.sizeof(c))
            c.position.x = cam.position.x + 0.002 * (i + 1)
            c.position.y = cam.position.y + 0.001 * (i + 1)
            return c

        mv = dev_ms(lambda i: scene.render_device(moved(i), aa, slab.data_ptr(), sp, S, rank, world), reps=7)
        saved = os.environ.get("RT_HOT_UNITS")
        os.environ["RT_HOT_UNITS"] = "0"
        try:
            cscene = pkg.Scene.from_xml(xml, device=local, render_path=a.path)
        finally:
            if saved is None:
                os.environ.pop("RT_HOT_UNITS", None)
            else:
                os.environ["RT_HOT_UNITS"] = saved
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        cscene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world)
        torch.cuda.synchronize(dev)
        first_wall = (time.perf_counter() - t1) * 1e3
        cold = dev_ms(lambda i: cscene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world), reps=7)
        cold_ws = cscene.memory()["workspace_bytes"]
        cscene.close()
        lone_extra = {
            "single_frame_cold": {"ms": round(sorted(cold)[len(cold) // 2], 4),
                                  "first_call_wall_ms": round(first_wall, 3),
                                  "workspace_bytes": cold_ws,
                                  "definition": "one frame alone, device time, phase-A units dealt without any "
                                                "previous frame's costs (RT_HOT_UNITS=0: what a first render of a "
                                                "camera does), median of 7; first_call_wall_ms: the scene's first "
                                                "call incl. workspace allocation, host wall"},
            "single_frame_moving": {"ms": round(sorted(mv)[len(mv) // 2], 4),
                                    "definition": "one frame alone, device time, camera moved every frame (the unit "
                                                  "order comes from the previous, different view), median of 7"},
        }
    tmax = torch.tensor([elapsed, kern_ms, lat_ms], dtype=torch.float64, device=dev)
    tmax = all_reduce(tmax, dist.ReduceOp.MAX)
    elapsed, kern_ms_max, lat_ms = tmax.tolist()

    # SURVEY §8(d) ms/frame (rank 0, N=1 only; beside `value`): rt_render wall time = camera upload,
    # render, D2H of the uint8 frame, one frame at a time
    host_ms = None
    if world == 1 and not a.trace:
        scene.render(cam, aa)
        ts = []
        for _ in range(7):
            t1 = time.perf_counter()
            scene.render(cam, aa)
            ts.append(time.perf_counter() - t1)
        host_ms = sorted(ts)[len(ts) // 2] * 1e3

    footprint = scene.memory()
    footprint["total_bytes"] = footprint["scene_bytes"] + footprint["workspace_bytes"]

    # per-kernel device time (rank 0): a scene with RT_DEBUG 0x10 launches each kernel of a chain launch with
    # its own start / stop timestamps (hipExtLaunchKernel events: the dispatch's begin and end, as rocprofv3
    # --kernel-trace reports them) on ONE workspace slot (kernels back to back) -- the frame batches of the
    # timed configuration and one frame alone.  The slot's workspace share is the timed run's (the scene
    # and the 64 MB staging reserve off the budget, the rest over the slots), so its launches hold as many
    # frames as the timed run's do
    ktimes = None
    if rank == 0 and a.path == "chain" and not a.trace:
        saved = {k: os.environ.get(k) for k in ("RT_DEBUG", "RT_SLOTS", "RT_WS_BUDGET_MB")}
        os.environ.update(RT_DEBUG=str(int(saved["RT_DEBUG"] or "0", 0) | 0x10),
                          **(one_slot_env() if not a.one_slot else {}))
        try:
            kscene = pkg.Scene.from_xml(xml, device=local, render_path=a.path)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        ktimes = {}
        for mode, n in (("batched", F), ("one_frame", 1)):
            reps = 2 if n > 1 else 5
            for rep in range(reps + 1):
                if n > 1:
                    kscene.render_frames_device([cam] * n, aa, [slab_bufs[0][f].data_ptr() for f in range(n)], sp,
                                                S, rank, world)
                else:
                    kscene.render_device(cam, aa, slab.data_ptr(), sp, S, rank, world)
                torch.cuda.synchronize(dev)
                if rep == 0:
                    kscene.kernel_times(reset=True)       # the first round allocates the workspace
            ms, launches = kscene.kernel_times(reset=True)
            frames = reps * n
            ktimes[mode] = {k: round(v / frames, 5) for k, v in ms.items() if v > 0}
            ktimes[mode]["launches_per_frame"] = round(launches / frames, 4)
        kscene.close()
        ktimes["timing"] = ("hipExtLaunchKernel start/stop events per kernel (the dispatch's own timestamps, "
                            "rocprofv3-equivalent), one workspace slot with the timed run's share")

    # HBM bytes per frame from the committed rocprofv3 FETCH/WRITE passes of the SAME mode as the time they
    # are priced against: frame batches (one workspace slot) for `value`, one frame alone for --inflight 1
    traffic, traffic_src = None, None
    mode = "batched" if F > 1 else "one_frame"
    tfile = ROOT / "profiles" / (f"traffic_{mode}.json" if aa == 1 else f"traffic_{mode}_aa{aa}.json")
    if tfile.exists():
        t = json.loads(tfile.read_text())
        if (t.get("config") == config and t.get("aa", 1) == aa and t.get("path") == a.path
                and t.get("hbm_bytes_per_frame")):
            traffic = int(t["hbm_bytes_per_frame"] / world)
            traffic_src = (f"profiles/{t.get('tag')}_traffic.json ({mode}; rocprofv3 2*FETCH_SIZE+WRITE_SIZE, "
                           f"N=1 frame / N)")
    if rank == 0:
        ms = elapsed / a.steps * 1e3
        value = ps_frame * a.steps / elapsed / 1e6
        # priced against the driver-timed wall time per frame (ms_per_step), as the headline is
        achieved = alg_bytes / (ms / 1e3) / 1e9
        # each kernel's own fraction: its alg bytes per frame / its one-slot time per frame (RT_DEBUG 0x10),
        # against the measured L2 full-line peak (and the divergent-gather ceiling of its fetch shape)
        per_kernel, per_kernel_one, dominant = None, None, None

        def kernel_fracs(kb, kt):
            out = {}
            for k, b in kb.items():
                t = kt.get(k)
                gbps = b / (t / 1e3) / 1e9 if t else None
                out[k] = {"alg_bytes": int(b), "ms_one_slot": t,
                          "achieved": round(gbps, 1) if gbps else None,
                          "frac": round(gbps / peaks["l2_line_gbps"], 4) if gbps else None,
                          "frac_of_guide_l2": round(gbps / L2_GUIDE_GBPS, 4) if gbps else None,
                          "frac_of_divergent_gather": round(gbps / peaks["l2_gather_gbps"], 4) if gbps else None}
            return out
        if ktimes:
            kt = ktimes["batched" if F > 1 else "one_frame"]
            # the byte model follows the launches the one-slot timing actually made: several frames per launch
            # (A's shadow rays in k_occlude) or one (k_mix's shadow role)
            kb_slot = kernel_bytes(roles, cnt, rows * W, batched=F > 1 and kt.get("launches_per_frame", 1) < 1,
                                   nlights=nlights, compact=compact_frac >= 0.5)
            per_kernel = kernel_fracs(kb_slot, kt)
            per_kernel_one = kernel_fracs(kbytes_one, ktimes["one_frame"])
            # the dominant kernel by rocprofv3's names (k_occlude = A's and B's shadow launches together)
            by_name = {}
            for k, b in kb_slot.items():
                nm = "k_occlude" if k.startswith("k_occlude") else k
                bb, tt = by_name.get(nm, (0, 0.0))
                by_name[nm] = (bb + b, tt + (kt.get(k) or 0.0))
            dk = max((k for k in by_name if by_name[k][1] > 0), key=lambda k: by_name[k][1])
            db, dt = by_name[dk]
            gb = db / (dt / 1e3) / 1e9
            dominant = {"kernel": dk, "alg_bytes": int(db), "ms_one_slot": round(dt, 5), "achieved": round(gb, 1),
                        "frac": round(gb / peaks["l2_line_gbps"], 4), "frac_of_guide_l2": round(gb / L2_GUIDE_GBPS, 4),
                        "frac_of_divergent_gather": round(gb / peaks["l2_gather_gbps"], 4),
                        "named_by": "rocprofv3 kernel name, largest one-slot time"}
        traffic_gbps = traffic / (ms / 1e3) / 1e9 if traffic else None
        if backend != "nccl":
            desc += f" [REHEARSAL: {backend} host-staged gather, all ranks on one GPU; not a measurement]"
        line = {
            "metric": "Mray/s (primary+shadow), horse_and_mug 1920x1080 depth 6" if a.config == "C3"
                      else f"Mray/s (primary+shadow), {desc}",
            "value": round(value, 3), "unit": "Mray/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (reference scene file, derived per SURVEY §8d)",
            "config": {"workload": config, "description": desc, "width": W, "height": H, "aa": aa,
                       "max_recursion_depth": int(re.search(r"<MaxRecursionDepth>\s*(-?\d+)", Path(xml).read_text()).group(1)),
                       "parallelism": f"stripes{S}x{world}" + ("+rccl_gather" if world > 1 else ""),
                       "frames_in_flight": F, "frame_latency_ms": round(lat_ms, 4) if lat else None,
                       "workspace_slots": int(os.environ.get("RT_SLOTS", max(1, min(6, int(os.environ["GPU_MAX_HW_QUEUES"]) - 1)))),
                       "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                       # every frame this process rendered on the GPU (counting pass, warmup, timed, latency,
                       # host-buffer runs): the divisor for whole-run PMC totals (tools/summarize_profile.py)
                       "frames_rendered_total": 2 + max(a.warmup, F) + (F if F > 1 else 0) + a.steps
                                                + (0 if a.trace else 5 + (8 + 15 if world == 1 else 0)),
                       # frames the non-counting kernels rendered in a --trace run (warmup + timed)
                       "trace_frames": max(a.warmup, F) + (F if F > 1 else 0) + a.steps if a.trace else None,
                       "assembled_frames_equal_single_gpu": frames_ok,
                       "timed_frames_equal_golden": golden_ok,
                       "primary_rays": prim_frame, "shadow_rays": shadow_frame, "reflection_rays": refl_frame,
                       # of shadow_rays: rays the timed kernels do not trace because their result cannot
                       # change the pixel (light behind the surface, pathchain.hip light_needed); the
                       # image is the reference's either way (parity tests)
                       "shadow_rays_skipped": skip_frame,
                       "mray_s_traced": round((ps_frame - skip_frame) * a.steps / elapsed / 1e6, 3),
                       "mray_s_all": round((ps_frame + refl_frame) * a.steps / elapsed / 1e6, 3),
                       "scene_load_s": round(load_s, 4),
                       "host_build": {"bvh_build_ms": round(binfo["build_ms"], 2), "ref_tree_ms": round(binfo["ref_ms"], 2),
                                      "wide_tree_ms": round(binfo["wide_ms"], 2), "threads": binfo["build_threads"]},
                       "value_definition": f"REFERENCE-EQUIVALENT primary+shadow rays: the reference's own "
                                           f"counters for a frame (incl. the shadow_rays_skipped that the timed "
                                           f"kernels provably need not trace; mray_s_traced excludes them) x "
                                           f"frames / wall time; frames submitted {F} at a time as frame batches, "
                                           "scene and frames resident in HBM, max-over-ranks wall time"},
            "single_frame": ({"ms": round(lat_ms, 4), "mray_s": round(ps_frame / lat_ms / 1e3, 3),
                              "definition": "one frame alone on the GPU (rt_render_device), device time, the same camera "
                                            "again (after two untimed frames of it), median of 9"}
                             if lat else None),
            **(lone_extra or {}),
            "hbm_footprint": footprint,
            "fallback": fallback,
            "kernel_ms_one_slot": ktimes,
            "drop_in": ({"ms_per_frame": round(host_ms, 4), "mray_s": round(ps_frame / host_ms / 1e3, 3),
                         "definition": "SURVEY §8(d): rt_render wall time, camera upload to the uint8 frame in "
                                       "host memory (PCIe included), one frame at a time"} if host_ms else None),
            "roofline": {"bound": "l2", "achieved": round(achieved, 2), "peak": round(peaks["l2_line_gbps"], 1),
                         "unit": "GB/s", "frac": round(achieved / peaks["l2_line_gbps"], 4), "traffic": traffic,
                         "frac_of_guide_l2": round(achieved / L2_GUIDE_GBPS, 4), "peak_guide_l2": L2_GUIDE_GBPS,
                         "time_basis": "ms_per_step (the driver-timed wall time per frame); kernel_ms beside it",
                         "bound_note": "the walks gather 128-B lines of a ~5 MB cache-resident scene; the bytes the "
                                       "timed kernels fetch and move are priced against the MEASURED L2 bandwidth for "
                                       "full-line fetches (rt_measure_peaks l2_line_gbps: random lines of a table inside "
                                       "one XCD's L2, 8 lanes per line).  The walks fetch each node per lane (64 distinct "
                                       "lines per wave instruction), whose measured ceiling is the divergent gather "
                                       "(l2_gather_gbps, the texture-address path): frac_of_divergent_gather.  The HBM "
                                       "bytes they actually move (PMC) are `hbm`, priced against the measured HBM copy",
                         "frac_of_divergent_gather": round(achieved / peaks["l2_gather_gbps"], 4),
                         "peak_measured": {k: round(v, 1) for k, v in peaks.items()},
                         "walk_hot_set_bytes": hot_bytes,
                         "alg_bytes_per_launch": int(alg_bytes), "launch_unit": "one frame (this rank's stripes)",
                         "alg_bytes_split": {"traversal": int(trav_bytes), "workspace": int(ws_bytes)},
                         "per_kernel": per_kernel,
                         "per_kernel_one_frame": per_kernel_one,
                         "dominant": dominant,
                         "alg_bytes_per_kernel": {k: int(v) for k, v in kbytes.items()},
                         "hbm": {"bytes_per_frame": traffic, "gbps": round(traffic_gbps, 2) if traffic else None,
                                 "peak": round(peaks["hbm_copy_gbps"], 1), "peak_guide": HBM_GUIDE_GBPS,
                                 "spec": HBM_SPEC_GBPS,
                                 "frac": round(traffic_gbps / peaks["hbm_copy_gbps"], 4) if traffic else None,
                                 "frac_of_guide": round(traffic_gbps / HBM_GUIDE_GBPS, 4) if traffic else None,
                                 "mode": mode, "source": traffic_src},
                         "reference_model": {"bytes_per_frame": int(ref_alg_bytes),
                                             "note": "SURVEY §8(d) per-operation model of the reference's own walk "
                                                     "(32 B/node visit, 36 B/triangle test, 16 B/sphere test, 3 B/px)",
                                             "counts": {k: cnt[k] for k in ("node_visits", "tri_tests",
                                                                            "sphere_tests")}},
                         "path": a.path, "kernels": PATH_KERNELS[a.path],
                         "kernel": "one frame = " + " + ".join(PATH_KERNELS[a.path])
                                   + (f" (frames in batches of up to {F}: kernel_ms = batch time / frames)" if F > 1 else ""),
                         "kernel_ms": round(kern_ms, 4)},
        }
        if world == 1 and not a.no_cpu_baseline and not a.trace:
            line["cpu_baseline"] = cpu_baseline(xml, aa, ps_frame, a.cpu_seconds)
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
