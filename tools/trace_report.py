#!/usr/bin/env python3
"""Diagnostics: render the C3 frame once per render path with RT_TRACE set and
summarise the per-sample wall-clock trace (100 MHz counter, 10 ns ticks):
when samples start / finish, how many are in flight over time, the slowest
ones.  Answers "is the frame bound by bulk throughput or by its tail?".

  python tools/trace_report.py [chain|megakernel ...]     (env TRACE_FRAMES=n: one n-frame batch instead)
"""
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

TICK_US = 0.01


def load(path):
    raw = np.fromfile(path, dtype=np.uint32)
    assert raw[0] == 0x52545452
    kind, a, b, n = (int(x) for x in raw[1:5])
    return kind, a, b, raw[5:5 + n]


def rel(x, t0):
    return ((x.astype(np.int64) - int(t0)) & 0xffffffff).astype(np.int64) * TICK_US


def summarise(name, starts, ends, W=None):
    ok = ends != 0
    idx = np.nonzero(ok)[0]
    t0 = starts[ok].min()
    s, e = rel(starts[ok], t0), rel(ends[ok], t0)
    dur = e - s
    span = e.max()
    out = {"path": name, "samples": int(ok.sum()), "span_us": round(float(span), 1)}
    out["end_pct_us"] = {p: round(float(np.percentile(e, p)), 1) for p in (50, 90, 99, 99.9, 100)}
    out["start_pct_us"] = {p: round(float(np.percentile(s, p)), 1) for p in (50, 90, 99, 100)}
    out["dur_pct_us"] = {p: round(float(np.percentile(dur, p)), 1) for p in (50, 90, 99, 99.9, 100)}
    bins = np.linspace(0, span, 21)
    inflight = [int(((s <= t) & (e > t)).sum()) for t in bins[:-1]]
    out["inflight_by_5pct"] = inflight
    top = np.argsort(dur)[::-1][:8]
    rows = []
    for j in top:
        q = int(idx[j])
        rows.append({"q": q, "rc": [q // W, q % W] if W else None, "start": round(float(s[j]), 1),
                     "dur": round(float(dur[j]), 1)})
    out["slowest"] = rows
    last = np.argsort(e)[::-1][:5]
    out["last_to_finish"] = [{"q": int(idx[j]), "start": round(float(s[j]), 1), "dur": round(float(dur[j]), 1)}
                             for j in last]
    return out


def main():
    paths = sys.argv[1:] or ["chain", "megakernel"]
    pkg = graft.import_pkg()
    d = tempfile.mkdtemp()
    xml = pkg.scenes.write_config("C3_hm_1080p_d6", d)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    res = []
    for path in paths:
        tf = os.path.join(d, f"trace_{path}.bin")
        os.environ["RT_TRACE"] = tf
        sc = pkg.Scene.from_xml(xml, device=0, render_path=path)
        cam = sc.camera(0)
        nf = int(os.environ.get("TRACE_FRAMES", "1"))   # > 1: one frame batch of nf frames (one launch if it fits)
        out = torch.empty((nf, cam.image_height, cam.image_width, 3), dtype=torch.uint8, device=dev)
        for _ in range(3):
            if nf == 1:
                sc.render_device(cam, 1, out[0].data_ptr(), st.cuda_stream)
            else:
                sc.render_frames_device([cam] * nf, 1, [out[i].data_ptr() for i in range(nf)], st.cuda_stream)
        torch.cuda.synchronize()
        kind, a, b, tr = load(tf)
        if kind == 2:     # megakernel: per output pixel
            res.append(summarise(path, tr[0::2], tr[1::2], W=a))
        else:             # chain: samples then k_occlude blocks
            cap, og = a, b
            smp = tr[:2 * cap]
            r = summarise(path + "/k_chain", smp[0::2], smp[1::2])
            # per 8x8 tile (the 64 samples a wave grabs together): grab, last end, span -- the phase-A tail
            g0, g1 = smp[0::2].astype(np.int64), smp[1::2].astype(np.int64)
            ntile = cap // 64
            okt = (g1[:ntile * 64] != 0).reshape(ntile, 64)
            t00 = g0[g1 != 0].min()
            gs = np.where(okt, ((g0[:ntile * 64] - t00) & 0xffffffff).reshape(ntile, 64), 1 << 40).min(axis=1) * TICK_US
            ge = np.where(okt, ((g1[:ntile * 64] - t00) & 0xffffffff).reshape(ntile, 64), -1).max(axis=1) * TICK_US
            ge_med = np.array([np.median(((g1[t * 64:(t + 1) * 64][okt[t]] - t00) & 0xffffffff) * TICK_US)
                               if okt[t].any() else -1 for t in range(ntile)])
            live = okt.any(axis=1)
            order = np.argsort(-(ge - gs) * live)[:10]
            r["tiles"] = {"n": int(live.sum()),
                          "span_pct_us": {p: round(float(np.percentile((ge - gs)[live], p)), 1) for p in (50, 90, 99, 100)},
                          "longest": [{"tile": int(t), "grab": round(float(gs[t]), 1), "end": round(float(ge[t]), 1),
                                       "median_end": round(float(ge_med[t]), 1), "live": int(okt[t].sum()),
                                       # the tile's distinct (start, end) pairs: lanes of one wave end together
                                       "spans": sorted({(round(float(((g0[t * 64 + i] - t00) & 0xffffffff) * TICK_US), 1),
                                                         round(float(((g1[t * 64 + i] - t00) & 0xffffffff) * TICK_US), 1))
                                                        for i in range(64) if okt[t, i]})[:16]}
                                      for t in order]}
            ob = tr[2 * cap:2 * (cap + og)]
            okb = ob[1::2] != 0
            t0 = smp[0::2][smp[1::2] != 0].min()
            if okb.any():      # k_occlude block spans (the leaf-queue walker does not record them)
                os_, oe = rel(ob[0::2][okb], t0), rel(ob[1::2][okb], t0)
                r["k_occlude_blocks"] = {"start_min": round(float(os_.min()), 1), "start_max": round(float(os_.max()), 1),
                                         "end_pct_us": {p: round(float(np.percentile(oe, p)), 1) for p in (0, 50, 90, 99, 100)}}
            pb = tr[2 * (cap + og):2 * (cap + og) + 4 * cap].reshape(-1, 4)
            okp = pb[:, 1] != 0
            if okp.any():        # phase-B continuations (k_mix chain role): grab, end, last level, walk steps
                q = np.nonzero(okp)[0]
                bs, be = rel(pb[okp, 0], t0), rel(pb[okp, 1], t0)
                bd = be - bs
                lv, stp = (pb[okp, 2] & 255).astype(np.int64), (pb[okp, 3] & 0x7fffffff).astype(np.int64)
                coop = (pb[okp, 3] >> 31).astype(np.int64)      # the chain walked in coop rounds (pathchain.hip)
                wit = (pb[okp, 2] >> 8).astype(np.int64)      # the wave's walk iterations meanwhile
                top = np.argsort(bd)[::-1][:8]
                # each continuation's phase-A end (same path index): when a streaming A->B hand-off
                # could have started it, and the frame end that would give at the same chain times
                a_end = rel(smp[1::2][q], t0)
                a_end = np.where(smp[1::2][q] != 0, a_end, 0.0)
                last_b = np.argsort(be)[::-1][:8]
                r["stream_whatif"] = {
                    "end_if_started_at_a_end_us": round(float((a_end + bd).max()), 1),
                    "end_pct_if_started_at_a_end_us": {p: round(float(np.percentile(a_end + bd, p)), 1)
                                                       for p in (50, 99, 99.9, 100)},
                    "last_to_finish": [{"q": int(q[j]), "a_end": round(float(a_end[j]), 1),
                                        "b_start": round(float(bs[j]), 1), "b_dur": round(float(bd[j]), 1),
                                        "level": int(lv[j])} for j in last_b]}
                r["phase_b"] = {
                    "chains": int(okp.sum()),
                    "start_pct_us": {p: round(float(np.percentile(bs, p)), 1) for p in (0, 50, 100)},
                    "end_pct_us": {p: round(float(np.percentile(be, p)), 1) for p in (50, 90, 99, 99.9, 100)},
                    "dur_pct_us": {p: round(float(np.percentile(bd, p)), 1) for p in (50, 90, 99, 100)},
                    "steps_pct": {p: int(np.percentile(stp, p)) for p in (50, 90, 99, 100)},
                    "wave_iters_pct": {p: int(np.percentile(wit, p)) for p in (50, 90, 99, 100)},
                    "inflight_by_5pct": [int(((bs <= t) & (be > t)).sum()) for t in
                                         np.linspace(bs.min(), be.max(), 21)[:-1]],
                    "last_level_hist": np.bincount(lv).tolist(),
                    "coop_chains": int(coop.sum()),
                    "coop_by_level": np.bincount(lv[coop == 1], minlength=lv.max() + 1).tolist(),
                    "slowest": [{"q": int(q[j]), "start": round(float(bs[j]), 1), "dur": round(float(bd[j]), 1),
                                 "level": int(lv[j]), "steps": int(stp[j]), "wave_iters": int(wit[j]),
                                 "coop": int(coop[j]),
                                 "us_per_step": round(float(bd[j]) / max(1, int(stp[j])), 2)} for j in top]}
            res.append(r)
        sc.close()
        del os.environ["RT_TRACE"]
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
