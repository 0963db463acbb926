#!/usr/bin/env python3
"""Same-box A/B (and call-size sweeps) of the production entry points, interleaved rounds.

Each argument is one configuration, "-" or "K=V,K2=V2" (environment knobs, RT_LIB=path for another build);
each runs in its own child process per round (knobs are read when the scene is created).  A child loads one
scene, warms up with two 96-frame calls (as bench.py does), then measures, for every call size n in
AB_CALLS, rt_render_frames_device of n frames (device time per frame, median of AB_REPS calls; n = 1 is
rt_render_device: one frame alone, the reference's calling pattern, median of AB_LONE frames) and checks
the last call's frames against the golden sha where one exists.

  python tools/ab_quick.py - RT_LIB=raytracer-ceng477-graphics-hw-1_amd/librt_old.so
  env AB_SCENE (C3_hm_1080p_d6 | mirror_spheres.xml | marbles.xml ...), AB_AA (1), AB_CALLS ("1,20"),
      AB_REPS (7), AB_LONE (41), AB_ROUNDS (3), AB_STRIPE (4)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child():
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    import torch
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as graft
    import bench
    pkg = graft.import_pkg()
    config = os.environ.get("AB_SCENE", "C3_hm_1080p_d6")
    aa = int(os.environ.get("AB_AA", "1"))
    calls = [int(x) for x in os.environ.get("AB_CALLS", "1,20").split(",")]
    reps, lone = int(os.environ.get("AB_REPS", "7")), int(os.environ.get("AB_LONE", "41"))
    S = int(os.environ.get("AB_STRIPE", "4"))
    xml = pkg.scenes.write_config(config, tempfile.mkdtemp())
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sp = st.cuda_stream
    want = bench.golden_sha(config, aa)
    res = {}
    with pkg.Scene.from_xml(xml, device=0) as s:
        cam = s.camera(0)
        H, W = cam.image_height, cam.image_width
        nmax = max(96, max(calls))
        bufs = torch.empty((nmax, H, W, 3), dtype=torch.uint8, device=dev)
        ptrs = [bufs[i].data_ptr() for i in range(nmax)]
        for _ in range(2):
            s.render_frames_device([cam] * 96, aa, ptrs[:96], sp, S)
        torch.cuda.synchronize()

        def timed(fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1)

        for n in calls:
            if n == 1:
                for _ in range(3):
                    s.render_device(cam, aa, ptrs[0], sp, S)
                ts = sorted(timed(lambda: s.render_device(cam, aa, ptrs[0], sp, S)) for _ in range(lone))
                ms = ts[len(ts) // 2]
            else:
                s.render_frames_device([cam] * n, aa, ptrs[:n], sp, S)
                ts = sorted(timed(lambda: s.render_frames_device([cam] * n, aa, ptrs[:n], sp, S)) / n
                            for _ in range(reps))
                ms = ts[len(ts) // 2]
            s.check()
            shas = {hashlib.sha256(bufs[i].cpu().numpy().tobytes()).hexdigest() for i in range(n)}
            res[str(n)] = {"ms_per_frame": round(ms, 4), "golden": (shas == {want}) if want else None}
    print(json.dumps(res))


def main():
    cfgs = sys.argv[1:] or ["-"]
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    allres = {c: [] for c in cfgs}
    for r in range(rounds):
        for cfg in cfgs:
            env = dict(os.environ)
            if cfg != "-":
                for kv in cfg.split(","):
                    k, v = kv.split("=", 1)
                    env[k] = v
            env["AB_CHILD"] = "1"
            p = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=400)
            line = [l for l in p.stdout.splitlines() if l.startswith("{")]
            if p.returncode != 0 or not line:
                print(json.dumps({"config": cfg, "round": r, "error": p.stderr[-600:]}), flush=True)
                sys.exit(p.returncode or 1)
            res = json.loads(line[-1])
            allres[cfg].append(res)
            print(json.dumps({"config": cfg, "round": r, **res}), flush=True)
    for cfg, rs in allres.items():
        summ = {n: round(sorted(x[n]["ms_per_frame"] for x in rs)[len(rs) // 2], 4) for n in rs[0]}
        ok = all(x[n]["golden"] is not False for x in rs for n in x)
        print(json.dumps({"summary": cfg, "median_of_rounds_ms_per_frame": summ, "golden_ok": ok}), flush=True)


if __name__ == "__main__":
    child() if os.environ.get("AB_CHILD") else main()
