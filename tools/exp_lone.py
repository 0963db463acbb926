#!/usr/bin/env python3
"""Experiment: one C3 frame alone (the reference's calling pattern), device time per frame,
under environment knobs.  Each argument is one configuration, "-" or "K=V,K2=V2"; each runs
in its own child process (the knobs are read when the scene is created).

  python tools/exp_lone.py - RT_EXP_SKIP_OCC=1 RT_BTAIL=16      (env EXP_REPS, EXP_SCENE)
"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path


def child():
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import __graft_entry__ as graft
    pkg = graft.import_pkg()
    xml = pkg.scenes.write_config(os.environ.get("EXP_SCENE", "C3_hm_1080p_d6"), tempfile.mkdtemp())
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    reps = int(os.environ.get("EXP_REPS", "31"))
    with pkg.Scene.from_xml(xml, device=0) as s:
        cam = s.camera(0)
        out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device=dev)
        for _ in range(3):
            s.render_device(cam, 1, out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        s.counters_reset(st.cuda_stream)
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            s.render_device(cam, 1, out.data_ptr(), st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        kt = None
        if os.environ.get("RT_KTIME"):
            ms, n = s.kernel_times(reset=True)
            kt = {k: round(v / (reps + 3), 4) for k, v in ms.items()}
        fbr = s.counters_raw()           # what the timed kernels left to k_fallback, per frame
        fb = {(k[3:] if k.startswith("fb_") else k): round(fbr[k] / reps, 1) for k in s.FALLBACK_SLOTS if k != "fb_launches" and fbr[k]}
        print(json.dumps({"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4), "fallback": fb,
                          "sha_prefix": __import__("hashlib").sha256(out.cpu().numpy().tobytes()).hexdigest()[:12],
                          "kernel_times": kt}))


def main():
    for cfg in sys.argv[1:] or ["-"]:
        env = dict(os.environ)
        if cfg != "-":
            for kv in cfg.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        env["EXP_LONE_CHILD"] = "1"
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        res = json.loads(line[-1]) if line else {"error": r.stderr[-400:]}
        res["config"] = cfg
        print(json.dumps(res), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    child() if os.environ.get("EXP_LONE_CHILD") else main()
