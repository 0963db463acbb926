#!/usr/bin/env python3
"""Experiment: the drop-in call (rt_render: one C3 frame into a host buffer, PCIe read-back included),
wall time per frame under environment knobs.  Each argument is one configuration, "-" or "K=V,K2=V2",
each in its own child process (knobs are read at scene creation).

  python tools/exp_dropin.py - RT_PIPE_PARTS=1 RT_PIPE_PARTS=8      (env EXP_REPS, EXP_SCENE)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path


def child():
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import __graft_entry__ as graft
    torch.cuda.init()
    pkg = graft.import_pkg()
    xml = pkg.scenes.write_config(os.environ.get("EXP_SCENE", "C3_hm_1080p_d6"), tempfile.mkdtemp())
    reps = int(os.environ.get("EXP_REPS", "41"))
    with pkg.Scene.from_xml(xml, device=0) as s:
        cam = s.camera(0)
        for _ in range(3):
            img, _ = s.render(cam, aa=1, stats=False)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            img, _ = s.render(cam, aa=1, stats=False)
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        print(json.dumps({"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                          "sha_prefix": hashlib.sha256(img.tobytes()).hexdigest()[:12]}))


def main():
    for cfg in sys.argv[1:] or ["-"]:
        env = dict(os.environ)
        if cfg != "-":
            for kv in cfg.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        env["EXP_DROPIN_CHILD"] = "1"
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        res = json.loads(line[-1]) if line else {"error": r.stderr[-400:]}
        res["config"] = cfg
        print(json.dumps(res), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    child() if os.environ.get("EXP_DROPIN_CHILD") else main()
