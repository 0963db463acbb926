#!/usr/bin/env python3
"""End-to-end drop-in timing: the drop-in CLI (raytracer-ceng477-graphics-hw-1_amd/raytracer,
csrc/raytracer_cli.cpp) beside the reference's own executable (oracle/_ref/ref_stock: its main, raytracer.cpp:
487-525, SSAA factor 2 hard-coded) and, for other SSAA factors, the reference harness writing the same PPMs
(oracle/_ref/ref_harness --aa F --out-dir).  Each run is a fresh process, wall time from exec to exit (the CLI's
includes HIP initialisation); the PPM bytes of both are compared.  The README's published figures
(reference README.md: horse_and_mug 0.452 s; 256x AA 40 s; low poly 4x AA 1 s; 8K 4x AA 44.7 s) sit beside them.

  python tools/exp_cli.py [--reps N] [--quick]
  python tools/exp_cli.py --phases [--reps N]     (the CLI's wall time split by phase, horse_and_mug AA1/AA2)
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402

CLI = ROOT / "raytracer-ceng477-graphics-hw-1_amd" / "raytracer"
STOCK = ROOT / "oracle" / "_ref" / "ref_stock"
HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"


def run(cmd, cwd):
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=600)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{cmd}: rc {r.returncode}: {r.stderr[-400:]}")
    lines = {}
    for k in ("Planted trees in", "Rendered in", "Total:"):
        m = re.search(re.escape(k) + r" ([0-9.]+) seconds", r.stdout)
        if m:
            lines[k.split()[0].lower()] = float(m.group(1))
    return wall, lines


def shas(d):
    return {p.name: hashlib.sha256(p.read_bytes()).hexdigest()[:16] for p in sorted(Path(d).glob("*.ppm"))}


def phases(hm, reps, extra_env=None, aa=1):
    """One CLI process per rep with --timing and RT_DEBUG=1: the steady-clock (CLOCK_MONOTONIC) stamps the
    CLI and the library's warm-up thread print, against the parent's own stamps around the process."""
    rows = []
    for _ in range(reps):
        wd = tempfile.mkdtemp()
        env = dict(os.environ, **(extra_env or {}))
        env["RT_DEBUG"] = str(int(env.get("RT_DEBUG", "0"), 0) | 1)
        t_spawn = time.monotonic() * 1e3
        r = subprocess.run([str(CLI), hm, "--aa", str(aa), "--timing"], cwd=wd, capture_output=True, text=True,
                           timeout=120, env=env)
        t_end = time.monotonic() * 1e3
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-400:])
        ev = {}
        for l in r.stderr.splitlines():
            if l.startswith("{"):
                ev.update(json.loads(l))
        c, i, i2 = ev["cli"], ev.get("rt_init", {}), ev.get("rt_init2", {})
        row = {"wall": t_end - t_spawn, "spawn_to_main": c["main"] - t_spawn,
               "load": c["loaded"] - c["main"], "render_d2h": c["rendered"] - c["loaded"],
               "write_ppm": c["written"] - c["rendered"], "after_write_to_exit": t_end - c["written"],
               "xml": c["xml_ms"], "tree_build": c["prep_ms"] + c["ref_tree_ms"] + c["flat_ms"] + c["refwide_ms"],
               "stree": c["stree_ms"], "upload_after_build": c["upload_ms"]}
        if i:
            row.update({"init_start_after_main": i["start"] - c["main"], "hip_device_count": i["device_count"] - i["start"],
                        "hip_context": i["context"] - i["device_count"], "first_device_op": i["first_op"] - i["context"],
                        "init_end_after_main": i["first_op"] - c["main"]})
            if i2:     # the second warm-up thread (joined after the upload)
                row.update({"code_objects": i2["code_objects"] - i["context"], "readback_warm": i2["readback"] - i2["code_objects"],
                            "init2_end_after_main": i2["readback"] - c["main"]})
        rc = ev.get("rt_render_cameras")
        if rc:     # inside render_d2h: output buffers, submission, GPU done, D2H copies (ms from the call's start)
            row.update({"rc_outputs": rc["outputs_ms"], "rc_submit": rc["submitted_ms"] - rc["outputs_ms"],
                        "rc_gpu_wait": rc["gpu_done_ms"] - rc["submitted_ms"], "rc_d2h": rc["copied_ms"] - rc["gpu_done_ms"]})
        rows.append(row)
    keys = rows[0].keys()
    return {k: round(sorted(r[k] for r in rows)[len(rows) // 2], 2) for k in keys}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--quick", action="store_true", help="skip the 8K and 256x cases")
    ap.add_argument("--phases", action="store_true", help="only the CLI's per-phase split (ms, medians)")
    a = ap.parse_args()
    pkg = graft.import_pkg()
    d = tempfile.mkdtemp()
    if a.phases:
        hm = pkg.scenes.write_config("hm_verbatim", d)
        for aa in (1, 2):
            variants = [("default", None), ("normal_exit", {"RT_CLI_EXIT": "normal"}), ("no_warmup", {"RT_DEBUG": "9"})]
            if os.environ.get("EXP_CLI_VARIANTS"):    # "name:K=V,K2=W;name2:..." instead of the three above
                variants = [(v.split(":")[0], dict(kv.split("=", 1) for kv in v.split(":", 1)[1].split(",") if kv))
                            for v in os.environ["EXP_CLI_VARIANTS"].split(";")]
            for name, env in variants:
                print(json.dumps({"scene": "horse_and_mug.xml", "aa": aa, "variant": name,
                                  "median_ms": phases(hm, a.reps, env, aa)}), flush=True)
        return
    hm = pkg.scenes.write_config("hm_verbatim", d)
    lp = pkg.scenes.write_config("low_poly.xml", d)
    text = Path(hm).read_text()
    hm8k = Path(d) / "horse_and_mug_8k.xml"
    hm8k.write_text(pkg.scenes.derive_xml(text, res=(7680, 4320), image_name="horse_and_mug_8k.ppm"))
    cases = [("horse_and_mug.xml", hm, 2, "README: 0.452 s (Ubuntu), 0.7 s (Windows)"),
             ("horse_and_mug.xml", hm, 1, None),
             ("low_poly.xml", lp, 2, "README: 1 s with 4x AA")]
    if not a.quick:
        cases += [("horse_and_mug 7680x4320", str(hm8k), 2, "README: 44.7 s, 8K with 4x AA"),
                  ("horse_and_mug.xml", hm, 16, "README: 40 s with 256x AA")]
    out = []
    for name, xml, aa, pub in cases:
        res = {"scene": name, "aa": aa, "published": pub}
        for who in ("cli", "reference"):
            walls, lines, sha = [], None, None
            reps = a.reps if (who == "cli" or aa <= 2) and "7680" not in name else 1
            for _ in range(reps):
                wd = tempfile.mkdtemp()
                if who == "cli":
                    cmd = [str(CLI), xml, "--aa", str(aa)]
                elif aa == 2:
                    cmd = [str(STOCK), xml]
                else:
                    cmd = [str(HARNESS), xml, "--aa", str(aa), "--out-dir", wd]
                w, lines = run(cmd, wd)
                walls.append(w)
                sha = shas(wd)
            walls.sort()
            res[who] = {"wall_s_median": round(walls[len(walls) // 2], 4), "wall_s": [round(w, 4) for w in walls],
                        "printed": lines, "ppm_sha": sha,
                        "cmd": "drop-in CLI" if who == "cli" else ("reference main (ref_stock)" if aa == 2
                                                                    else "reference harness --out-dir")}
            print(f"{name} aa{aa} {who}: {res[who]['wall_s_median']} s {lines}", file=sys.stderr, flush=True)
        res["ppm_identical"] = res["cli"]["ppm_sha"] == res["reference"]["ppm_sha"]
        res["speedup_wall"] = round(res["reference"]["wall_s_median"] / res["cli"]["wall_s_median"], 2)
        out.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
