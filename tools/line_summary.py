#!/usr/bin/env python3
"""One-line digest of bench.py JSON lines: python tools/line_summary.py FILE... (or stdin)."""
import json
import sys


def digest(d: dict) -> str:
    g = d.get("config", {}).get("timed_frames_equal_golden") or {}
    sf, cold, mv, di = (d.get(k) or {} for k in ("single_frame", "single_frame_cold", "single_frame_moving", "drop_in"))
    fp = d.get("hbm_footprint", {})
    kt = (d.get("kernel_ms_one_slot") or {})
    one = {k: v for k, v in (kt.get("one_frame") or {}).items() if k.startswith("k_")}
    return (f"{d['config']['workload']} aa{d['config']['aa']} steps {d['steps']}: {d['ms_per_step']} ms/frame "
            f"({d['value']} Mray/s) | lone {sf.get('ms')} cold {cold.get('ms')} (first {cold.get('first_call_wall_ms')}) "
            f"moving {mv.get('ms')} drop-in {di.get('ms_per_frame')} | golden {g.get('equal')} "
            f"| total HBM {fp.get('total_bytes', 0) / 2**30:.2f} GiB | roofline frac {d['roofline']['frac']} "
            f"| one-frame {one}")


files = sys.argv[1:] or ["-"]
for f in files:
    text = sys.stdin.read() if f == "-" else open(f).read()
    for line in text.splitlines():
        if line.startswith("{"):
            print(digest(json.loads(line)))
