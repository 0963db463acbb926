#!/usr/bin/env python3
"""Diagnostics: work counters of one C3 frame (counting pass) under the current env (e.g. RT_STREE=2)."""
import json, sys, tempfile
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft
pkg = graft.import_pkg()
d = tempfile.mkdtemp()
xml = pkg.scenes.write_config(sys.argv[1] if len(sys.argv) > 1 else "C3_hm_1080p_d6", d)
s = pkg.Scene.from_xml(xml, device=0)
img, st = s.render(s.camera(0), 1, stats=True)
print(json.dumps(st))
