import sys, time, tempfile
sys.path.insert(0, "/root/repo")
import torch
import __graft_entry__ as g
pkg = g.import_pkg()
torch.cuda.init(); torch.zeros(1, device="cuda")
xml = pkg.scenes.write_config("C3_hm_1080p_d6", tempfile.mkdtemp())
for i in range(3):
    t0 = time.perf_counter(); s = pkg.Scene.from_xml(xml, host_only=True); t1 = time.perf_counter()
    d = pkg.Scene.from_xml(xml, device=0); t2 = time.perf_counter()
    print(f"host_only {1e3*(t1-t0):.1f} ms, device {1e3*(t2-t1):.1f} ms", s.bvh_info()["build_ms"])
    s.close(); d.close()
