import time, torch, numpy as np
dev = torch.device("cuda", 0)
src = torch.randint(0, 255, (1080, 1920, 3), dtype=torch.uint8, device=dev)
pin = torch.empty_like(src, device="cpu").pin_memory()
page = torch.empty_like(src, device="cpu")
def t(f, n=31):
    f(); torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter(); f(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    ts.sort(); return round(ts[n // 2] * 1e3, 4)
print("pageable copy_", t(lambda: page.copy_(src)))
print("pinned copy_", t(lambda: pin.copy_(src, non_blocking=True)))
print("pageable .cpu()", t(lambda: src.cpu()))
a = np.empty((1080, 1920, 3), np.uint8)
print("numpy memcpy 6.2MB", t(lambda: np.copyto(a, pin.numpy())))
