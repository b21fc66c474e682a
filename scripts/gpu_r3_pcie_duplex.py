"""Pinned H2D and D2H copies alone and at the same time (two streams)."""
import time
import torch
n = 256 << 20
h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h, reps=8):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d1.copy_(h1, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    return reps * n / (time.perf_counter() - t0) / 1e9


run(True, True, 2)
print(f"H2D alone {run(True, False):.1f} GB/s", flush=True)
print(f"D2H alone {run(False, True):.1f} GB/s", flush=True)
both = run(True, True)
print(f"both at once: {both:.1f} GB/s each way, {2 * both:.1f} GB/s in total", flush=True)
