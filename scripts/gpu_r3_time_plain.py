"""Finalize step on MessageSets that do not compress (random bytes, kept plain by the codec
choice): 8192 x 64 KiB and 512 x 1 MiB, exact and throughput mode, HIP events.
Usage: python scripts/gpu_r3_time_plain.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import librdkafka_amd as L  # noqa: E402
from librdkafka_amd import workload as W  # noqa: E402

L.init(0)
rng = np.random.default_rng(7)
for n, size in ((8192, 65536), (512, 1 << 20)):
    slot = 64 + size
    host = np.zeros(n * slot + 256, dtype=np.uint8)
    view = host[:n * slot].reshape(n, slot)
    view[:, 61:61 + size] = rng.integers(0, 256, (n, size), dtype=np.uint8)
    hdr = np.frombuffer(W.v2_header(0, 61 + size), dtype=np.uint8)
    view[:, :61] = hdr
    d_in = torch.from_numpy(host).cuda()
    in_offs = torch.arange(n, dtype=torch.int64, device="cuda") * slot + 61
    in_lens = torch.full((n,), size, dtype=torch.int32, device="cuda")
    cap = (61 + L.lz4f_compress_bound(size) + 255) // 256 * 256
    d_out = torch.empty(n * cap + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * cap
    caps = torch.full((n,), cap, dtype=torch.int32, device="cuda")
    flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    for mode in (0, 1):
        fn = lambda: L.msgset_v2_finalize(d_in, in_offs, in_lens, d_out, out_offs, caps, flens, blens, crcs, mode=mode)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        L.msgset_v2_crc(d_out, out_offs, caps, st, L.V2_CRC_VERIFY)
        ok = int(st.abs().sum()) == 0 and bool((blens == size + 61).all())
        print(f"plain {n} x {size} mode {mode}: {ms:.3f} ms {n * size / ms / 1e6:.1f} GB/s verified={ok}", flush=True)
