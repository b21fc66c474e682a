"""Record writer throughput against the record size (the writer assembles a chunk of 256
records in LDS tiles: one tile up to ~140-byte records, several passes beyond).
Usage: time_serialize_sizes.py [VALUE_BYTES ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import librdkafka_amd as L  # noqa: E402


def messages(n, vbytes, seed):
    rnd = np.random.default_rng(seed)
    arena = rnd.integers(0, 256, n * vbytes + 64, dtype=np.uint8)
    m = {"arena": arena, "ts": 1600000000000 + np.arange(n, dtype=np.int64),
         "key_off": np.zeros(n, np.uint64), "key_len": np.full(n, -1, np.int32),
         "val_off": (np.arange(n, dtype=np.uint64) * np.uint64(vbytes)),
         "val_len": np.full(n, vbytes, np.int32)}
    d = {}
    for k, v in m.items():
        a = v.view(np.int64) if v.dtype == np.uint64 else v
        d[k] = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return d


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [100, 200, 1000, 5000, 100000]
    for vb in sizes:
        per_batch = max(1, (1 << 20) // (vb + 8))
        nb = 256
        d = messages(nb * per_batch, vb, 1)
        b = np.zeros(nb, dtype=L.V2_BATCH_DTYPE)
        b["first_msg"] = np.arange(nb) * per_batch
        b["msg_count"] = per_batch
        L.msgset_v2_build(d, b, crc=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            out, offs, sizes_, _ = L.msgset_v2_build(d, b, crc=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        total = int(sizes_.to(torch.int64).sum())
        print(f"value {vb:7d} B: {per_batch:6d} records x {nb} batches, {total / dt / 1e9:7.1f} GB/s "
              f"({dt * 1e3:.3f} ms)", flush=True)


if __name__ == "__main__":
    main()
