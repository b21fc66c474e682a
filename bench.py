#!/usr/bin/env python3
"""bench.py -- librdkafka record-batch engine on MI355X.

Headline (BASELINE.json configs[1]): CRC32C over 1M synthetic MsgVersion 2
record batches of 16 KiB on one MI355X, device-resident, bit-exact with
crc32c.c.  One step = one pass of the hot path (rd_kafka_msgset_writer
CRC finalize, rdkafka_msgset_writer.c:1229-1246) over all batches.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload crc|lz4c|lz4d|consumer]

For N>1 it is launched by torch.distributed.run, one rank per GPU.  Batches
shard by topic-partition across GPUs with no data-path collective (weak
scaling); gloo carries only the barrier and the max-over-ranks time.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
CRC_BATCHES = 1 << 20          # configs[1]: 1M batches
CRC_BATCH_BYTES = 16384        # of 16 KiB
CPU_THREADS = 16               # the GPU box's CPU share per GPU


def shard_partitions(n_partitions: int, rank: int, world: int) -> list[int]:
    """toppar -> GPU round-robin: partition p runs on rank p % world."""
    return [p for p in range(n_partitions) if p % world == rank]


def dist_env():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


# --------------------------------------------------------------- CRC32C leg
def bench_crc(args, rank, world):
    import torch
    import librdkafka_amd as L
    n, size = args.batches, CRC_BATCH_BYTES
    stream = torch.cuda.current_stream()
    buf = torch.empty(n * size + 64, dtype=torch.uint8, device="cuda")
    L.gen_v2_batches(buf, n, size, seed=0x5EED + rank, stream=stream)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * size
    caps = torch.full((n,), size, dtype=torch.int32, device="cuda")
    out = torch.zeros(n, dtype=torch.int32, device="cuda")

    def step():
        L.msgset_v2_crc(buf, offs, caps, out, L.V2_CRC_FINALIZE, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness gate on the timed configuration: VERIFY must be all-zero
    L.msgset_v2_crc(buf, offs, caps, out, L.V2_CRC_VERIFY, stream=stream)
    torch.cuda.synchronize()
    bad = int(out.abs().sum())
    if bad:
        raise SystemExit(f"rank {rank}: {bad} CRC verify failures")

    barrier(world)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier(world)
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    crc_len = size - 21                       # Length-4-1-4 = bytes CRC'd
    alg_bytes = n * (crc_len + 4 + 4 + 4)     # CRC range + Length read + CRC store + out
    res = {
        "wall_s": wall, "kernel_ms": kernel_ms, "bytes": n * size, "records": n,
        "alg_bytes": alg_bytes, "host_sample": (buf, n, size) if rank == 0 else None,
    }
    return res


def cpu_baseline_crc(buf, n, size, seconds=8.0):
    """The oracle's restatement of crc32c_hw (crc32c.c:255-338, SSE4.2 3-way),
    on CPU_THREADS host threads over a bounded 1 GiB sample of the batches."""
    import ctypes as C
    import numpy as np
    import oracle
    sample = min(n, 65536)
    host = buf[:sample * size].cpu().numpy()
    offs = (np.arange(sample, dtype=np.uint64) * size + 21).astype(np.uint64)
    lens = np.full(sample, size - 21, dtype=np.uint32)
    out = np.zeros(sample, dtype=np.uint32)
    lib = oracle.lib()
    passes, t0 = 0, time.perf_counter()
    while True:
        lib.or_crc32c_batches_mt(host.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                 out.ctypes.data, sample, CPU_THREADS)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gbs = passes * sample * size / el / 1e9
    hw = bool(lib.or_crc32c_hw_available())
    del C
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": CPU_THREADS, "kind": "port",
            "sample": f"{sample} x {size} B v2 batches (1 GiB), {passes} passes, "
                      f"{'SSE4.2 crc32q 3-way (crc32c_hw restated)' if hw else 'slicing-by-8 (crc32c_sw)'}"
                      f", {cpu_model()}"}


# ------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="crc", choices=["crc"])
    ap.add_argument("--batches", type=int, default=CRC_BATCHES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank, local_rank, world = dist_env()
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank)
    import librdkafka_amd as L
    if not os.path.exists(L.LIB_PATH):
        L.build()
    L.init(local_rank)

    res = bench_crc(args, rank, world)
    # whole-job time per step: max over ranks of the host clock around the
    # K synchronised steps; the HIP-event kernel time feeds the roofline
    t_max = max_over_ranks(res["wall_s"] * 1e3 / args.steps, world)
    total_bytes = res["bytes"] * world
    value = total_bytes / (t_max / 1e3) / 1e9
    if rank == 0:
        achieved = res["alg_bytes"] / (res["kernel_ms"] / 1e3) / 1e9
        line = {
            "metric": "record-batch GB/s (CRC32C+LZ4F) at 1/2/4/8 GPUs; % of HBM roofline",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 record bytes, valid v2 headers, device-generated)",
            "config": {"workload": "configs[1]: CRC32C of 1M MsgVersion 2 record batches x 16 KiB "
                                   "per GPU (writer finalize: CRC over [21,12+Length), stored BE at 17)",
                       "batches_per_gpu": args.batches, "batch_bytes": CRC_BATCH_BYTES,
                       "parallelism": f"toppar-sharded x{world}, no collective"},
            "msgs_per_s": round(args.batches * world / (t_max / 1e3), 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": "crc32c_msgset_v2_kernel<FINALIZE>",
                         "alg_bytes_per_launch": res["alg_bytes"]},
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline and world == 1:
            buf, n, size = res["host_sample"]
            line["cpu_baseline"] = cpu_baseline_crc(buf, n, size)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
