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


def launch_ranks(n: int) -> int:
    """python -m torch.distributed.run, one rank per GPU on this node, same arguments."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    return subprocess.call(cmd + sys.argv[1:])


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


# ---------------------------------------------------------------- LZ4F legs
JSON_BATCH = 1 << 20          # configs[3]/[4]: 1 MiB record batches


def _timed(fn, steps, warmup, world):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier(world)
    return wall * 1e3 / steps, ev0.elapsed_time(ev1) / steps


def json_batches(n, size=JSON_BATCH, seed=42):
    """n device-resident 1 MiB batches of JSON-like records (8 distinct MiB
    rotated: generation cost stays off the GPU clock, contents stay realistic)."""
    import torch
    import librdkafka_amd as L
    distinct = 8
    host = L.gen_json(size * distinct, seed)
    base = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    buf = torch.empty(n * size + 256, dtype=torch.uint8, device="cuda")
    for i in range(n):
        j = i % distinct
        buf[i * size:(i + 1) * size] = base[j * size:(j + 1) * size]
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * size
    lens = torch.full((n,), size, dtype=torch.int32, device="cuda")
    return buf, offs, lens


def bench_lz4c(args, rank, world, n=None, fast=False, level=0):
    """configs[2]: LZ4F compress (rd_kafka_lz4_compress semantics) of 1 MiB
    JSON batches.  fast=False: frames byte-identical to the reference's;
    fast=True: the throughput-mode encoder (reference-decodable frames, ratio
    within 5 % of the reference's)."""
    import torch
    import librdkafka_amd as L
    n = n or args.partitions // world
    src, offs, lens = json_batches(n, seed=42 + rank)
    bound = (L.lz4f_compress_bound(JSON_BATCH) + 255) // 256 * 256
    dst = torch.empty(n * bound + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(n, dtype=torch.int64, device="cuda") * bound
    olens = torch.zeros(n, dtype=torch.int32, device="cuda")
    if fast:
        comp = L.lz4f_compress_fast_batch
    else:
        comp = lambda *a: L.lz4f_compress_batch(*a, level=level)  # noqa: E731
    ms, kms = _timed(lambda: comp(src, offs, lens, dst, ooffs, olens),
                     args.steps, args.warmup, world)
    clen = int(olens.sum())
    return {"ms": ms, "kernel_ms": kms, "bytes": n * JSON_BATCH, "records": n,
            "alg_bytes": n * JSON_BATCH + clen, "ratio": n * JSON_BATCH / clen,
            "frames": (dst, ooffs, olens)}


def bench_consumer(args, rank, world, n=None):
    """configs[3]: consumer path per fetched v2 batch: CRC32C verify
    (check.crcs, rdkafka_msgset_reader.c:982-1015) then LZ4F decompress
    (rdkafka_msgset_reader.c:393-407) of 1 MiB-record batches."""
    import numpy as np
    import torch
    import librdkafka_amd as L
    from librdkafka_amd import workload as W
    n = n or args.partitions // world
    c = bench_lz4c(argparse.Namespace(steps=1, warmup=0, partitions=n * world), rank, world, n)
    frames, foffs, flens = c["frames"]
    fl = flens.cpu().numpy().astype(np.int64)
    slot = (61 + int(fl.max()) + 255) // 256 * 256
    batches = torch.zeros(n * slot + 256, dtype=torch.uint8, device="cuda")
    fo = foffs.cpu().numpy()
    hdrs = bytearray()
    for i in range(n):  # v2 header: Length, Attributes = LZ4 (3), RecordCount
        h = bytearray(W.v2_header(i, 64))
        h[8:12] = int(61 + fl[i] - 12).to_bytes(4, "big")
        h[21:23] = (3).to_bytes(2, "big")
        hdrs += h
        batches[i * slot + 61:i * slot + 61 + fl[i]] = frames[fo[i]:fo[i] + fl[i]]
    hd = torch.frombuffer(hdrs, dtype=torch.uint8).cuda().view(n, 61)
    batches[:n * slot].view(n, slot)[:, :61] = hd
    boffs = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    bcaps = torch.full((n,), slot, dtype=torch.int32, device="cuda")
    crc_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    L.msgset_v2_crc(batches, boffs, bcaps, crc_out, L.V2_CRC_FINALIZE)
    pay_offs = boffs + 61
    pay_lens = flens.clone()
    out = torch.empty(n * JSON_BATCH + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(n, dtype=torch.int64, device="cuda") * JSON_BATCH
    ocaps = torch.full((n,), JSON_BATCH, dtype=torch.int32, device="cuda")
    olens = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")

    def step():
        L.msgset_v2_crc(batches, boffs, bcaps, crc_out, L.V2_CRC_VERIFY)
        L.lz4f_decompress_batch(batches, pay_offs, pay_lens, out, ooffs, ocaps, olens, st)

    ms, kms = _timed(step, args.steps, args.warmup, world)
    assert int(crc_out.abs().sum()) == 0 and int(st.abs().sum()) == 0
    src, _, _ = json_batches(min(n, 8), seed=42 + rank)
    assert torch.equal(out[:min(n, 8) * JSON_BATCH], src[:min(n, 8) * JSON_BATCH])
    csum = int(fl.sum())
    return {"ms": ms, "kernel_ms": kms, "bytes": n * JSON_BATCH, "records": n,
            "alg_bytes": csum + (csum + 61 * n) + n * JSON_BATCH}


def tiled_messages(n_batches, per_batch, seed=42):
    """n_batches x per_batch producer messages (~100 B JSON values, keys, nulls,
    headers: workload.gen_messages) for the record writer: 16384 distinct messages
    tiled, sharing one arena; timestamps continue across tiles."""
    import numpy as np
    import torch
    from librdkafka_amd import workload as W
    base = W.gen_messages(16384, seed=seed)
    n = n_batches * per_batch
    reps = (n + 16383) // 16384
    d = {}
    for k, v in base.items():
        if k == "arena":
            d[k] = torch.from_numpy(v).cuda()
            continue
        t = np.tile(v, reps)[:n]
        if k == "ts":
            span = int(v.max() - v.min()) + 1
            t = t + np.repeat(np.arange(reps, dtype=np.int64) * span, 16384)[:n]
        if t.dtype == np.uint64:
            t = t.view(np.int64)
        elif t.dtype == np.uint32:
            t = t.view(np.int32)
        d[k] = torch.from_numpy(np.ascontiguousarray(t)).cuda()
    payload = int(np.maximum(base["key_len"], 0).sum() + np.maximum(base["val_len"], 0).sum()
                  + base["hdr_len"].sum()) * n // 16384
    return base, d, payload


def bench_serialize(args, rank, world, n=None, per_batch=9500):
    """SURVEY §8f rank 1 / configs[4] shape: linger-accumulated ~1 MiB MsgVersion 2
    batches of ~100-byte JSON records built on the device (record sizes + scan, record
    writer, CRC32C finalize) from per-message key / value / header arrays."""
    import ctypes as C
    import numpy as np
    import torch
    import librdkafka_amd as L
    n = n or args.partitions // world
    base, d, payload = tiled_messages(n, per_batch, seed=42 + rank)
    b = np.zeros(n, dtype=L.V2_BATCH_DTYPE)
    b["first_msg"] = np.arange(n) * per_batch
    b["msg_count"] = per_batch
    b["producer_id"] = -1
    b["base_sequence"] = -1
    b["producer_epoch"] = -1
    out, offs, sizes, crcs = L.msgset_v2_build(d, b, crc=True)
    m = L._Msgs(*(d[k].data_ptr() for k in ("arena", "ts", "key_off", "key_len", "val_off",
                                            "val_len", "hdr_off", "hdr_len", "hdr_cnt")))
    rec_offs = torch.empty(n * per_batch, dtype=torch.int32, device="cuda")
    max_ts = torch.empty(n, dtype=torch.int64, device="cuda")
    s = L._stream(None)
    lib = L.lib()

    def step():
        lib.rdk_hip_msgset_v2_sizes(C.byref(m), b.ctypes.data, n, L._ptr(rec_offs), L._ptr(sizes),
                                    L._ptr(max_ts), s)
        lib.rdk_hip_msgset_v2_write(C.byref(m), b.ctypes.data, n, L._ptr(rec_offs), L._ptr(sizes),
                                    L._ptr(max_ts), L._ptr(offs), L._ptr(out), L._ptr(crcs), s)

    ms, kms = _timed(step, args.steps, args.warmup, world)
    total = int(sizes.to(torch.int64).sum())
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    L.msgset_v2_crc(out, offs, sizes, st, L.V2_CRC_VERIFY)
    assert int(st.abs().sum()) == 0
    # per message: 48 B of metadata read, its payload bytes read; every batch byte written
    return {"ms": ms, "kernel_ms": kms, "bytes": total, "records": n,
            "alg_bytes": payload + 48 * n * per_batch + total,
            "host_sample": (base, per_batch)}


def bench_index(args, rank, world, n=None, per_batch=9500):
    """the consumer's record index (rd_kafka_msgset_reader_msg_v2,
    rdkafka_msgset_reader.c:715-927) over ~1 MiB MsgVersion 2 batches of ~100-byte JSON
    records (built on the device by the record writer): one row per record with offset,
    timestamp, key / value / headers positions."""
    import numpy as np
    import torch
    import librdkafka_amd as L
    n = n or args.partitions // world
    base, d, _ = tiled_messages(n, per_batch, seed=42 + rank)
    b = np.zeros(n, dtype=L.V2_BATCH_DTYPE)
    b["first_msg"] = np.arange(n) * per_batch
    b["msg_count"] = per_batch
    out, offs, sizes, _ = L.msgset_v2_build(d, b, crc=True)
    rec_offs = offs + 61
    rec_lens = sizes - 61
    row_offs = torch.arange(n, dtype=torch.int64, device="cuda") * per_batch
    caps = torch.full((n,), per_batch, dtype=torch.int32, device="cuda")
    rows = {k: torch.empty(n * per_batch, dtype=getattr(torch, t), device="cuda")
            for k, t in L.V2_ROW_FIELDS}
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    ms, kms = _timed(lambda: L.msgset_v2_index(out, offs, out, rec_offs, rec_lens, row_offs,
                                               caps, rows, cnt), args.steps, args.warmup, world)
    assert bool((cnt == per_batch).all())
    total = int(rec_lens.to(torch.int64).sum())
    return {"ms": ms, "kernel_ms": kms, "bytes": total, "records": n,
            "alg_bytes": total + 61 * n + 40 * n * per_batch,
            "host_sample": (base, per_batch)}


def bench_legacy(args, rank, world, n=None, set_bytes=1 << 20):
    """MsgVersion 1 MessageSets (~1 MiB of ~150-byte JSON messages each)
    through the consumer's per-message check.crcs (rd_kafka_msgset_reader_msg_v0_1,
    rdkafka_msgset_reader.c:566-628: message walk + CRC-32 of [16, 12+MessageSize)).
    The sets are laid out on the host, tiled, and given their CRCs by the engine's FINALIZE
    (the writer side, rdkafka_msgset_writer.c:613-641) before the timed VERIFY steps."""
    import numpy as np
    import torch
    import librdkafka_amd as L
    from librdkafka_amd import workload as W
    n = n or args.partitions // world
    base = W.gen_messages(16384, seed=42 + rank)
    one = W.msgset_v01_bytes(base, 0, 16384, magic=1, max_bytes=set_bytes)
    msgs = 0
    p = 0
    while p < len(one):
        p += 12 + int.from_bytes(one[p + 8:p + 12], "big")
        msgs += 1
    sz = len(one)
    buf = torch.from_numpy(np.frombuffer(one, dtype=np.uint8).copy()).cuda().repeat(n)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * sz
    lens = torch.full((n,), sz, dtype=torch.int32, device="cuda")
    row_offs = torch.arange(n, dtype=torch.int64, device="cuda") * msgs
    caps = torch.full((n,), msgs, dtype=torch.int32, device="cuda")
    pos = torch.empty(n * msgs, dtype=torch.int32, device="cuda")
    out = torch.empty(n * msgs, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    run = lambda mode: L.msgset_v01_crc(buf, offs, lens, row_offs, caps, pos, out, cnt, mode)
    fin_ms, fin_kms = _timed(lambda: run(L.V2_CRC_FINALIZE), 1, 0, world)
    ms, kms = _timed(lambda: run(L.V2_CRC_VERIFY), args.steps, args.warmup, world)
    assert bool((cnt == msgs).all()) and int(out.abs().sum()) == 0
    total = n * sz
    return {"ms": ms, "kernel_ms": kms, "bytes": total, "records": n,
            "alg_bytes": total + 8 * n * msgs, "finalize_kernel_ms": round(fin_kms, 3),
            "host_sample": (one, msgs)}


def cpu_baseline_legacy(one, msgs, seconds=3.0):
    """The reader walk restated (msgset_oracle.c) with the system zlib's crc32() -- the
    CRC function the reference itself calls (rdcrc32.h, WITH_ZLIB) -- one host thread."""
    import numpy as np
    import oracle
    import librdkafka_amd as L
    # fill the CRCs the way the writer does, then time VERIFY passes
    st = np.frombuffer(one, dtype=np.uint8).copy()
    pos = np.zeros(msgs, dtype=np.uint32)
    out = np.zeros(msgs, dtype=np.uint32)
    lib = oracle.lib()
    assert lib.or_msgset_v01_crc_zlib(st.ctypes.data, len(one), L.V2_CRC_FINALIZE,
                                      pos.ctypes.data, out.ctypes.data, msgs) == msgs
    passes, t0 = 0, time.perf_counter()
    while True:
        assert lib.or_msgset_v01_crc_zlib(st.ctypes.data, len(one), L.V2_CRC_VERIFY,
                                          pos.ctypes.data, out.ctypes.data, msgs) == msgs
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(passes * len(one) / el / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "reference", "sample": f"{passes} VERIFY passes over one MsgVersion 1 set "
            f"({msgs} JSON messages, {len(one)} B): reader walk restated, zlib crc32() "
            f"(the reference's CRC-32), {cpu_model()}"}


def cpu_baseline_index(base, per_batch, seconds=3.0):
    """The oracle restatement of rd_kafka_msgset_reader_msg_v2 (msgset_oracle.c), one host
    thread, over a batch of the same messages."""
    import oracle
    per_batch = min(per_batch, 16384)
    b = oracle.msgset_v2_write(base, 0, per_batch)
    rec = b[61:]
    passes, t0 = 0, time.perf_counter()
    while True:
        n, _ = oracle.msgset_v2_index(rec, 0, 0, max_rows=per_batch)
        assert n == per_batch
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(passes * len(rec) / el / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "port", "sample": f"{passes} passes over {per_batch} JSON records "
                                      f"({len(rec)} B), reader_msg_v2 restated, {cpu_model()}"}


def cpu_baseline_serialize(base, per_batch, seconds=3.0):
    """The oracle restatement of rd_kafka_msgset_writer_write_msg_v2 + header finalize +
    calc_crc_v2 (msgset_oracle.c), one host thread, batches of the same messages."""
    import oracle
    per_batch = min(per_batch, 16384)
    passes, nbytes, t0 = 0, 0, time.perf_counter()
    while True:
        nbytes += len(oracle.msgset_v2_write(base, 0, per_batch))
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(nbytes / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{passes} batches x {per_batch} JSON messages, write_msg_v2 + finalize + "
                      f"CRC32C restated, {cpu_model()}"}


def bench_producer(args, rank, world, n=None, threads=None, mode=1, slot_mib=None):
    """configs[4] (full producer pipeline), bounded: n toppars per GPU each
    hand one linger-accumulated 1 MiB batch of JSON records (61-byte v2
    header + records in host memory) to the producer front-end.  `threads`
    broker threads, each with its own rdk_hip_producer_t (pinned staging ring
    of 4 slots, one HIP stream per slot), gather the batches into
    the ring; slots run H2D -> LZ4F compress -> v2 finalize -> CRC32C -> D2H
    while the next slot fills.  Timed: first produce() to the last finished
    batch polled.  PCIe-inclusive by construction."""
    import threading
    import numpy as np
    import librdkafka_amd as L
    from librdkafka_amd import workload as W
    n = n or args.partitions // world
    # measured sweep (threads x slot MiB): 1x256 17, 2x128 20.3, 2x64 18.7, 4x64 16.2,
    # 4x128 14.7, 8x16 11.6 GB/s -- host gather + PCIe bound, more streams than
    # the 4 hardware queues serialise the compress launches
    threads = threads or int(os.environ.get("RDK_BENCH_PRODUCER_THREADS", "2"))
    slot_mib = slot_mib or int(os.environ.get("RDK_BENCH_PRODUCER_SLOT_MIB", "128"))
    distinct = 8
    recs = [L.gen_json(JSON_BATCH, 42 + rank * 97 + j) for j in range(distinct)]
    hdrs = [W.v2_header(i, 61 + JSON_BATCH) for i in range(n)]
    parts = [list(range(t, n, threads)) for t in range(threads)]
    prods = [L.Producer(0, slot_bytes=slot_mib << 20, nslots=4, mode=mode) for _ in range(threads)]
    out_bytes = [0] * threads

    def run(t, todo, count_out):
        p = prods[t]
        done = 0
        for i in todo:
            while p.produce(hdrs[i], recs[i % distinct], i) == L.E_BUSY:
                for _, (_, ln), _ in p.poll(block=True, copy=False):
                    done += 1
                    if count_out:
                        out_bytes[t] += ln
        p.flush()
        while done < len(todo):
            for _, (_, ln), _ in p.poll(block=True, copy=False):
                done += 1
                if count_out:
                    out_bytes[t] += ln

    def once(count_out=False):
        ths = [threading.Thread(target=run, args=(t, parts[t], count_out)) for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()

    once()  # warm-up: staging allocations, first-touch of pinned memory
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        once(count_out=True)
    wall = (time.perf_counter() - t0) / args.steps
    barrier(world)
    for p in prods:
        p.close()
    total = n * JSON_BATCH
    return {"ms": wall * 1e3, "kernel_ms": None, "bytes": total, "records": n,
            "out_bytes": sum(out_bytes) // args.steps, "threads": threads}


def pcie_rates(nbytes=256 << 20, reps=4):
    """Pinned host <-> device copy rates on this GPU (north_star: reported
    separately, never folded into the device-resident value)."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d.copy_(h, non_blocking=True)
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(reps):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"h2d_GBps": round(reps * nbytes / (t1 - t0) / 1e9, 1),
            "d2h_GBps": round(reps * nbytes / (t2 - t1) / 1e9, 1), "bytes": nbytes}


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


def cpu_baseline_lz4(kind, n=64, seconds=4.0, level=0):
    """Oracle restatement of rd_kafka_lz4_compress / _decompress (the
    reference's lz4 1.9.2 LZ4F path, byte-identical output) on CPU_THREADS
    host threads over n x 1 MiB JSON batches."""
    import numpy as np
    import oracle
    import librdkafka_amd as L
    data = np.frombuffer(L.gen_json(JSON_BATCH * 8, 42), dtype=np.uint8)
    src = np.concatenate([data] * (n // 8))
    offs = (np.arange(n, dtype=np.uint64) * JSON_BATCH).astype(np.uint64)
    lens = np.full(n, JSON_BATCH, dtype=np.uint32)
    bound = int(oracle.lib().or_lz4f_compress_bound(JSON_BATCH))
    cbuf = np.zeros(n * bound, dtype=np.uint8)
    coffs = (np.arange(n, dtype=np.uint64) * bound).astype(np.uint64)
    clens = np.zeros(n, dtype=np.uint32)
    lib = oracle.lib()
    comp = lambda: lib.or_lz4f_compress_batches_level_mt(  # noqa: E731
        src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, cbuf.ctypes.data,
        coffs.ctypes.data, clens.ctypes.data, level, CPU_THREADS)
    comp()
    dbuf = np.zeros(n * JSON_BATCH, dtype=np.uint8)
    dlens = np.zeros(n, dtype=np.uint32)
    dec = lambda: lib.or_lz4f_decompress_batches_mt(  # noqa: E731
        cbuf.ctypes.data, coffs.ctypes.data, clens.ctypes.data, n, dbuf.ctypes.data,
        offs.ctypes.data, lens.ctypes.data, dlens.ctypes.data, CPU_THREADS)
    fn = comp if kind == "compress" else dec
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(passes * n * JSON_BATCH / el / 1e9, 3), "unit": "GB/s",
            "cores": CPU_THREADS, "kind": "port",
            "sample": f"{n} x 1 MiB JSON batches, {passes} passes, rd_kafka_lz4_{kind} restated"
                      f"{f' at compression.level {level}' if level else ''}, "
                      f"{cpu_model()}"}


def leg_line(name, res, steps, world, cpu=None):
    d = {"GB_per_s": round(res["bytes"] * world / (res["ms"] / 1e3) / 1e9, 2),
         "ms_per_step": round(res["ms"], 3), "batches": res["records"] * world}
    if res.get("kernel_ms"):
        ach = res["alg_bytes"] / (res["kernel_ms"] / 1e3) / 1e9
        d["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}
    if "out_bytes" in res:
        d["compression_ratio"] = round(res["bytes"] / max(1, res["out_bytes"]), 3)
        d["pcie_inclusive"] = True
        d["host_threads"] = res["threads"]
    if "ratio" in res:
        d["compression_ratio"] = round(res["ratio"], 3)
    if cpu:
        d["cpu_baseline"] = cpu
    return d


def index_leg(rank, world, no_cpu):
    res = bench_index(argparse.Namespace(steps=3, warmup=1, partitions=256), rank, world)
    cpu = None if no_cpu else cpu_baseline_index(*res.pop("host_sample"))
    res.pop("host_sample", None)
    return leg_line("index", res, 3, world, cpu)


def legacy_leg(rank, world, no_cpu):
    res = bench_legacy(argparse.Namespace(steps=3, warmup=1, partitions=256), rank, world)
    cpu = None if no_cpu else cpu_baseline_legacy(*res.pop("host_sample"))
    res.pop("host_sample", None)
    d = leg_line("legacy", res, 3, world, cpu)
    d["finalize_kernel_ms"] = res["finalize_kernel_ms"]
    return d


def serialize_leg(rank, world, no_cpu):
    res = bench_serialize(argparse.Namespace(steps=3, warmup=1, partitions=256), rank, world)
    cpu = None if no_cpu else cpu_baseline_serialize(*res.pop("host_sample"))
    res.pop("host_sample", None)
    return leg_line("serialize", res, 3, world, cpu)


# HBM bytes per launch from rocprofv3 PMC passes on this kernel and workload
# (scripts/profile_crc.sh -> scripts/pmc_summary.py; FETCH_SIZE x2 on gfx950).
# Counters cannot be read in-process, so the committed summary of the same
# kernel build and batch shape is used; null when they do not match.
CRC_VARIANT = "v1" if os.environ.get("RDK_HIP_CRC_V1") else "v" + os.environ.get("RDK_HIP_CRC_V", "4")
CRC_KERNEL = ("crc32c_msgset_v2_v4_kernel<FINALIZE>" if CRC_VARIANT == "v4"
              else "crc32c_msgset_v2_kernel<%d, FINALIZE>" % int(CRC_VARIANT[1:]))
CRC_PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_crc_%s" % CRC_VARIANT, "summary.json")


def pmc_traffic(path, alg_bytes):
    try:
        with open(path) as f:
            s = json.load(f)
    except (OSError, ValueError):
        return None, None
    if int(s.get("alg_bytes_per_launch", -1)) != int(alg_bytes) or "traffic_bytes" not in s:
        return None, None
    return int(s["traffic_bytes"]), os.path.relpath(path, ROOT)


# ------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="crc",
                    choices=["crc", "lz4c", "lz4c_fast", "lz4hc", "consumer", "producer", "serialize",
                             "index", "legacy"])
    ap.add_argument("--batches", type=int, default=CRC_BATCHES)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true")
    ap.add_argument("--level", type=int, default=9, help="compression.level of --workload lz4hc")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # Started by hand with --gpus N: this parent never touches the GPU; it starts one
        # rank per GPU the way the driver does and hands back the launcher's exit code.
        sys.exit(launch_ranks(args.gpus))
    rank, local_rank, world = dist_env()
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: start it with "
                 f"--nproc-per-node {args.gpus} (or without a launcher)")
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    # one rank per GPU; with fewer GPUs than ranks (a rehearsal on one device) ranks share
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    import librdkafka_amd as L
    if not os.path.exists(L.LIB_PATH):
        raise SystemExit(f"{L.LIB_PATH} is not built: run __graft_entry__.build()")
    L.init(device)

    if args.workload != "crc":
        if args.workload == "lz4hc":
            res = bench_lz4c(args, rank, world, level=args.level)
        elif args.workload.startswith("lz4c"):
            res = bench_lz4c(args, rank, world, fast=args.workload == "lz4c_fast")
        elif args.workload == "producer":
            res = bench_producer(args, rank, world)
        elif args.workload == "serialize":
            res = bench_serialize(args, rank, world)
        elif args.workload == "index":
            res = bench_index(args, rank, world)
        elif args.workload == "legacy":
            res = bench_legacy(args, rank, world)
        else:
            res = bench_consumer(args, rank, world)
        t_max = max_over_ranks(res["ms"], world)
        if rank == 0:
            cpu = None
            if not args.no_cpu_baseline and world == 1:
                if args.workload == "serialize":
                    cpu = cpu_baseline_serialize(*res["host_sample"])
                elif args.workload == "index":
                    cpu = cpu_baseline_index(*res["host_sample"])
                elif args.workload == "legacy":
                    cpu = cpu_baseline_legacy(*res["host_sample"])
                else:
                    cpu = cpu_baseline_lz4("decompress" if args.workload == "consumer"
                                           else "compress",
                                           level=args.level if args.workload == "lz4hc" else 0)
            res.pop("host_sample", None)
            res["ms"] = t_max
            print(json.dumps({"workload": args.workload, "n_gpus": world, "steps": args.steps,
                              **leg_line(args.workload, res, args.steps, world, cpu)}), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

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
                         "traffic": None, "kernel": CRC_KERNEL,
                         "alg_bytes_per_launch": res["alg_bytes"]},
            "cpu_baseline": None,
        }
        traffic, src = pmc_traffic(CRC_PMC_SUMMARY, res["alg_bytes"])
        if traffic is not None:
            line["roofline"]["traffic"] = traffic
            line["roofline"]["traffic_source"] = src
        if not args.no_cpu_baseline and world == 1:
            buf, n, size = res["host_sample"]
            line["cpu_baseline"] = cpu_baseline_crc(buf, n, size)
        del res
        line["pcie_pinned"] = pcie_rates()
        if not args.no_legs and world == 1:
            # the LZ4F legs of the same path (configs[2], configs[3]) at 256 x 1 MiB
            sub = argparse.Namespace(steps=3, warmup=1, partitions=256)
            cpu = (lambda k: None) if args.no_cpu_baseline else cpu_baseline_lz4
            line["legs"] = {
                "lz4f_compress_1MiB_json": leg_line("lz4c", bench_lz4c(sub, rank, world), 3, 1,
                                                    cpu("compress")),
                "lz4f_compress_fast_1MiB_json": leg_line(
                    "lz4c_fast", bench_lz4c(sub, rank, world, fast=True), 3, 1, cpu("compress")),
                # LZ4HC at its default level (LZ4HC_CLEVEL_DEFAULT = 9), 256 x 1 MiB
                "lz4hc_compress_level9_1MiB_json": leg_line(
                    "lz4hc", bench_lz4c(argparse.Namespace(steps=3, warmup=1, partitions=256),
                                        rank, world, level=9), 3, 1,
                    None if args.no_cpu_baseline else cpu_baseline_lz4("compress", level=9)),
                "consumer_crc_verify_lz4f_decompress_1MiB": leg_line(
                    "consumer", bench_consumer(argparse.Namespace(steps=3, warmup=1, partitions=1024),
                                               rank, world), 3, 1, cpu("decompress")),
                "v2_record_serialize_1MiB_json": serialize_leg(rank, world, args.no_cpu_baseline),
                "v2_record_index_1MiB_json": index_leg(rank, world, args.no_cpu_baseline),
                "v1_msgset_crc32_verify_1MiB_json": legacy_leg(rank, world, args.no_cpu_baseline),
                "producer_pipeline_1MiB_json_pcie": leg_line(
                    "producer", bench_producer(argparse.Namespace(steps=2, warmup=1, partitions=512),
                                               rank, world), 2, 1, cpu("compress")),
            }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
