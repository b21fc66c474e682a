#!/usr/bin/env python3
"""bench.py -- librdkafka record-batch engine on MI355X.

Headline = the metric "record-batch GB/s (CRC32C+LZ4F)": the writer's
finalize of device-resident MsgVersion 2 MessageSets (rd_kafka_msgset_writer_finalize,
rdkafka_msgset_writer.c:1335: LZ4F compress :1128-1221 with frames byte-identical to
rd_kafka_lz4_compress, header finalize :1251-1295, CRC32C :1229-1246) over `--partitions`
toppars per GPU, each with one linger-accumulated 1 MiB batch of JSON records
(configs[2] input, configs[4] shape).  One step = one rdk_hip_msgset_v2_finalize call over
all batches; value = uncompressed record bytes per second.  configs[1] (CRC32C only over
1M x 16 KiB batches) and the other configs are `legs` of the same JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ...]

--gpus N started by hand launches N ranks itself (torch.distributed.run); under a launcher
it checks WORLD_SIZE.  Batches shard by topic-partition across GPUs with no data-path
collective (weak scaling); gloo carries only the barrier and the max-over-ranks time.
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


def source_hash() -> str:
    """sha256 over the kernel sources the library is built from: ties a profile summary
    under profiles/ to the build that bench.py is timing."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "librdkafka_amd", "csrc")
    for f in sorted(os.listdir(d)) + ["../Makefile"]:
        with open(os.path.join(d, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


PROFILE_DIR = os.path.join(ROOT, "profiles", "r03")
SIMDS = 1024                   # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9               # MI355X peak engine clock (MI355X_MICROARCH.md)


def profile_summary(leg: str, alg_bytes: int, kernel_ms: float):
    """(traffic_bytes, note) from profiles/r03/<leg>.json -- the rocprofv3 summary of this leg
    (scripts/profile_r3.sh) -- only when it was taken from the same kernel sources and the
    same algorithmic bytes; its kernel-trace average must agree with the HIP-event time.
    With an SQ_INSTS_VALU pass in the summary the note carries `issue`: the vector
    instructions per launch and the time the chip needs just to issue them (one wave64
    vector instruction per SIMD per 4 cycles), the ceiling that binds the LZ4 / snappy legs
    long before HBM does."""
    path = os.path.join(PROFILE_DIR, leg + ".json")
    try:
        with open(path) as f:
            p = json.load(f)
    except (OSError, ValueError):
        return None, {"profile": None}
    note = {"profile": os.path.relpath(path, ROOT), "profile_source_hash": p.get("source_hash"),
            "profile_kernel_ms": round(p["avg_ns"] / 1e6, 4) if p.get("avg_ns") else None}
    if p.get("source_hash") != source_hash():
        note["profile_stale"] = "kernel sources changed since the profile was taken"
        return None, note
    if int(p.get("alg_bytes_per_launch", -1)) != int(alg_bytes):
        note["profile_stale"] = "different workload (algorithmic bytes differ)"
        return None, note
    if p.get("avg_ns") and kernel_ms:
        note["profile_vs_events"] = round(p["avg_ns"] / 1e6 / kernel_ms, 4)
    if p.get("valu_insts"):
        floor_ms = p["valu_insts"] * 4.0 / (SIMDS * CLOCK_HZ) * 1e3
        note["issue"] = {"valu_insts_per_launch": int(p["valu_insts"]),
                         "valu_per_alg_byte": round(p["valu_insts"] * 64.0 / alg_bytes, 3),
                         "lane_ops_per_alg_byte": round(p["valu_insts"] * 64.0 / alg_bytes, 3),
                         "issue_floor_ms": round(floor_ms, 4),
                         "frac_of_issue_ceiling": round(floor_ms / kernel_ms, 4) if kernel_ms else None,
                         "note": "SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz)"}
        note["issue"].pop("lane_ops_per_alg_byte")
        note["issue"]["valu_wave_insts_per_64_alg_bytes"] = note["issue"].pop("valu_per_alg_byte")
    return (int(p["traffic_bytes"]) if "traffic_bytes" in p else None), note


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


DISTINCT_BYTES = 512 << 20   # distinct JSON bytes behind every leg's batches
_JSON_STREAM = {}


def _json_stream(seed):
    """(host bytes, device tensor) of DISTINCT_BYTES of JSON-like records, generated once per
    process: 64 pieces of 8 MiB, each from its own seed, on 8 host threads (the generator is a
    sequential LCG at ~160 MB/s; the call releases the interpreter lock)."""
    if seed not in _JSON_STREAM:
        import warnings
        from concurrent.futures import ThreadPoolExecutor
        import numpy as np
        import torch
        import librdkafka_amd as L
        piece = 8 << 20
        with ThreadPoolExecutor(8) as ex:
            parts = list(ex.map(lambda k: L.gen_json(piece, seed + 1000003 * k),
                                range(DISTINCT_BYTES // piece)))
        host = b"".join(parts)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # (a read-only host array: it is only copied from)
            dev = torch.from_numpy(np.frombuffer(host, dtype=np.uint8)).cuda()
        _JSON_STREAM.clear()  # one stream resident at a time
        _JSON_STREAM[seed] = (host, dev)
    return _JSON_STREAM[seed]


def _json_base(size, seed):
    """(host bytes, device tensor [distinct, size], distinct): the stream cut into batches of
    `size` bytes; 512 x 1 MiB batches are all different, more than that rotate."""
    host, dev = _json_stream(seed)
    distinct = DISTINCT_BYTES // size
    return host, dev[:distinct * size].view(distinct, size), distinct


def json_record_count(host, size, n):
    """JSON records (lines) that end in n batches of `size` bytes cut from `host` in rotation:
    the messages the batches carry."""
    distinct = len(host) // size
    per = [host[j * size:(j + 1) * size].count(b"\n") for j in range(distinct)]
    return sum(per) * (n // distinct) + sum(per[:n % distinct])


def json_batches(n, size=JSON_BATCH, seed=42):
    """n device-resident batches of `size` bytes of JSON-like records, cut from 512 MiB of
    distinct records (rotated beyond that)."""
    import torch
    host, base, distinct = _json_base(size, seed)
    buf = torch.empty(n * size + 256, dtype=torch.uint8, device="cuda")
    idx = torch.arange(n, device="cuda") % distinct
    for lo in range(0, n, 4096):  # (in slices: the gather's temporary stays small)
        hi = min(n, lo + 4096)
        buf[lo * size:hi * size].view(hi - lo, size).copy_(base[idx[lo:hi]])
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * size
    lens = torch.full((n,), size, dtype=torch.int32, device="cuda")
    return buf, offs, lens


def json_msgsets(n, size=JSON_BATCH, seed=42):
    """n device-resident MessageSets as the writer leaves them before finalize: a 61-byte v2
    header directly followed by `size` bytes of JSON records (512 MiB of distinct records).
    Returns (buffer, record offsets, record lengths, records carried)."""
    import torch
    from librdkafka_amd import workload as W
    host, base, distinct = _json_base(size, seed)
    stride = (61 + size + 255) // 256 * 256
    buf = torch.zeros(n * stride + 256, dtype=torch.uint8, device="cuda")
    hdrs = torch.frombuffer(bytearray(b"".join(W.v2_header(i, 61 + size) for i in range(n))),
                            dtype=torch.uint8).cuda().view(n, 61)
    v = buf[:n * stride].view(n, stride)
    v[:, :61] = hdrs
    idx = torch.arange(n, device="cuda") % distinct
    for lo in range(0, n, 4096):
        hi = min(n, lo + 4096)
        v[lo:hi, 61:61 + size] = base[idx[lo:hi]]
    rec_offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride + 61
    rec_lens = torch.full((n,), size, dtype=torch.int32, device="cuda")
    return buf, rec_offs, rec_lens, json_record_count(host, size, n)


def bench_finalize(args, rank, world, n=None, mode=0, size=JSON_BATCH):
    """The headline step: rdk_hip_msgset_v2_finalize (LZ4F compress + v2 header finalize +
    CRC32C finalize, rdkafka_msgset_writer.c:1335) over n device-resident MessageSets of
    `size` record bytes.  mode 1 = the throughput compressor (reference-decodable frames,
    ratio within 5 % of the reference's: north_star's bar), 0 = frames byte-identical to
    rd_kafka_lz4_compress.  Its HIP-event time feeds the roofline.  The finished batches
    are checked on the device: CRC VERIFY all zero, every frame decompressed by the engine
    equals its records."""
    import torch
    import librdkafka_amd as L
    n = n or args.partitions
    src, rec_offs, rec_lens, nrecords = json_msgsets(n, size, seed=42 + rank)
    cap = (61 + L.lz4f_compress_bound(size) + 255) // 256 * 256
    dst = torch.empty(n * cap + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * cap
    out_caps = torch.full((n,), cap, dtype=torch.int32, device="cuda")
    flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))

    def step():
        L.msgset_v2_finalize(src, rec_offs, rec_lens, dst, out_offs, out_caps, flens, blens, crcs,
                             mode=mode)

    ms, kms = _timed(step, args.steps, args.warmup, world)
    frame_offs = out_offs + 61
    # correctness gate on the timed configuration
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    L.msgset_v2_crc(dst, out_offs, out_caps, st, L.V2_CRC_VERIFY)
    if int(st.abs().sum()):
        raise SystemExit(f"rank {rank}: CRC verify failures in the finished batches")
    dslot = (size + 255) // 256 * 256
    dec = torch.empty(n * dslot + 256, dtype=torch.uint8, device="cuda")
    doffs = torch.arange(n, dtype=torch.int64, device="cuda") * dslot
    dcaps = torch.full((n,), dslot, dtype=torch.int32, device="cuda")
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    L.lz4f_decompress_batch(dst, frame_offs, flens, dec, doffs, dcaps, dl, st)
    stride = (61 + size + 255) // 256 * 256
    recs = src[:n * stride].view(n, stride)[:, 61:61 + size]
    if int(st.abs().sum()) or not bool((dl == size).all()) or \
            not torch.equal(dec[:n * dslot].view(n, dslot)[:, :size], recs):
        raise SystemExit(f"rank {rank}: finished frames do not decompress to their records")
    if not bool((blens == flens + 61).all()):
        raise SystemExit(f"rank {rank}: a JSON batch was left uncompressed")
    clen = int(flens.to(torch.int64).sum())
    nbytes = n * size
    return {"ms": ms, "kernel_ms": kms, "bytes": nbytes, "records": n, "messages": nrecords,
            # step: records read + frame written, header read + written
            "alg_bytes": nbytes + clen + 2 * 61 * n, "ratio": nbytes / clen}


def bench_lz4c(args, rank, world, n=None, fast=False, level=0, size=JSON_BATCH, units=False):
    """configs[2]: LZ4F compress (rd_kafka_lz4_compress semantics) of JSON batches.
    fast=False: frames byte-identical to the reference's; fast=True: the throughput-mode
    encoder (reference-decodable frames, ratio within 5 % of the reference's); units=True:
    the same contract on the workgroup-per-block engine (rdk_hip_lz4f_compress_units)."""
    import torch
    import librdkafka_amd as L
    n = n or args.partitions
    src, offs, lens = json_batches(n, size, seed=42 + rank)
    bound = (L.lz4f_compress_bound(size) + 255) // 256 * 256
    dst = torch.empty(n * bound + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(n, dtype=torch.int64, device="cuda") * bound
    olens = torch.zeros(n, dtype=torch.int32, device="cuda")
    if units:
        comp = L.lz4f_compress_units_batch
    elif fast:
        comp = L.lz4f_compress_fast_batch
    else:
        comp = lambda *a: L.lz4f_compress_batch(*a, level=level)  # noqa: E731
    ms, kms = _timed(lambda: comp(src, offs, lens, dst, ooffs, olens),
                     args.steps, args.warmup, world)
    clen = int(olens.sum())
    return {"ms": ms, "kernel_ms": kms, "bytes": n * size, "records": n,
            "alg_bytes": n * size + clen, "ratio": n * size / clen,
            "frames": (dst, ooffs, olens)}


def bench_snappy(args, rank, world, n=None, decompress=False):
    """snappy (compression.codec=snappy) on 1 MiB JSON batches: the codec behind
    rd_kafka_msgset_writer_compress_snappy (rdkafka_msgset_writer.c:1041) or the reader's
    snappy case (rdkafka_msgset_reader.c:299-390).  Streams are the reference's
    compress_fragment parse; the decompress leg decodes them and compares."""
    import torch
    import librdkafka_amd as L
    n = n or args.partitions
    src, offs, lens = json_batches(n, seed=42 + rank)
    bound = (L.snappy_max_compressed_length(JSON_BATCH) + 255) // 256 * 256
    dst = torch.empty(n * bound + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(n, dtype=torch.int64, device="cuda") * bound
    olens = torch.zeros(n, dtype=torch.int32, device="cuda")
    comp = lambda: L.snappy_compress_batch(src, offs, lens, dst, ooffs, olens)  # noqa: E731
    if not decompress:
        ms, kms = _timed(comp, args.steps, args.warmup, world)
        clen = int(olens.sum())
        return {"ms": ms, "kernel_ms": kms, "bytes": n * JSON_BATCH, "records": n,
                "alg_bytes": n * JSON_BATCH + clen, "ratio": n * JSON_BATCH / clen}
    comp()
    clen = int(olens.sum())
    out = torch.empty(n * JSON_BATCH + 256, dtype=torch.uint8, device="cuda")
    caps = torch.full((n,), JSON_BATCH, dtype=torch.int32, device="cuda")
    dlens = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    ms, kms = _timed(lambda: L.snappy_uncompress_batch(dst, ooffs, olens, out, offs, caps, dlens, st),
                     args.steps, args.warmup, world)
    assert int(st.abs().sum()) == 0 and torch.equal(out[:n * JSON_BATCH], src[:n * JSON_BATCH])
    return {"ms": ms, "kernel_ms": kms, "bytes": n * JSON_BATCH, "records": n,
            "alg_bytes": n * JSON_BATCH + clen}


def cpu_baseline_snappy(kind, n=64, seconds=4.0):
    """The oracle's restatement of snappy.c (snappy.c itself needs the generated config.h)
    on CPU_THREADS host threads over n x 1 MiB JSON batches."""
    import numpy as np
    import oracle
    import librdkafka_amd as L
    lib = oracle.lib()
    data = np.frombuffer(L.gen_json(JSON_BATCH * 8, 42), dtype=np.uint8)
    src = np.concatenate([data] * (n // 8))
    offs = (np.arange(n, dtype=np.uint64) * JSON_BATCH).astype(np.uint64)
    lens = np.full(n, JSON_BATCH, dtype=np.uint32)
    bound = int(lib.or_snappy_max_compressed_length(JSON_BATCH))
    cbuf = np.zeros(n * bound, dtype=np.uint8)
    coffs = (np.arange(n, dtype=np.uint64) * bound).astype(np.uint64)
    clens = np.zeros(n, dtype=np.uint32)
    comp = lambda: lib.or_snappy_batches_mt(  # noqa: E731
        src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, cbuf.ctypes.data,
        coffs.ctypes.data, clens.ctypes.data, 0, CPU_THREADS)
    assert comp() == 0
    dbuf = np.zeros(n * JSON_BATCH, dtype=np.uint8)
    dlens = np.zeros(n, dtype=np.uint32)
    dec = lambda: lib.or_snappy_batches_mt(  # noqa: E731
        cbuf.ctypes.data, coffs.ctypes.data, clens.ctypes.data, n, dbuf.ctypes.data,
        offs.ctypes.data, dlens.ctypes.data, 1, CPU_THREADS)
    fn = comp if kind == "compress" else dec
    passes, t0 = 0, time.perf_counter()
    while True:
        assert fn() == 0
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(passes * n * JSON_BATCH / el / 1e9, 3), "unit": "GB/s",
            "cores": CPU_THREADS, "kind": "port",
            "sample": f"{n} x 1 MiB JSON batches, {passes} passes, snappy.c's "
                      f"{'compress_fragment' if kind == 'compress' else 'decoder'} restated, {cpu_model()}"}


def bench_consumer(args, rank, world, n=None, size=JSON_BATCH):
    """configs[3]: consumer path per fetched v2 batch: CRC32C verify
    (check.crcs, rdkafka_msgset_reader.c:982-1015) then LZ4F decompress
    (rdkafka_msgset_reader.c:393-407) of batches of `size` record bytes (frames made by the
    exact compressor: byte-identical to the reference's)."""
    import numpy as np
    import torch
    import librdkafka_amd as L
    from librdkafka_amd import workload as W
    n = n or args.partitions
    c = bench_lz4c(argparse.Namespace(steps=1, warmup=0, partitions=n), rank, world, n, size=size)
    frames, foffs, flens = c["frames"]
    fl = flens.cpu().numpy().astype(np.int64)
    slot = (61 + int(fl.max()) + 255) // 256 * 256
    bound = int(foffs[1] - foffs[0]) if n > 1 else slot
    batches = torch.zeros(n * slot + 256, dtype=torch.uint8, device="cuda")
    hdrs = bytearray()
    for i in range(n):  # v2 header: Length, Attributes = LZ4 (3), RecordCount
        h = bytearray(W.v2_header(i, 64))
        h[8:12] = int(61 + fl[i] - 12).to_bytes(4, "big")
        h[21:23] = (3).to_bytes(2, "big")
        hdrs += h
    keep = min(bound, slot - 61)  # every frame is shorter than both
    fv = frames[:n * bound].view(n, bound)[:, :keep]
    bv = batches[:n * slot].view(n, slot)
    for lo in range(0, n, 4096):
        hi = min(n, lo + 4096)
        bv[lo:hi, 61:61 + keep] = fv[lo:hi]
    hd = torch.frombuffer(hdrs, dtype=torch.uint8).cuda().view(n, 61)
    bv[:, :61] = hd
    boffs = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    bcaps = torch.full((n,), slot, dtype=torch.int32, device="cuda")
    crc_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    L.msgset_v2_crc(batches, boffs, bcaps, crc_out, L.V2_CRC_FINALIZE)
    pay_offs = boffs + 61
    pay_lens = flens.clone()
    dslot = (size + 255) // 256 * 256
    out = torch.empty(n * dslot + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(n, dtype=torch.int64, device="cuda") * dslot
    ocaps = torch.full((n,), dslot, dtype=torch.int32, device="cuda")
    olens = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")

    def step():
        L.msgset_v2_crc(batches, boffs, bcaps, crc_out, L.V2_CRC_VERIFY)
        L.lz4f_decompress_batch(batches, pay_offs, pay_lens, out, ooffs, ocaps, olens, st)

    ms, kms = _timed(step, args.steps, args.warmup, world)
    assert int(crc_out.abs().sum()) == 0 and int(st.abs().sum()) == 0 and bool((olens == size).all())
    k = min(n, 8)
    src, _, _ = json_batches(k, size, seed=42 + rank)
    assert torch.equal(out[:k * dslot].view(k, dslot)[:, :size], src[:k * size].view(k, size))
    csum = int(fl.sum())
    return {"ms": ms, "kernel_ms": kms, "bytes": n * size, "records": n,
            "alg_bytes": csum + (csum + 61 * n) + n * size}


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
    """The record writer (rdkafka_msgset_writer.c:652-754), configs[4] shape: linger-accumulated ~1 MiB MsgVersion 2
    batches of ~100-byte JSON records built on the device (record sizes + scan, record
    writer, CRC32C finalize) from per-message key / value / header arrays."""
    import ctypes as C
    import numpy as np
    import torch
    import librdkafka_amd as L
    n = n or args.partitions
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
    """The consumer's record index (rd_kafka_msgset_reader_msg_v2,
    rdkafka_msgset_reader.c:715-927) over ~1 MiB MsgVersion 2 batches of ~100-byte JSON
    records (built on the device by the record writer): one row per record with offset,
    timestamp, key / value / headers positions."""
    import numpy as np
    import torch
    import librdkafka_amd as L
    n = n or args.partitions
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


def bench_chain(args, rank, world, n=None, per_batch=9500, with_fast=True):
    """Both directions whole, every stage on the device and chained on one stream as a
    broker thread would chain them, over ~1 MiB batches of ~100-byte JSON messages:
      writer: record sizes + record writer (rdkafka_msgset_writer.c:652-754, :1117-1207)
              -> LZ4F compress + header finalize + CRC32C (rdkafka_msgset_writer.c:1229-1335)
      reader: CRC32C verify (rdkafka_msgset_reader.c:982-1015) -> LZ4F decompress
              (rdkafka_msgset_reader.c:393-407) -> record index (rdkafka_msgset_reader.c:715-927)
    Returns (writer result, reader result); the reader runs on the writer's batches, and the
    rows it ends with are compared with the messages the writer began with."""
    import ctypes as C
    import numpy as np
    import torch
    import librdkafka_amd as L
    n = n or args.partitions
    base, d, payload = tiled_messages(n, per_batch, seed=42 + rank)
    b = np.zeros(n, dtype=L.V2_BATCH_DTYPE)
    b["first_msg"] = np.arange(n) * per_batch
    b["msg_count"] = per_batch
    b["producer_id"] = -1
    b["base_sequence"] = -1
    b["producer_epoch"] = -1
    sets, offs, sizes, _ = L.msgset_v2_build(d, b, crc=False)
    m = L._Msgs(*(d[k].data_ptr() for k in ("arena", "ts", "key_off", "key_len", "val_off",
                                            "val_len", "hdr_off", "hdr_len", "hdr_cnt")))
    rec_pos = torch.empty(n * per_batch, dtype=torch.int32, device="cuda")
    max_ts = torch.empty(n, dtype=torch.int64, device="cuda")
    rec_offs, rec_lens = offs + 61, sizes - 61
    rl = rec_lens.cpu().numpy().astype(np.int64)
    cap = (61 + L.lz4f_compress_bound(int(rl.max())) + 255) // 256 * 256
    out = torch.empty(n * cap + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * cap
    out_caps = torch.full((n,), cap, dtype=torch.int32, device="cuda")
    flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    s = L._stream(None)
    lib = L.lib()

    def write_step(mode=L.PRODUCER_EXACT):
        lib.rdk_hip_msgset_v2_sizes(C.byref(m), b.ctypes.data, n, L._ptr(rec_pos), L._ptr(sizes),
                                    L._ptr(max_ts), s)
        lib.rdk_hip_msgset_v2_write(C.byref(m), b.ctypes.data, n, L._ptr(rec_pos), L._ptr(sizes),
                                    L._ptr(max_ts), L._ptr(offs), L._ptr(sets), None, s)
        L.msgset_v2_finalize(sets, rec_offs, rec_lens, out, out_offs, out_caps, flens, blens, crcs,
                             mode=mode)

    total = int(rl.sum())
    fast = None
    if with_fast:  # (not when the workload runs alone: a profile of the leg then holds its kernels only)
        # the same chain with the throughput compressor (reported beside the leg, which is the
        # byte-identical one); its batches are CRC-verified and decoded back before the exact
        # run overwrites them
        fms, fkms = _timed(lambda: write_step(L.PRODUCER_FAST), args.steps, args.warmup, world)
        if not bool((blens == flens + 61).all()):
            raise SystemExit(f"rank {rank}: a JSON batch was left uncompressed (throughput compressor)")
        fclen = int(flens.to(torch.int64).sum())
        fdec = torch.empty(n * ((int(rl.max()) + 255) // 256 * 256) + 256, dtype=torch.uint8, device="cuda")
        fdo = torch.arange(n, dtype=torch.int64, device="cuda") * ((int(rl.max()) + 255) // 256 * 256)
        fdc = torch.full((n,), (int(rl.max()) + 255) // 256 * 256, dtype=torch.int32, device="cuda")
        fdl, fst, fvst = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
        L.msgset_v2_crc(out, out_offs, out_caps, fvst, L.V2_CRC_VERIFY)
        L.lz4f_decompress_batch(out, out_offs + 61, flens, fdec, fdo, fdc, fdl, fst)
        if int(fvst.abs().sum()) or int(fst.abs().sum()) or not bool((fdl == rec_lens).all()):
            raise SystemExit(f"rank {rank}: the throughput compressor's batches do not verify / decode")
        i0 = int(rec_offs[0])
        if not torch.equal(fdec[:int(rl[0])], sets[i0:i0 + int(rl[0])]):
            raise SystemExit(f"rank {rank}: the throughput compressor's first batch decodes to other records")
        del fdec
        fast = {"GB_per_s": round(total * world / (max_over_ranks(fms, world) / 1e3) / 1e9, 2),
                "ms_per_step": round(fms, 4), "kernel_ms": round(fkms, 4), "ratio": round(total / fclen, 3)}

    wms, wkms = _timed(write_step, args.steps, args.warmup, world)
    if not bool((blens == flens + 61).all()):
        raise SystemExit(f"rank {rank}: a JSON batch was left uncompressed")
    clen = int(flens.to(torch.int64).sum())
    writer = {"ms": wms, "kernel_ms": wkms, "bytes": total, "records": n,
              # messages read (metadata + payload), MessageSets written, then read by the
              # compressor, frames written, headers read + written
              "alg_bytes": payload + 48 * n * per_batch + 2 * (total + 61 * n) + clen + 2 * 61 * n,
              "ratio": total / clen, "fast": fast}
    # ---- reader over the finished batches
    dslot = (int(rl.max()) + 255) // 256 * 256
    dec = torch.empty(n * dslot + 256, dtype=torch.uint8, device="cuda")
    doffs = torch.arange(n, dtype=torch.int64, device="cuda") * dslot
    dcaps = torch.full((n,), dslot, dtype=torch.int32, device="cuda")
    dl, st, vst, cnt = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(4))
    pay_offs = out_offs + 61
    row_offs = torch.arange(n, dtype=torch.int64, device="cuda") * per_batch
    row_caps = torch.full((n,), per_batch, dtype=torch.int32, device="cuda")
    rows = {k: torch.empty(n * per_batch, dtype=getattr(torch, t), device="cuda")
            for k, t in L.V2_ROW_FIELDS}

    def read_step():
        L.msgset_v2_crc(out, out_offs, out_caps, vst, L.V2_CRC_VERIFY)
        L.lz4f_decompress_batch(out, pay_offs, flens, dec, doffs, dcaps, dl, st)
        L.msgset_v2_index(out, out_offs, dec, doffs, dl, row_offs, row_caps, rows, cnt)

    rms, rkms = _timed(read_step, args.steps, args.warmup, world)
    if int(vst.abs().sum()) or int(st.abs().sum()) or not bool((dl == rec_lens).all()) or \
            not bool((cnt == per_batch).all()):
        raise SystemExit(f"rank {rank}: the reader rejected the writer's batches")
    # the rows against the messages: timestamps and value lengths of every record, value
    # bytes of the first batch
    if not torch.equal(rows["timestamp"], d["ts"]) or not torch.equal(rows["val_len"], d["val_len"]):
        raise SystemExit(f"rank {rank}: rows differ from the messages")
    arena = base["arena"]
    r0 = {k: rows[k][:per_batch].cpu().numpy() for k in ("val_off", "val_len")}
    d0 = dec[:dslot].cpu().numpy()
    for j in range(0, per_batch, 97):
        ln = int(r0["val_len"][j])
        if ln > 0:
            o = int(base["val_off"][j])
            if bytes(d0[int(r0["val_off"][j]):int(r0["val_off"][j]) + ln]) != bytes(arena[o:o + ln]):
                raise SystemExit(f"rank {rank}: row {j} value bytes differ from the message")
    reader = {"ms": rms, "kernel_ms": rkms, "bytes": total, "records": n,
              # batch read for the CRC, frame read + records written by the decoder, records
              # + header read and 40 B of row written per record by the index
              "alg_bytes": (clen + 61 * n) + clen + total + total + 61 * n + 40 * n * per_batch}
    return writer, reader


def perf_tool_messages(msgs):
    """configs[0]'s producer input: `rdkafka_performance -P -s 100 -c msgs -z lz4`
    (examples/rdkafka_performance.c:798, :1318-1325), cut into MessageSets by write_msgq's
    rule (rdkafka_msgset_writer.c:859-863, batch.num.messages 10000, message.max.bytes
    1000000).  The messages are uniform, so the rule is run on the first MessageSet and the
    others take its count."""
    from librdkafka_amd import workload as W
    m = W.gen_perf_messages(msgs)
    head = {k: (v if k == "arena" else v[:12000]) for k, v in m.items()}
    per = W.perf_batches(head)[0][1]
    spec = [(f, min(per, msgs - f)) for f in range(0, msgs, per)]
    return m, spec


def bench_perf_tool(args, rank, world, msgs=1000000, with_fast=True):
    """configs[0]'s workload through the engine, device-resident: 1M x 100-byte messages of
    the perf tool's payload -> record sizes + record writer (rdkafka_msgset_writer.c:652-754)
    -> rdk_hip_msgset_v2_finalize with frames byte-identical to rd_kafka_lz4_compress ->
    finished batches.  One step = all ~110 MessageSets (one broker thread's worth each).
    Gate: CRC VERIFY, decompress, record index: every message comes back."""
    import ctypes as C
    import numpy as np
    import torch
    import librdkafka_amd as L
    m, spec = perf_tool_messages(msgs)
    n = len(spec)
    d = {}
    for k, v in m.items():
        a = v.view(np.int64) if v.dtype == np.uint64 else (v.view(np.int32) if v.dtype == np.uint32 else v)
        d[k] = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    b = np.zeros(n, dtype=L.V2_BATCH_DTYPE)
    for i, (first, cnt) in enumerate(spec):
        b[i] = (first, cnt, -1, -1, -1, 0)
    sets, offs, sizes, _ = L.msgset_v2_build(d, b, crc=False)
    mm = L._Msgs(*(d[k].data_ptr() for k in ("arena", "ts", "key_off", "key_len", "val_off",
                                             "val_len", "hdr_off", "hdr_len", "hdr_cnt")))
    rec_pos = torch.empty(msgs, dtype=torch.int32, device="cuda")
    max_ts = torch.empty(n, dtype=torch.int64, device="cuda")
    rec_offs, rec_lens = offs + 61, sizes - 61
    rl = rec_lens.cpu().numpy().astype(np.int64)
    cap = (61 + L.lz4f_compress_bound(int(rl.max())) + 255) // 256 * 256
    out = torch.empty(n * cap + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * cap
    out_caps = torch.full((n,), cap, dtype=torch.int32, device="cuda")
    flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    s = L._stream(None)
    lib = L.lib()

    def step(mode=L.PRODUCER_EXACT):
        lib.rdk_hip_msgset_v2_sizes(C.byref(mm), b.ctypes.data, n, L._ptr(rec_pos), L._ptr(sizes),
                                    L._ptr(max_ts), s)
        lib.rdk_hip_msgset_v2_write(C.byref(mm), b.ctypes.data, n, L._ptr(rec_pos), L._ptr(sizes),
                                    L._ptr(max_ts), L._ptr(offs), L._ptr(sets), None, s)
        L.msgset_v2_finalize(sets, rec_offs, rec_lens, out, out_offs, out_caps, flens, blens, crcs,
                             mode=mode)

    st, dl, ds, cnt = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(4))
    dslot = (int(rl.max()) + 255) // 256 * 256
    dec = torch.empty(n * dslot + 256, dtype=torch.uint8, device="cuda")
    doffs = torch.arange(n, dtype=torch.int64, device="cuda") * dslot
    dcaps = torch.full((n,), dslot, dtype=torch.int32, device="cuda")
    fast = None
    if with_fast:  # (not when the workload runs alone: a profile of the leg then holds its kernels only)
        # the same steps with the throughput compressor, reported beside the leg (which is the
        # byte-identical one): its batches are verified and decoded back to the records
        fms, fkms = _timed(lambda: step(L.PRODUCER_FAST), args.steps, args.warmup, world)
        L.msgset_v2_crc(out, out_offs, out_caps, st, L.V2_CRC_VERIFY)
        L.lz4f_decompress_batch(out, out_offs + 61, flens, dec, doffs, dcaps, dl, ds)
        i0, l0 = int(rec_offs[0]), int(rl[0])
        if int(st.abs().sum()) or int(ds.abs().sum()) or not bool((dl == rec_lens).all()) or \
                not bool((blens == flens + 61).all()) or not torch.equal(dec[:l0], sets[i0:i0 + l0]):
            raise SystemExit(f"rank {rank}: the throughput compressor's perf-tool batches do not verify / decode")
        fast = {"msgs_per_s": round(msgs * world / (max_over_ranks(fms, world) / 1e3), 1),
                "ms_per_step": round(fms, 4), "kernel_ms": round(fkms, 4),
                "ratio": round(int(rl.sum()) / int(flens.to(torch.int64).sum()), 3)}

    ms, kms = _timed(step, args.steps, args.warmup, world)
    # gate: the reader side hands every message back
    L.msgset_v2_crc(out, out_offs, out_caps, st, L.V2_CRC_VERIFY)
    L.lz4f_decompress_batch(out, out_offs + 61, flens, dec, doffs, dcaps, dl, ds)
    row_offs = torch.tensor(np.asarray([f for f, _ in spec], np.int64), device="cuda")
    row_caps = torch.tensor(np.asarray([c for _, c in spec], np.int32), device="cuda")
    rows = {k: torch.empty(msgs, dtype=getattr(torch, t), device="cuda") for k, t in L.V2_ROW_FIELDS}
    L.msgset_v2_index(out, out_offs, dec, doffs, dl, row_offs, row_caps, rows, cnt)
    if int(st.abs().sum()) or int(ds.abs().sum()) or not bool((dl == rec_lens).all()) or \
            cnt.cpu().tolist() != [c for _, c in spec] or not torch.equal(rows["timestamp"], d["ts"]) \
            or not bool((rows["val_len"] == 100).all()):
        raise SystemExit(f"rank {rank}: the perf-tool batches did not come back from the reader side")
    if not bool((blens == flens + 61).all()):
        raise SystemExit(f"rank {rank}: a perf-tool batch was left uncompressed")
    total = int(rl.sum())
    clen = int(flens.to(torch.int64).sum())
    return {"ms": ms, "kernel_ms": kms, "bytes": total, "records": n, "messages": msgs,
            "alg_bytes": 100 + 48 * msgs + 2 * (total + 61 * n) + clen + 2 * 61 * n,
            "ratio": total / clen, "host_sample": (m, spec), "fast": fast}


def cpu_baseline_perf_tool(m, spec, seconds=6.0):
    """configs[0]'s producer-side work on ONE host core: the oracle's restatement of the v2
    record writer (msgset_oracle.c), the reference's own compiled lz4frame.c / lz4.c driven as
    rd_kafka_lz4_compress drives it (oracle/_ref; the restatement when it is not in the
    tree), CRC32C of the finished batch (crc32c_hw restated)."""
    import oracle
    use_ref = oracle.ref_available()
    done, nmsgs, t0 = 0, 0, time.perf_counter()
    while True:
        first, cnt = spec[done % len(spec)]
        mset = oracle.msgset_v2_write(m, first, cnt, -1, -1, -1, 0)
        err, frame = (oracle.ref_rdk_lz4_compress([mset[61:]]) if use_ref
                      else oracle.rdk_lz4_compress(mset[61:]))
        assert err == 0
        oracle.crc32c_hw(0, mset[21:61] + frame)
        done += 1
        nmsgs += cnt
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(nmsgs / el, 1), "unit": "msgs/s", "cores": 1,
            "kind": "reference" if use_ref else "port",
            "sample": f"{done} MessageSets ({nmsgs} messages of 100 B) in {el:.1f} s: v2 record writer "
                      f"restated + {'the reference lz4frame.c' if use_ref else 'lz4 restated'} + "
                      f"CRC32C (crc32c_hw restated), {cpu_model()}"}


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
    n = n or args.partitions
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
    n = n or args.partitions
    # measured sweep (threads x slot MiB, 4 slots each): 1x32 18.5, 1x64 22.2, 1x128 27.4,
    # 2x64 26.5, 2x128 9.6, 1x256 5.8 GB/s -- host gather + PCIe bound; past ~1 GiB of pinned
    # staging in the rings the host-side gather slows down sharply on this box
    threads = threads or int(os.environ.get("RDK_BENCH_PRODUCER_THREADS", "1"))
    slot_mib = slot_mib or int(os.environ.get("RDK_BENCH_PRODUCER_SLOT_MIB", "128"))
    distinct = 8
    recs = [L.gen_json(JSON_BATCH, 42 + rank * 97 + j) for j in range(distinct)]
    hdrs = [W.v2_header(i, 61 + JSON_BATCH) for i in range(n)]
    parts = [list(range(t, n, threads)) for t in range(threads)]
    nslots = int(os.environ.get("RDK_BENCH_PRODUCER_NSLOTS", "4"))
    prods = [L.Producer(0, slot_bytes=slot_mib << 20, nslots=nslots, mode=mode) for _ in range(threads)]
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

    once()  # warm-up: staging allocations, first touch of every slot's pinned memory
    once()
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


def cpu_reference_lz4(kind, n=64, seconds=4.0, level=0, with_crc=False):
    """The reference's own compiled lz4frame.c / lz4.c / lz4hc.c (oracle/_ref, built from
    /root/reference/src in the build container), driven like rd_kafka_lz4_compress /
    _decompress (rdkafka_lz4.c:329-442 / :167-317: fresh LZ4F context and malloc per call),
    on CPU_THREADS host threads over n x 1 MiB JSON batches.  with_crc adds the CRC32C pass
    of calc_crc_v2 over the frames (crc32c_hw restated: crc32c.c itself needs the generated
    config.h).  Falls back to the restatement (kind "port") when the reference build is not
    in the tree."""
    import numpy as np
    import oracle
    import librdkafka_amd as L
    R = oracle.ref()
    if R is None:
        return cpu_baseline_lz4(kind, n, seconds, level)
    data = np.frombuffer(L.gen_json(JSON_BATCH * 8, 42), dtype=np.uint8)
    src = np.concatenate([data] * (n // 8))
    offs = (np.arange(n, dtype=np.uint64) * JSON_BATCH).astype(np.uint64)
    lens = np.full(n, JSON_BATCH, dtype=np.uint32)
    bound = int(oracle.lib().or_lz4f_compress_bound(JSON_BATCH))
    cbuf = np.zeros(n * bound, dtype=np.uint8)
    coffs = (np.arange(n, dtype=np.uint64) * bound).astype(np.uint64)
    clens = np.zeros(n, dtype=np.uint32)
    crcs = np.zeros(n, dtype=np.uint32)
    lib = oracle.lib()

    def comp():
        assert R.ref_lz4f_compress_batches_mt(src.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                              n, cbuf.ctypes.data, coffs.ctypes.data,
                                              clens.ctypes.data, level, CPU_THREADS) == 0
        if with_crc:
            lib.or_crc32c_batches_mt(cbuf.ctypes.data, coffs.ctypes.data, clens.ctypes.data,
                                     crcs.ctypes.data, n, CPU_THREADS)

    comp()
    dbuf = np.zeros(n * JSON_BATCH, dtype=np.uint8)
    dlens = np.zeros(n, dtype=np.uint32)

    def dec():
        if with_crc:
            lib.or_crc32c_batches_mt(cbuf.ctypes.data, coffs.ctypes.data, clens.ctypes.data,
                                     crcs.ctypes.data, n, CPU_THREADS)
        assert R.ref_lz4f_decompress_batches_mt(cbuf.ctypes.data, coffs.ctypes.data,
                                                clens.ctypes.data, n, 1 << 30, dbuf.ctypes.data,
                                                offs.ctypes.data, dlens.ctypes.data,
                                                CPU_THREADS) == 0

    fn = comp if kind == "compress" else dec
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    what = f"rd_kafka_lz4_{kind} driven through the reference's compiled lz4frame.c"
    if level:
        what += f" at compression.level {level}"
    if with_crc:
        what += " + CRC32C of the frames (crc32c_hw restated)"
    return {"value": round(passes * n * JSON_BATCH / el / 1e9, 3), "unit": "GB/s",
            "cores": CPU_THREADS, "kind": "reference",
            "sample": f"{n} x 1 MiB JSON batches, {passes} passes, {what}, {cpu_model()}"}


def dropin_threads_lib():
    """bench_native/libdropin_threads.so: pthreads calling one drop-in symbol through a function
    pointer (built by __graft_entry__.build())."""
    import ctypes as C
    h = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_native",
                            "libdropin_threads.so"))
    h.dropin_threads_run.restype = C.c_double
    h.dropin_threads_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32,
                                     C.c_size_t, C.c_int, C.c_double]
    return h


def bench_dropin_calls(seconds=0.3, cpu=True, thread_counts=(1, 8)):
    """Per-call cost of the drop-in symbols (host buffer in, host result out: gather into
    pinned staging, H2D, kernels, D2H, stream synchronise) at the reference's batch sizes,
    called from 1 and from 8 native threads at once (wall time / calls of all threads: the
    broker threads' concurrent calls go to the device together), beside the reference's
    compiled code on one host core.  Microseconds per call."""
    import ctypes as C
    import oracle
    import librdkafka_amd as L
    lib, olib, R = L.lib(), oracle.lib(), oracle.ref()
    T = dropin_threads_lib()
    out = {}

    def per_call(fn):
        fn()
        calls, t0 = 0, time.perf_counter()
        while True:
            fn()
            calls += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return round(el / calls * 1e6, 1)

    def fptr(f):
        return C.cast(f, C.c_void_p)

    before = L.dropin_combined()
    for size in (16384, 65536, 1 << 20):
        data = L.gen_json(size, 7)
        buf = C.create_string_buffer(data, size)
        err, frame = L.rd_kafka_lz4_compress(1, 0, data)
        assert err == 0
        fbuf = C.create_string_buffer(frame, len(frame))
        crc = oracle.crc32c(0, data)
        row = {}
        for th in thread_counts:
            tag = "gpu_us" if th == 1 else f"gpu_us_{th}_threads"
            for name, which, fn, b, n, xl in (
                    ("crc32c", 0, lib.crc32c, buf, size, 0),
                    ("rd_slice_crc32c", 1, lib.rd_slice_crc32c, buf, size, 0),
                    ("lz4_compress", 2, lib.rd_kafka_lz4_compress, buf, size, len(frame)),
                    ("lz4_decompress", 3, lib.rd_kafka_lz4_decompress, fbuf, len(frame), size)):
                us = T.dropin_threads_run(which, fptr(fn), b, n, crc, xl, th, seconds)
                assert us > 0, f"{name} x {th} threads at {size} B: wrong result"
                row[f"{name}_{tag}"] = round(us, 1)
        if cpu:
            row["crc32c_cpu_us"] = per_call(lambda: olib.or_crc32c_hw(0, buf, size))
        if cpu and R is not None:
            seg = C.c_char_p(data)
            sl1 = C.c_size_t(size)
            o, ol, g = C.c_void_p(), C.c_size_t(), C.c_int()

            def ref_c():
                assert R.ref_rdk_lz4_compress(1, 0, C.byref(seg), C.byref(sl1), 1, C.byref(o),
                                              C.byref(ol)) == 0
                R.ref_free(o)

            def ref_d():
                assert R.ref_rdk_lz4_decompress(1, fbuf, len(frame), 1 << 30, C.byref(o),
                                                C.byref(ol), C.byref(g)) == 0
                R.ref_free(o)
            row["lz4_compress_cpu_us"] = per_call(ref_c)
            row["lz4_decompress_cpu_us"] = per_call(ref_d)
        out[f"{size}B"] = row
    after = L.dropin_combined()
    nb, nr = after[0] - before[0], after[1] - before[1]
    out["combined"] = {"batches": nb, "requests_per_batch": round(nr / nb, 2) if nb else 0,
                       "largest": after[2], "fallbacks": after[3] - before[3],
                       "enabled": os.environ.get("RDK_HIP_COMBINE", "1") != "0"}
    out["note"] = ("gpu: drop-in symbol through the C ABI on a host buffer (PCIe round trip + "
                   "synchronise per launch), called by native threads in a loop, wall time / all "
                   "threads' calls; concurrent calls are served as one launch (combined); "
                   "cpu: the reference's compiled lz4frame.c (kind reference) and crc32c_hw "
                   "restated (port), one core, " + cpu_model())
    return out


def dropin_uncombined_columns():
    """The 8-thread columns once more with RDK_HIP_COMBINE=0 (every call on its own thread's
    stream), in a child process: the switch is read once per process."""
    import subprocess
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--workload", "dropin", "--no-cpu-baseline"],
                       env=dict(os.environ, RDK_HIP_COMBINE="0"), capture_output=True, text=True,
                       timeout=300)
    if p.returncode:
        return {"error": p.stderr[-300:]}
    rows = json.loads(p.stdout.strip().splitlines()[-1])
    return {k: {n: v for n, v in row.items() if n.endswith("_threads")}
            for k, row in rows.items() if k.endswith("B")}


def leg_line(name, res, steps, world, cpu=None):
    d = {"GB_per_s": round(res["bytes"] * world / (res["ms"] / 1e3) / 1e9, 2),
         "ms_per_step": round(res["ms"], 3), "batches": res["records"] * world}
    if res.get("kernel_ms"):
        ach = res["alg_bytes"] / (res["kernel_ms"] / 1e3) / 1e9
        traffic, note = profile_summary(name, res["alg_bytes"], res["kernel_ms"])
        d["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel_ms": round(res["kernel_ms"], 4),
                         "alg_bytes_per_launch": int(res["alg_bytes"]), **note}
        if "issue" in note:  # the binding roofline beside the HBM one, under its own key too
            d["roofline_issue"] = {"bound": "valu_issue", "frac": note["issue"]["frac_of_issue_ceiling"],
                                   "floor_ms": note["issue"]["issue_floor_ms"],
                                   "valu_insts_per_launch": note["issue"]["valu_insts_per_launch"],
                                   "ceiling": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction"}
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
    res = bench_index(argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=256), rank, world)
    cpu = None if no_cpu else cpu_baseline_index(*res.pop("host_sample"))
    res.pop("host_sample", None)
    return leg_line("v2_record_index_1MiB_json", res, LEG_STEPS, world, cpu)


def legacy_leg(rank, world, no_cpu):
    res = bench_legacy(argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=256), rank, world)
    cpu = None if no_cpu else cpu_baseline_legacy(*res.pop("host_sample"))
    res.pop("host_sample", None)
    d = leg_line("v1_msgset_crc32_verify_1MiB_json", res, LEG_STEPS, world, cpu)
    d["finalize_kernel_ms"] = res["finalize_kernel_ms"]
    return d


def serialize_leg(rank, world, no_cpu):
    res = bench_serialize(argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=256), rank, world)
    cpu = None if no_cpu else cpu_baseline_serialize(*res.pop("host_sample"))
    res.pop("host_sample", None)
    return leg_line("v2_record_serialize_1MiB_json", res, LEG_STEPS, world, cpu)


# ------------------------------------------------------------------ main
def crc_leg(args, rank, world):
    """configs[1]: CRC32C only, 1M x 16 KiB MsgVersion 2 batches (writer finalize)."""
    res = bench_crc(args, rank, world)
    ms = res["wall_s"] * 1e3 / args.steps
    achieved = res["alg_bytes"] / (res["kernel_ms"] / 1e3) / 1e9
    traffic, note = profile_summary("crc32c_only_16KiB_batches", res["alg_bytes"], res["kernel_ms"])
    d = {"GB_per_s": round(res["bytes"] / (ms / 1e3) / 1e9, 2), "ms_per_step": round(ms, 4),
         "batches": res["records"], "batch_bytes": CRC_BATCH_BYTES,
         "msgs_per_s": round(res["records"] / (ms / 1e3), 1),
         "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                      "kernel": "crc32c_msgset_v2_v4_kernel<FINALIZE>",
                      "kernel_ms": round(res["kernel_ms"], 4),
                      "alg_bytes_per_launch": int(res["alg_bytes"]), **note}}
    return d, res


SIZE_NAMES = {16384: "16KiB", 65536: "64KiB", 262144: "256KiB", 1 << 20: "1MiB"}
LEG_STEPS = 10


def finalize_leg_name(mode, size):
    return f"writer_finalize{'_fast' if mode else ''}_{SIZE_NAMES[size]}_json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="finalize_fast",
                    choices=["finalize", "finalize_fast", "crc", "lz4c", "lz4c_fast", "lz4c_units",
                             "lz4hc", "consumer", "producer", "serialize", "index", "legacy",
                             "snappyc", "snappyd", "perf_tool", "chain_writer", "chain_reader",
                             "dropin"])
    ap.add_argument("--batches", type=int, default=CRC_BATCHES, help="--workload crc: batches per GPU")
    ap.add_argument("--partitions", type=int, default=512,
                    help="toppars (batches) per GPU")
    ap.add_argument("--batch-bytes", type=int, default=JSON_BATCH, choices=sorted(SIZE_NAMES),
                    help="record bytes per batch of the LZ4 workloads")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true")
    ap.add_argument("--level", type=int, default=9, help="compression.level of --workload lz4hc")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than GPUs (ranks then share devices; labelled so)")
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
    # one rank per GPU; with fewer GPUs than ranks (a rehearsal on one device) ranks share,
    # and the line says so: n_gpus counts the devices actually used
    ndev = max(1, torch.cuda.device_count())
    device = local_rank % ndev
    shared = world > ndev
    if shared and not args.rehearsal:
        sys.exit(f"bench.py: {world} ranks but {ndev} GPU(s): pass --rehearsal to let ranks share "
                 f"devices (the line is then labelled shared_device, not a scaling point)")
    gpus_used = min(world, ndev)
    torch.cuda.set_device(device)
    import librdkafka_amd as L
    if not os.path.exists(L.LIB_PATH):
        raise SystemExit(f"{L.LIB_PATH} is not built: run __graft_entry__.build()")
    L.init(device)
    no_cpu = args.no_cpu_baseline or world > 1
    size = args.batch_bytes
    where = {"n_gpus": gpus_used, "ranks": world, **({"shared_device": True} if shared else {})}

    def finish():
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()

    if args.workload not in ("finalize", "finalize_fast") or size != JSON_BATCH:
        # single legs (profiling, A/B runs): one short JSON line
        if args.workload == "dropin":
            print(json.dumps(bench_dropin_calls(cpu=not no_cpu)), flush=True)
            return finish()
        if args.workload == "crc":
            d, res = crc_leg(args, rank, world)
            t_max = max_over_ranks(d["ms_per_step"], world)
            if rank == 0:
                d["GB_per_s"] = round(res["bytes"] * world / (t_max / 1e3) / 1e9, 2)
                if not no_cpu:
                    d["cpu_baseline"] = cpu_baseline_crc(*res["host_sample"])
                print(json.dumps({"workload": "crc", **where, "steps": args.steps,
                                  "source_hash": source_hash(), **d}), flush=True)
            return finish()
        name = LEG_NAMES.get(args.workload, args.workload)
        if args.workload in ("finalize", "finalize_fast"):
            mode = 1 if args.workload == "finalize_fast" else 0
            res = bench_finalize(args, rank, world, n=args.partitions, mode=mode, size=size)
            name = finalize_leg_name(mode, size)
        elif args.workload == "lz4hc":
            res = bench_lz4c(args, rank, world, n=args.partitions, level=args.level)
            name = f"lz4hc_compress_level{args.level}_1MiB_json"
        elif args.workload.startswith("lz4c"):
            res = bench_lz4c(args, rank, world, n=args.partitions, fast=args.workload == "lz4c_fast",
                             units=args.workload == "lz4c_units", size=size)
            name = name.replace("1MiB", SIZE_NAMES[size])
        elif args.workload == "producer":
            res = bench_producer(args, rank, world, n=args.partitions)
        elif args.workload == "serialize":
            res = bench_serialize(args, rank, world, n=args.partitions)
        elif args.workload == "index":
            res = bench_index(args, rank, world, n=args.partitions)
        elif args.workload == "legacy":
            res = bench_legacy(args, rank, world, n=args.partitions)
        elif args.workload == "perf_tool":
            res = bench_perf_tool(args, rank, world, with_fast=False)
        elif args.workload.startswith("chain"):
            wr, rd = bench_chain(args, rank, world, n=args.partitions, with_fast=False)
            res = wr if args.workload == "chain_writer" else rd
        elif args.workload.startswith("snappy"):
            res = bench_snappy(args, rank, world, n=args.partitions,
                               decompress=args.workload == "snappyd")
        else:
            res = bench_consumer(args, rank, world, n=args.partitions, size=size)
            name = name.replace("1MiB", SIZE_NAMES[size])
        t_max = max_over_ranks(res["ms"], world)
        if rank == 0:
            cpu = None
            if not no_cpu:
                if args.workload == "serialize":
                    cpu = cpu_baseline_serialize(*res["host_sample"])
                elif args.workload == "index":
                    cpu = cpu_baseline_index(*res["host_sample"])
                elif args.workload == "legacy":
                    cpu = cpu_baseline_legacy(*res["host_sample"])
                elif args.workload == "perf_tool":
                    cpu = cpu_baseline_perf_tool(*res["host_sample"])
                elif args.workload.startswith("snappy"):
                    cpu = cpu_baseline_snappy("compress" if args.workload == "snappyc" else "decompress")
                elif not args.workload.startswith("chain"):
                    cpu = cpu_reference_lz4("decompress" if args.workload == "consumer"
                                            else "compress",
                                            level=args.level if args.workload == "lz4hc" else 0,
                                            with_crc=args.workload in ("consumer", "finalize", "finalize_fast"))
            res.pop("host_sample", None)
            res["ms"] = t_max
            print(json.dumps({"workload": args.workload, **where, "steps": args.steps,
                              "source_hash": source_hash(),
                              **leg_line(name, res, args.steps, world, cpu)}), flush=True)
        return finish()

    # ------------------------------------------------------------ headline
    # north_star's bar for the compress half is "frames decode with the reference's
    # rd_kafka_lz4_decompress, ratio within 5 % of the reference's": the throughput
    # compressor (mode 1) meets it and is the headline; the byte-identical compressor is the
    # leg writer_finalize_1MiB_json.
    mode = 1 if args.workload == "finalize_fast" else 0
    res = bench_finalize(args, rank, world, mode=mode)
    # whole-job time per step: max over ranks of the host clock around the K synchronised
    # steps; the HIP-event time of the step feeds the roofline
    t_max = max_over_ranks(res["ms"], world)
    legs = {}
    if world > 1 and not args.no_legs:
        # configs[3] is quoted sharded over 2/4/8 GPUs: the consumer leg runs on every rank
        cres = bench_consumer(argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=1024 // world),
                              rank, world, n=1024 // world)
        cres["ms"] = max_over_ranks(cres["ms"], world)
        if rank == 0:
            legs["consumer_crc_verify_lz4f_decompress_1MiB"] = leg_line(
                "consumer_crc_verify_lz4f_decompress_1MiB_sharded", cres, LEG_STEPS, world)
    if rank == 0:
        n = res["records"]
        value = res["bytes"] * world / (t_max / 1e3) / 1e9
        achieved = res["alg_bytes"] / (res["kernel_ms"] / 1e3) / 1e9
        leg = finalize_leg_name(mode, JSON_BATCH)
        traffic, note = profile_summary(leg, res["alg_bytes"], res["kernel_ms"])
        kernels = (("lz4_units_blocks_kernel + lz4f_assemble_kernel<finalize> + crc32c_msgset_v2 kernels"
                    if os.environ.get("RDK_HIP_LZ4_FAST_ENGINE", "").startswith("u") else
                    "lz4_fast_blocks_kernel + lz4f_assemble_kernel<finalize>") if mode else
                   "lz4_compress_blocks_kernel<windows> + lz4f_assemble_kernel<finalize>")
        head = {
            "metric": "record-batch GB/s (CRC32C+LZ4F) at 1/2/4/8 GPUs; % of HBM roofline",
            "value": round(value, 2),
            "unit": "GB/s",
            **where,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded JSON-like records, valid v2 headers, device-resident)",
            "config": {"workload": "combined CRC32C+LZ4F, writer side: rdk_hip_msgset_v2_finalize = "
                                   "LZ4F compress (" + ("throughput compressor: frames decode with the "
                                                        "reference decoder, ratio within 5 % of the reference's"
                                                        if mode else
                                                        "frames byte-identical to rd_kafka_lz4_compress")
                                   + ") + v2 header finalize + CRC32C finalize of 1 MiB JSON "
                                   "MessageSets (configs[2] input, configs[4] shape), device-resident; "
                                   "value counts uncompressed record bytes",
                       "batches_per_gpu": n, "batch_bytes": JSON_BATCH,
                       "parallelism": f"toppar-sharded x{world}, no collective"},
            "msgs_per_s": round(res["messages"] * world / (t_max / 1e3), 1),
            "msgs_note": "JSON records (lines) carried by the batches, counted",
            "compression_ratio": round(res["ratio"], 3),
            "source_hash": source_hash(),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": kernels + " (the whole step)",
                         "kernel_ms": round(res["kernel_ms"], 4),
                         "alg_bytes_per_launch": int(res["alg_bytes"]), **note},
            "cpu_baseline": None,
        }
        if "issue" in note:
            head["roofline_issue"] = {"bound": "valu_issue", "frac": note["issue"]["frac_of_issue_ceiling"],
                                      "floor_ms": note["issue"]["issue_floor_ms"],
                                      "valu_insts_per_launch": note["issue"]["valu_insts_per_launch"],
                                      "ceiling": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction"}
        if not no_cpu:
            head["cpu_baseline"] = cpu_reference_lz4("compress", seconds=10.0, with_crc=True)
        del res
        torch.cuda.empty_cache()
        if world == 1:
            head["pcie_pinned"] = pcie_rates()
        if not args.no_legs and world == 1:
            sub = argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=256)
            cpu = (lambda *a, **k: None) if no_cpu else cpu_reference_lz4
            # configs[1]
            crc_args = argparse.Namespace(steps=10, warmup=2, batches=CRC_BATCHES)
            d, cres = crc_leg(crc_args, rank, world)
            if not no_cpu:
                d["cpu_baseline"] = cpu_baseline_crc(*cres["host_sample"])
            del cres
            torch.cuda.empty_cache()
            legs["crc32c_only_16KiB_batches"] = d
            # configs[0]'s workload through the engine
            pres = bench_perf_tool(sub, rank, world)
            pcpu = None if no_cpu else cpu_baseline_perf_tool(*pres.pop("host_sample"))
            pres.pop("host_sample", None)
            pl = leg_line("perf_tool_1M_x_100B_messages", pres, LEG_STEPS, 1, pcpu)
            pl["msgs_per_s"] = round(pres["messages"] / (pres["ms"] / 1e3), 1)
            pl["with_throughput_compressor"] = pres["fast"]
            legs["perf_tool_1M_x_100B_messages"] = pl
            del pres
            torch.cuda.empty_cache()
            # the other compressor on the headline's step
            other = bench_finalize(sub, rank, world, n=512, mode=1 - mode)
            legs[finalize_leg_name(1 - mode, JSON_BATCH)] = leg_line(
                finalize_leg_name(1 - mode, JSON_BATCH), other, LEG_STEPS, 1,
                cpu("compress", with_crc=True))
            del other
            # batch-size sweep of the combined step and of the consumer path, 512 MiB each
            for bsz in (16384, 65536, 262144):
                nb = (512 << 20) // bsz
                for m_ in (1, 0):
                    r_ = bench_finalize(sub, rank, world, n=nb, mode=m_, size=bsz)
                    ll = leg_line(finalize_leg_name(m_, bsz), r_, LEG_STEPS, 1)
                    ll["msgs_per_s"] = round(r_["messages"] / (r_["ms"] / 1e3), 1)
                    legs[finalize_leg_name(m_, bsz)] = ll
                    del r_
                    torch.cuda.empty_cache()
                r_ = bench_consumer(sub, rank, world, n=nb, size=bsz)
                legs[f"consumer_crc_verify_lz4f_decompress_{SIZE_NAMES[bsz]}"] = leg_line(
                    f"consumer_crc_verify_lz4f_decompress_{SIZE_NAMES[bsz]}", r_, LEG_STEPS, 1)
                del r_
                torch.cuda.empty_cache()
            legs["lz4f_compress_1MiB_json"] = leg_line(
                "lz4f_compress_1MiB_json", bench_lz4c(sub, rank, world, n=256), LEG_STEPS, 1, cpu("compress"))
            legs["lz4f_compress_fast_1MiB_json"] = leg_line(
                "lz4f_compress_fast_1MiB_json", bench_lz4c(sub, rank, world, n=256, fast=True), LEG_STEPS, 1,
                cpu("compress"))
            legs["lz4f_compress_units_1MiB_json"] = leg_line(
                "lz4f_compress_units_1MiB_json", bench_lz4c(sub, rank, world, n=256, units=True), LEG_STEPS, 1)
            # LZ4HC at its default level (LZ4HC_CLEVEL_DEFAULT = 9)
            legs["lz4hc_compress_level9_1MiB_json"] = leg_line(
                "lz4hc_compress_level9_1MiB_json", bench_lz4c(sub, rank, world, n=256, level=9), LEG_STEPS, 1,
                cpu("compress", level=9))
            # LZ4HC optimal parser at its top level (LZ4HC_CLEVEL_MAX = 12)
            legs["lz4hc_compress_level12_1MiB_json"] = leg_line(
                "lz4hc_compress_level12_1MiB_json",
                bench_lz4c(argparse.Namespace(steps=3, warmup=1, partitions=256), rank, world, n=256,
                           level=12), 3, 1, cpu("compress", level=12))
            legs["snappy_compress_1MiB_json"] = leg_line(
                "snappy_compress_1MiB_json", bench_snappy(sub, rank, world, n=256), LEG_STEPS, 1,
                None if no_cpu else cpu_baseline_snappy("compress"))
            legs["snappy_uncompress_1MiB_json"] = leg_line(
                "snappy_uncompress_1MiB_json",
                bench_snappy(argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=1024), rank, world,
                             n=1024, decompress=True), LEG_STEPS, 1,
                None if no_cpu else cpu_baseline_snappy("decompress"))
            legs["consumer_crc_verify_lz4f_decompress_1MiB"] = leg_line(
                "consumer_crc_verify_lz4f_decompress_1MiB",
                bench_consumer(argparse.Namespace(steps=LEG_STEPS, warmup=2, partitions=1024), rank, world,
                               n=1024), LEG_STEPS, 1, cpu("decompress", with_crc=True))
            legs["v2_record_serialize_1MiB_json"] = serialize_leg(rank, world, no_cpu)
            legs["v2_record_index_1MiB_json"] = index_leg(rank, world, no_cpu)
            legs["v1_msgset_crc32_verify_1MiB_json"] = legacy_leg(rank, world, no_cpu)
            wr, rd = bench_chain(sub, rank, world, n=256)
            legs["writer_messages_to_batches_1MiB_json"] = leg_line(
                "writer_messages_to_batches_1MiB_json", wr, LEG_STEPS, 1)
            legs["writer_messages_to_batches_1MiB_json"]["with_throughput_compressor"] = wr["fast"]
            legs["reader_batches_to_rows_1MiB_json"] = leg_line(
                "reader_batches_to_rows_1MiB_json", rd, LEG_STEPS, 1)
            prod = {}
            # ring shape per thread count (slot MiB, slots): large slots amortise the block
            # kernel's fixed latency, a small ring keeps the gather's destination in cache
            shapes = {1: (128, 8), 2: (128, 8), 4: (64, 2), 8: (32, 2)}
            for th in (1, 2, 4, 8):
                os.environ["RDK_BENCH_PRODUCER_NSLOTS"] = str(shapes[th][1])
                pr = bench_producer(argparse.Namespace(steps=2, warmup=1, partitions=2048), rank, world,
                                    n=2048, threads=th, slot_mib=shapes[th][0])
                prod[f"{th}_threads"] = round(pr["bytes"] / (pr["ms"] / 1e3) / 1e9, 2)
                if th == 1 or prod[f"{th}_threads"] >= max(prod.values()):
                    best = pr
            pl = leg_line("producer_pipeline_1MiB_json_pcie", best, 2, 1, cpu("compress", with_crc=True))
            pl["GB_per_s_by_host_threads"] = prod
            legs["producer_pipeline_1MiB_json_pcie"] = pl
            if not no_cpu:
                legs["dropin_per_call_us"] = bench_dropin_calls()
                legs["dropin_per_call_us"]["uncombined_8_threads"] = dropin_uncombined_columns()
        # the legs first: whoever keeps only the end of this line keeps the headline
        line = {"legs": legs, **head} if legs else head
        # configs[1] once more among the last keys, where a truncated tail still shows it
        if "crc32c_only_16KiB_batches" in legs:
            c = legs["crc32c_only_16KiB_batches"]
            line["crc32c_only_16KiB_batches"] = {"GB_per_s": c["GB_per_s"], "frac": c["roofline"]["frac"],
                                                 "kernel_ms": c["roofline"]["kernel_ms"],
                                                 "traffic": c["roofline"]["traffic"]}
        print(json.dumps(line), flush=True)
    finish()


# bench leg name of a single --workload run (profiles/r03/<leg>.json)
LEG_NAMES = {"lz4c": "lz4f_compress_1MiB_json", "lz4c_fast": "lz4f_compress_fast_1MiB_json",
             "lz4c_units": "lz4f_compress_units_1MiB_json",
             "lz4hc": "lz4hc_compress_level9_1MiB_json",
             "consumer": "consumer_crc_verify_lz4f_decompress_1MiB",
             "serialize": "v2_record_serialize_1MiB_json", "index": "v2_record_index_1MiB_json",
             "legacy": "v1_msgset_crc32_verify_1MiB_json",
             "snappyc": "snappy_compress_1MiB_json", "snappyd": "snappy_uncompress_1MiB_json",
             "producer": "producer_pipeline_1MiB_json_pcie",
             "perf_tool": "perf_tool_1M_x_100B_messages",
             "chain_writer": "writer_messages_to_batches_1MiB_json",
             "chain_reader": "reader_batches_to_rows_1MiB_json"}


if __name__ == "__main__":
    main()
