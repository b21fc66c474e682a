"""Throughput-compressor soak on data that moves between matching and not matching: blocks
built from random stretches, JSON records, zero runs, short-period repeats and word soup in
random order and lengths (so that the rounds change between stride 1, 2 and 8 at arbitrary
positions); every frame decoded by the oracle and by the GPU decoder, worst ratio relative to
the reference's printed (over the inputs the reference shrinks less than 8-fold).  Usage: gpu_r3_soak_fast_mixed.py FIRST_SEED N_SEEDS."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import librdkafka_amd as L  # noqa: E402
import oracle  # noqa: E402
from librdkafka_amd import workload as W  # noqa: E402
from test_gpu_lz4 import _fast_compress  # noqa: E402

first, nseeds = int(sys.argv[1]), int(sys.argv[2])
L.init(0)
worst, frames_done = 9.0, 0
for seed in range(first, first + nseeds):
    rnd = random.Random(seed)
    words = [rnd.randbytes(rnd.randrange(2, 9)) for _ in range(100)]
    inputs, descr = [], []
    for _ in range(24):
        parts, kinds, total = [], [], rnd.randrange(1000, 400000)
        while sum(map(len, parts)) < total:
            n = rnd.choice((50, 300, 900, 1100, 2100, 5000, 30000, 70000))
            n = rnd.randrange(n // 2 + 1, n + 1)
            kind = rnd.randrange(5)
            kinds.append((kind, n))
            if kind == 0:
                parts.append(rnd.randbytes(n))
            elif kind == 1:
                parts.append(W.gen_json(n, rnd.randrange(1 << 20)))
            elif kind == 2:
                parts.append(bytes(n))
            elif kind == 3:
                parts.append((rnd.randbytes(rnd.randrange(1, 40)) * n)[:n])
            else:
                parts.append(b" ".join(rnd.choice(words) for _ in range(n // 4 + 1))[:n])
        inputs.append(b"".join(parts))
        descr.append(kinds)
    frames = _fast_compress(L, inputs)
    for i, (b, fr) in enumerate(zip(inputs, frames)):
        e, out = oracle.rdk_lz4_decompress(fr)
        if e != 0 or out != b or L.rd_kafka_lz4_decompress(1, 0, fr) != (0, b):
            print(f"FAST_MIXED_MISMATCH seed {seed} input {i} len {len(b)} err {e}", flush=True)
            sys.exit(1)
        ref = oracle.rdk_lz4_compress(b)[1]
        # (inputs the reference shrinks more than 8-fold are left out of the comparison: there
        # a few dozen bytes -- a round's worth of literals at the start of a run -- decide the
        # quotient)
        if len(b) < 8 * len(ref) and len(ref) / len(fr) < worst:
            worst = len(ref) / len(fr)
            print(f"worst so far {worst:.4f}: seed {seed} input {i} len {len(b)} gpu {len(fr)} ref {len(ref)} parts {descr[i][:12]}", flush=True)
    frames_done += len(frames)
    if (seed - first) % 10 == 9:
        print(f"seed {seed} ok, {frames_done} frames, worst ratio rel {worst:.4f}", flush=True)
print(f"FAST_MIXED_OK {nseeds} seeds, {frames_done} frames, worst ratio relative to the reference {worst:.4f}", flush=True)
