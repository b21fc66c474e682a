"""Ratio of the throughput compressor relative to the reference's on data that alternates
between stretches without matches and JSON records (the inputs of
test_fast_compress_data_that_stops_and_starts_matching), one line per input.
RDK_HIP_LIB selects the build.  Usage: python scripts/gpu_r3_sparse_ratios.py"""
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

L.init(0)
rnd = random.Random(46)
inputs, names = [], []
for stretch in (600, 1100, 1400, 2048, 5000, 20000, 70000):
    parts = [rnd.randbytes(stretch) if j % 2 == 0 else W.gen_json(stretch, 40 + j) for j in range(12)]
    inputs += [b"".join(parts), b"".join(parts[1:])]
    names += [f"random/json x {stretch}", f"json/random x {stretch}"]
key = rnd.randbytes(24)
inputs.append(b"".join(rnd.randbytes(rnd.randrange(100, 700)) + key for _ in range(400)))
names.append("24-byte key every 100-700 random bytes")
frames = _fast_compress(L, inputs)
for name, b, fr in zip(names, inputs, frames):
    ref = oracle.rdk_lz4_compress(b)[1]
    print(f"SPARSE_RATIO {name:42s} gpu {len(fr):8d} ref {len(ref):8d} rel {len(ref) / len(fr):.4f}", flush=True)
