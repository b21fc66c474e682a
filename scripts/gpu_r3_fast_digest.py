"""Digest of the throughput compressor's frames over a fixed set of inputs (the wave engine's
parse is deterministic, so a change that is meant to keep the parse must keep this digest).
usage: python scripts/gpu_r3_fast_digest.py  -> prints FAST_DIGEST <sha256> <frames> <bytes>"""
import hashlib
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import librdkafka_amd as L  # noqa: E402
from librdkafka_amd import workload as W  # noqa: E402
from test_gpu_lz4 import _fast_compress, _fast_inputs  # noqa: E402

L.init(0)
rnd = random.Random(9)
words = [bytes(rnd.choice(b"abcdefghij") for _ in range(rnd.randrange(2, 10))) for _ in range(500)]
text = b" ".join(rnd.choice(words) for _ in range(300000))[:1 << 20]
inputs = _fast_inputs(41, 30) + _fast_inputs(44, 8) + [W.gen_json(1 << 20, s) for s in range(24)] + \
    [text, (rnd.randbytes(3000) * 400)[:1 << 20], (rnd.randbytes(70) * 3000)[:200000], bytes(300000),
     W.PERF_PATTERN * 4000] + [W.gen_json(n, n) for n in (2047, 2048, 2049, 2060, 2061, 2200, 4096, 16384, 65535)]
frames = _fast_compress(L, inputs)
h = hashlib.sha256()
for fr in frames:
    h.update(len(fr).to_bytes(4, "little"))
    h.update(fr)
print("FAST_DIGEST", h.hexdigest(), len(frames), sum(len(f) for f in frames), flush=True)
per = [hashlib.sha256(f).hexdigest()[:8] for f in frames]
print("PER_FRAME", " ".join(per), flush=True)
