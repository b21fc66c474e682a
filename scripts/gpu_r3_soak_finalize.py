"""Finalize soak on the GPU: many seeds of the parity tests' input families (JSON, random,
zeros, repeats, word soup, small alphabets, sparse matches, short periods; edge sizes;
multi-block concatenations) as MessageSets through rdk_hip_msgset_v2_finalize, exact and
throughput mode, at every input alignment; every finished batch checked field by field
against the oracle (frame byte for byte in exact mode, decoded back in throughput mode), the
frame lengths, and a CRC VERIFY pass over all of them.
Usage: gpu_r3_soak_finalize.py FIRST_SEED N_SEEDS [COUNT]."""
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import librdkafka_amd as L  # noqa: E402
import oracle  # noqa: E402
from librdkafka_amd import workload as W  # noqa: E402
from test_gpu_producer import _check_batch  # noqa: E402
from test_window_sim import _inputs  # noqa: E402

first, nseeds = int(sys.argv[1]), int(sys.argv[2])
count = int(sys.argv[3]) if len(sys.argv) > 3 else 120
L.init(0)
t64 = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device="cuda")  # noqa: E731
t32 = lambda a: torch.tensor(np.asarray(a, dtype=np.int32), device="cuda")  # noqa: E731
batches = 0
for seed in range(first, first + nseeds):
    rnd = random.Random(seed)
    recs = _inputs(seed, count)
    recs += [b"".join(recs[i] for i in range(k, k + rnd.randrange(2, 9))) for k in range(0, 40, 8)]
    recs += [W.gen_json(rnd.randrange(1, 300000), seed * 7 + j) for j in range(6)]
    items = []
    for i, rec in enumerate(recs):
        hdr = bytearray(W.v2_header(i, 61 + len(rec)))
        hdr[21:23] = (0x10 if i % 3 == 0 else 0).to_bytes(2, "big")
        items.append((bytes(hdr), rec))
    in_offs, pos = [], 0
    for i, (hdr, rec) in enumerate(items):
        pos += (i + seed) % 4
        in_offs.append(pos + 61)
        pos += 61 + len(rec)
    hbuf = bytearray(pos + 256)
    for o, (hdr, rec) in zip(in_offs, items):
        hbuf[o - 61:o] = hdr
        hbuf[o:o + len(rec)] = rec
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    n = len(items)
    for mode in (0, 1):
        caps = [61 + L.lz4f_compress_bound(len(rec)) + (i * 5 + seed) % 11 for i, (_, rec) in enumerate(items)]
        out_offs = np.concatenate([[0], np.cumsum(caps)[:-1]])
        d_out = torch.zeros(int(sum(caps)) + 256, dtype=torch.uint8, device="cuda")
        flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
        L.msgset_v2_finalize(d_in, t64(in_offs), t32([len(r) for _, r in items]), d_out,
                             t64(out_offs), t32(caps), flens, blens, crcs, mode=mode)
        host = bytes(d_out.cpu().numpy())
        bl, fl = blens.cpu().numpy(), flens.cpu().numpy()
        cr = crcs.cpu().numpy().view(np.uint32)
        for i, (hdr, rec) in enumerate(items):
            out = host[out_offs[i]:out_offs[i] + bl[i]]
            try:
                _check_batch(oracle, hdr, rec, out, int(cr[i]), mode == 0)
                if int.from_bytes(out[21:23], "big") & 7 == 3:
                    assert fl[i] == bl[i] - 61
                if mode == 0:
                    assert fl[i] == len(oracle.rdk_lz4_compress(rec)[1])
            except AssertionError:
                print(f"FINALIZE_MISMATCH seed {seed} mode {mode} item {i} len {len(rec)}", flush=True)
                raise
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        L.msgset_v2_crc(d_out, t64(out_offs), t32(caps), st, L.V2_CRC_VERIFY)
        assert int(st.abs().sum()) == 0, (seed, mode)
        batches += n
    if (seed - first) % 5 == 4:
        print(f"seed {seed} ok, {batches} batches so far", flush=True)
print(f"FINALIZE_SOAK_OK {nseeds} seeds, {batches} batches", flush=True)
