"""Parity soak on the GPU: many more seeds of the input families the parity tests use
(JSON, random, zeros, repeats, word soup, small alphabets, sparse matches, short periods;
edge sizes; multi-block concatenations) through the batch API, compared with the oracle:
exact LZ4F frames, LZ4HC level 9 frames (a subset), snappy streams byte for byte, and both
decoders on the oracle's output.  Usage: gpu_soak_parity.py FIRST_SEED N_SEEDS [COUNT]."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import librdkafka_amd as L  # noqa: E402
import oracle  # noqa: E402
from test_window_sim import _inputs  # noqa: E402


def pack(chunks, align=64):
    offs, pos = [], 0
    for c in chunks:
        offs.append(pos)
        pos += (len(c) + align - 1) // align * align
    buf = bytearray(pos + 256)
    for o, c in zip(offs, chunks):
        buf[o:o + len(c)] = c
    return buf, offs


def dev(chunks):
    buf, offs = pack(chunks)
    return (torch.frombuffer(buf, dtype=torch.uint8).cuda(),
            torch.tensor(offs, dtype=torch.int64, device="cuda"),
            torch.tensor([len(c) for c in chunks], dtype=torch.int32, device="cuda"))


def run_out(fn, src, bound):
    d_in, in_offs, in_lens = dev(src)
    bounds = [(bound(len(b)) + 63) // 64 * 64 for b in src]
    ooffs = np.concatenate([[0], np.cumsum(bounds)[:-1]]).astype(np.int64)
    d_out = torch.zeros(int(sum(bounds)) + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(ooffs, device="cuda")
    out_lens = torch.zeros(len(src), dtype=torch.int32, device="cuda")
    fn(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    host = bytes(d_out.cpu().numpy())
    ln = out_lens.cpu().numpy()
    return [host[ooffs[i]:ooffs[i] + ln[i]] for i in range(len(src))]


def run_dec(fn, frames, sizes):
    d_in, in_offs, in_lens = dev(frames)
    caps = [(n + 63) // 64 * 64 + 64 for n in sizes]
    ooffs = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    d_out = torch.zeros(int(sum(caps)) + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(ooffs, device="cuda")
    out_caps = torch.tensor(np.asarray(sizes, np.int32), device="cuda")
    out_lens = torch.zeros(len(frames), dtype=torch.int32, device="cuda")
    st = torch.zeros(len(frames), dtype=torch.int32, device="cuda")
    fn(d_in, in_offs, in_lens, d_out, out_offs, out_caps, out_lens, st)
    host = bytes(d_out.cpu().numpy())
    ln = out_lens.cpu().numpy()
    return st.cpu().numpy(), [host[ooffs[i]:ooffs[i] + ln[i]] for i in range(len(frames))]


def main():
    first, nseeds = int(sys.argv[1]), int(sys.argv[2])
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 250
    total = 0
    for seed in range(first, first + nseeds):
        src = _inputs(seed, count)
        src += [b"".join(src[i] for i in range(k, k + 7)) for k in range(0, 70, 7)]  # multi-block
        ref = [oracle.rdk_lz4_compress(b)[1] for b in src]
        got = run_out(L.lz4f_compress_batch, src, L.lz4f_compress_bound)
        for i, (a, b) in enumerate(zip(got, ref)):
            assert a == b, ("lz4 exact", seed, i, len(src[i]))
        st, dec = run_dec(L.lz4f_decompress_batch, ref, [len(b) for b in src])
        assert not st.any(), ("lz4 decode status", seed, np.nonzero(st)[0][:5])
        for i, (a, b) in enumerate(zip(dec, src)):
            assert a == b, ("lz4 decode", seed, i, len(b))
        sub = src[::9]
        refh = [oracle.rdk_lz4_compress(b, 1, 9)[1] for b in sub]
        goth = run_out(lambda *a: L.lz4f_compress_batch(*a, level=9), sub, L.lz4f_compress_bound)
        for i, (a, b) in enumerate(zip(goth, refh)):
            assert a == b, ("lz4hc 9", seed, i, len(sub[i]))
        refs = [oracle.snappy_compress(b) for b in src]
        gots = run_out(L.snappy_compress_batch, src, L.snappy_max_compressed_length)
        for i, (a, b) in enumerate(zip(gots, refs)):
            assert a == b, ("snappy", seed, i, len(src[i]))
        st, dec = run_dec(L.snappy_uncompress_batch, refs, [len(b) for b in src])
        assert not st.any(), ("snappy decode status", seed, np.nonzero(st)[0][:5])
        for i, (a, b) in enumerate(zip(dec, src)):
            assert a == b, ("snappy decode", seed, i, len(b))
        total += len(src)
        print(f"seed {seed}: {len(src)} inputs ok", flush=True)
    print(f"SOAK_OK {total} inputs")


if __name__ == "__main__":
    main()
