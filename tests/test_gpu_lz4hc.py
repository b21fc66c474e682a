"""LZ4HC (compression.level 3..12) on the GPU: frames byte-identical to the
reference's LZ4F + lz4hc.c (golden frames from the reference build, and the
oracle restatement oracle/lz4hc_oracle.c), through the drop-in
rd_kafka_lz4_compress and the batch API rdk_hip_lz4f_compress."""
import hashlib
import importlib.util
import os
import random

import numpy as np
import pytest

from librdkafka_amd import workload as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _mg():
    spec = importlib.util.spec_from_file_location("mg", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def test_dropin_hc_matches_reference_golden(engine, golden):
    mg = _mg()
    for key, rec in golden("lz4hc_frames.json").items():
        data = mg.input_by_name(rec["input"])
        err, fr = engine.rd_kafka_lz4_compress(1, rec["level"], data)
        assert err == 0, key
        assert len(fr) == rec["frame_len"] and sha(fr) == rec["frame_sha256"], key


def _inputs(seed):
    rnd = random.Random(seed)
    out = [W.gen_json(1 << 20, 42), W.gen_json(200001, 3), bytes(70000), b"ab" * 40000,
           (b"0000" + b"1" * 7 + b"\0" * 9) * 5000, rnd.randbytes(70000), b"", b"x" * 12,
           b"x" * 13, b"hello world" * 3]
    for it in range(14):
        n = rnd.choice([14, 63, 4096, 65535, 65536, 65537, rnd.randrange(1, 200000)])
        kind = it % 3
        if kind == 0:
            out.append(W.gen_json(n, it))
        elif kind == 1:
            alpha = rnd.choice([1, 2, 4, 16])
            out.append(bytes(rnd.randrange(alpha) for _ in range(n)))
        else:
            base = rnd.randbytes(max(1, n // 40))
            out.append((base * 41)[:n])
    return out


def _pack(items, align=64):
    offs, pos = [], 0
    for b in items:
        offs.append(pos)
        pos += (len(b) + align - 1) // align * align
    buf = bytearray(pos + 256)
    for o, b in zip(offs, items):
        buf[o:o + len(b)] = b
    return buf, offs


@pytest.mark.parametrize("level", [3, 5, 7, 9, 10, 11, 12])
def test_batch_hc_matches_oracle(engine, oracle_mod, level):
    import torch
    inputs = _inputs(level)
    hbuf, hoffs = _pack(inputs)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    bounds = [engine.lz4f_compress_bound(len(b)) for b in inputs]
    ooffs = np.concatenate([[0], np.cumsum([(b + 63) // 64 * 64 for b in bounds])[:-1]])
    d_out = torch.zeros(int(ooffs[-1]) + bounds[-1] + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
    out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens, level=level)
    host = bytes(d_out.cpu().numpy())
    fl = out_lens.cpu().numpy()
    for i, b in enumerate(inputs):
        fr = host[ooffs[i]:ooffs[i] + fl[i]]
        err, want = oracle_mod.rdk_lz4_compress(b, comp_level=level)
        assert err == 0 and fr == want, (level, i, len(b), len(fr), len(want))


def test_hc_levels_above_12_clamp(engine, oracle_mod):
    """MIN(LZ4HC_CLEVEL_MAX, cLevel), lz4hc.c:798"""
    data = W.gen_json(100000, 8)
    err, fr = engine.rd_kafka_lz4_compress(1, 13, data)
    assert err == 0 and fr == oracle_mod.rdk_lz4_compress(data, comp_level=12)[1]


def test_batch_hc_many_frames_queue_and_scratch_growth(engine, oracle_mod):
    """96 and 272 x 1 MiB at level 9 after a one-frame call: 1536 block items over a scratch that
    was last sized for 16 (it grows), then 4352 blocks in two chunks of the build and parse
    kernels.  Four distinct inputs rotate, so the oracle runs 4x."""
    import torch
    distinct = [W.gen_json(1 << 20, 90 + i) for i in range(4)]
    want = [oracle_mod.rdk_lz4_compress(b, comp_level=9)[1] for b in distinct]
    # 272 frames: 4352 blocks, more than one 4096-item chunk of the build / parse kernels holds
    for inputs in ([distinct[0]], [distinct[i % 4] for i in range(96)],
                   [distinct[i % 4] for i in range(272)]):
        hbuf, hoffs = _pack(inputs)
        d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
        in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
        in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
        bound = (engine.lz4f_compress_bound(1 << 20) + 63) // 64 * 64
        d_out = torch.zeros(len(inputs) * bound + 256, dtype=torch.uint8, device="cuda")
        out_offs = torch.arange(len(inputs), dtype=torch.int64, device="cuda") * bound
        out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
        engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens, level=9)
        host = bytes(d_out.cpu().numpy())
        fl = out_lens.cpu().numpy()
        for i in range(len(inputs)):
            assert host[i * bound:i * bound + fl[i]] == want[i % 4], (len(inputs), i)


@pytest.mark.parametrize("level", [4, 10])
def test_hc_frame_of_more_than_64_blocks(engine, oracle_mod, level):
    """a 4.3 MiB frame has 66 blocks: the parser's wave builds the tables of blocks 64 and 65
    itself (the build kernel serves the first block of each of the 64 block slots)"""
    data = W.gen_json(64 * 65536 + 70000, 17)
    err, fr = engine.rd_kafka_lz4_compress(1, level, data)
    assert err == 0 and fr == oracle_mod.rdk_lz4_compress(data, comp_level=level)[1]
