"""GPU parity for LZ4F: frames from the HIP encoder are byte-identical to the
reference encoder's (golden frames made by the reference build, and the
oracle restatement that is pinned to it); the HIP decoder reproduces the
reference decoder's verdict (error code, length, bytes) on valid, malformed
and other-producer frames."""
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


def golden_inputs():
    spec = importlib.util.spec_from_file_location("mg", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


# ------------------------------------------------------------ drop-in path
def test_dropin_compress_matches_reference_frames(engine, golden):
    mg = golden_inputs()
    frames = golden("lz4f_frames.json")
    for name, data in mg.inputs():
        err, fr = engine.rd_kafka_lz4_compress(1, 0, data)
        assert err == 0, name
        rec = frames[name]
        assert len(fr) == rec["frame_len"] and sha(fr) == rec["frame_sha256"], name


def test_dropin_compress_segments_levels_legacy(engine, oracle_mod):
    rnd = random.Random(31)
    data = W.gen_json(300001, 3)
    cuts = sorted(rnd.sample(range(1, len(data)), 9))
    segs = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
    s = engine.RdSlice(segs)
    err, fr = engine.rd_kafka_lz4_compress(1, 0, s)
    assert err == 0 and fr == oracle_mod.rdk_lz4_compress(data)[1]
    assert s.remains() == 0                                   # slice consumed (lz4.c:409)
    for level in (-1, -3, 1, 2):
        assert engine.rd_kafka_lz4_compress(1, level, data)[1] == \
            oracle_mod.rdk_lz4_compress(data, comp_level=level)[1], level
    assert engine.rd_kafka_lz4_compress(0, 0, data)[1] == \
        oracle_mod.rdk_lz4_compress(data, proper_hc=0)[1]     # broken HC for MsgVersion 0
    s10 = engine.RdSlice(segs)
    err, fr = engine.rd_kafka_lz4_compress(1, 10, s10)        # LZ4HC optimal, through segments
    assert err == 0 and s10.remains() == 0
    assert fr == oracle_mod.rdk_lz4_compress(data, comp_level=10)[1]


def test_dropin_compress_random_shapes(engine, oracle_mod):
    rnd = random.Random(32)
    for it in range(60):
        kind = it % 4
        n = rnd.choice([0, 1, 5, 12, 13, 14, 63, 100, 4095, 4096, 65535, 65536, 65537, 131072,
                        rnd.randrange(0, 300000)])
        if kind == 0:
            data = W.gen_json(n, it)
        elif kind == 1:
            data = rnd.randbytes(n)
        elif kind == 2:
            data = bytes(n)
        else:
            base = rnd.randbytes(max(1, n // 50))
            data = (base * 60)[:n]
        assert engine.rd_kafka_lz4_compress(1, 0, data)[1] == oracle_mod.rdk_lz4_compress(data)[1], (it, n)


def test_dropin_decompress_golden_frames(engine, golden):
    mg = golden_inputs()
    frames = golden("lz4f_frames.json")
    for name, data in mg.inputs():
        rec = frames[name]
        if "frame_file" not in rec:
            continue
        err, out = engine.rd_kafka_lz4_decompress(1, 0, golden(rec["frame_file"]))
        assert err == 0 and out == data, name


def test_dropin_decompress_reference_verdicts(engine, golden):
    for c in golden("lz4f_decode_cases.json"):
        err, out = engine.rd_kafka_lz4_decompress(1, 0, bytes.fromhex(c["hex"]))
        assert err == c["err"], c["hex"][:80]
        if err == 0:
            assert len(out) == c["out_len"] and sha(out) == c["out_sha256"], c["hex"][:80]


def _apply_edit(frame, edit):
    f = bytearray(frame)
    for pos, val in edit.get("flip", []):
        f[pos] = val
    if "truncate" in edit:
        f = f[:edit["truncate"]]
    if "append" in edit:
        f += bytes.fromhex(edit["append"])
    return bytes(f)


def test_dropin_decompress_other_producers(engine, golden):
    var = golden("lz4f_variants.json")
    frames = {k: golden(v["file"]) for k, v in var["frames"].items()}
    for k, v in var["frames"].items():
        err, out = engine.rd_kafka_lz4_decompress(1, 0, frames[k])
        assert err == 0 and sha(out) == v["payload_sha256"], k
    for c in var["cases"]:
        err, out = engine.rd_kafka_lz4_decompress(1, 0, _apply_edit(frames[c["base"]], c))
        assert err == c["err"], c
        if err == 0:
            assert len(out) == c["out_len"] and sha(out) == c["out_sha256"], c


def test_dropin_decompress_legacy_hc_patches_input(engine, oracle_mod):
    data = W.gen_json(9000)
    fr = bytearray(oracle_mod.rdk_lz4_compress(data, proper_hc=0)[1])
    err, out = engine.rd_kafka_lz4_decompress(0, 0, fr)
    assert err == 0 and out == data
    assert fr[6] == 0x82                                      # fixed up in place


def test_dropin_decompress_block_fuzz_vs_oracle(engine, oracle_mod):
    """Mutated single-block frames: GPU verdict == oracle verdict (the oracle
    is checked against the compiled reference decoder in test_oracle)."""
    rnd = random.Random(33)
    for it in range(150):
        src = W.gen_json(rnd.randrange(20, 5000), 1000 + it)
        fr = bytearray(oracle_mod.rdk_lz4_compress(src)[1])
        for _ in range(rnd.randrange(1, 4)):
            p = rnd.randrange(11, max(12, len(fr) - 4))
            fr[p] = rnd.getrandbits(8)
        e1, o1 = engine.rd_kafka_lz4_decompress(1, 0, bytes(fr))
        e2, o2 = oracle_mod.rdk_lz4_decompress(bytes(fr))
        assert e1 == e2 and o1 == o2, it


def _lz4_block(seqs, last):
    """LZ4 block from (literals, offset, match_length) triples and the last literals."""
    out = bytearray()

    def ext(v):
        b = bytearray()
        v -= 15
        while v >= 255:
            b.append(255)
            v -= 255
        b.append(v)
        return b

    for lit, off, ml in seqs:
        mc = ml - 4
        out.append((min(len(lit), 15) << 4) | min(mc, 15))
        if len(lit) >= 15:
            out += ext(len(lit))
        out += lit + bytes([off & 0xFF, off >> 8])
        if mc >= 15:
            out += ext(mc)
    out.append(min(len(last), 15) << 4)
    if len(last) >= 15:
        out += ext(len(last))
    return bytes(out + last)


def test_decompress_matches_around_the_history_ring_edge(engine, oracle_mod):
    """Matches whose sources lie just inside and just outside the decoder's on-chip history
    (4 KiB per wavefront, written out in 1 KiB pieces): offsets 4096 +- a few, offsets that
    reach back to a piece written moments ago, and sources that straddle the edge.  Each
    frame is one hand-made block; the oracle decides what it decodes to."""
    rnd = random.Random(77)
    for base in (3000, 4096, 5000, 6000, 9000, 20000):
        first = bytes(rnd.randrange(256) for _ in range(base))
        seqs = [(first, 1, 4)]
        pos = base + 4
        for off in (4090, 4094, 4095, 4096, 4097, 4098, 4100, 4160, 3072, 3071, 3073, 5120, 2048, 1024,
                    1025, 1023, 8191, 8192, 12000):
            for ml in (4, 7, 19, 64, 70, 300):
                if off > pos:
                    continue
                lit = bytes(rnd.randrange(256) for _ in range(rnd.choice((0, 1, 3, 17))))
                seqs.append((lit, off, ml))
                pos += len(lit) + ml
                if pos > 60000:
                    break
            if pos > 60000:
                break
        block = _lz4_block(seqs, bytes(rnd.randrange(256) for _ in range(12)))
        frame = (bytes([0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82]) + len(block).to_bytes(4, "little") + block +
                 bytes(4))
        e2, want = oracle_mod.rdk_lz4_decompress(frame)
        assert e2 == 0 and len(want) > base
        e1, got = engine.rd_kafka_lz4_decompress(1, 0, frame)
        assert e1 == 0 and got == want, base


# ------------------------------------------------------- device batch engine
def _pack(items, align=64):
    offs, pos = [], 0
    for b in items:
        offs.append(pos)
        pos += (len(b) + align - 1) // align * align
    buf = bytearray(pos + 256)
    for o, b in zip(offs, items):
        buf[o:o + len(b)] = b
    return buf, offs


def test_batch_compress_decompress_roundtrip(engine, oracle_mod):
    import torch
    rnd = random.Random(34)
    sizes = [16384, 65536, 1000000, 1 << 20, 0, 13, 70000, 262144] + \
            [rnd.randrange(1, 200000) for _ in range(40)]
    inputs = [W.gen_json(n, i) if i % 5 else rnd.randbytes(n) for i, n in enumerate(sizes)]
    hbuf, hoffs = _pack(inputs)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    bounds = [engine.lz4f_compress_bound(len(b)) for b in inputs]
    ooffs = np.concatenate([[0], np.cumsum([(b + 63) // 64 * 64 for b in bounds])[:-1]])
    d_out = torch.empty(int(sum((b + 63) // 64 * 64 for b in bounds)) + 256, dtype=torch.uint8,
                        device="cuda")
    out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
    out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    host_out = bytes(d_out.cpu().numpy())
    flens = out_lens.cpu().numpy()
    frames = []
    for i, b in enumerate(inputs):
        fr = host_out[ooffs[i]:ooffs[i] + flens[i]]
        assert fr == oracle_mod.rdk_lz4_compress(b)[1], (i, len(b))
        frames.append(fr)
    # decompress the device frames in place on the device
    caps = [max(64, (len(b) + 65535) // 65536 * 65536) for b in inputs]
    doffs = np.concatenate([[0], np.cumsum(caps)[:-1]])
    d_dec = torch.empty(int(sum(caps)) + 256, dtype=torch.uint8, device="cuda")
    dec_offs = torch.tensor(doffs, dtype=torch.int64, device="cuda")
    dec_caps = torch.tensor(caps, dtype=torch.int32, device="cuda")
    dec_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    status = torch.full((len(inputs),), 7, dtype=torch.int32, device="cuda")
    engine.lz4f_decompress_batch(d_out, out_offs, out_lens, d_dec, dec_offs, dec_caps, dec_lens,
                                 status)
    st = status.cpu().numpy()
    dl = dec_lens.cpu().numpy()
    hdec = bytes(d_dec.cpu().numpy())
    for i, b in enumerate(inputs):
        assert st[i] == 0 and dl[i] == len(b), (i, st[i], dl[i], len(b))
        assert hdec[doffs[i]:doffs[i] + len(b)] == b, i


def test_batch_decompress_unaligned_destinations(engine, oracle_mod):
    """outputs at every byte alignment, capacity exactly the decoded size, guard bytes between
    them: each frame's bytes arrive and nothing next to them is touched (the decoder writes its
    output in 16-byte stores)"""
    import torch
    rnd = random.Random(77)
    sizes = [1, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 4095, 4096, 4097, 65535, 65536, 65537,
             70001, 131072 + 5, 200003] + [rnd.randrange(1, 150000) for _ in range(29)]
    inputs = [W.gen_json(n, 100 + i) if i % 4 else (rnd.randbytes(7) * (n // 7 + 1))[:n]
              for i, n in enumerate(sizes)]
    frames = [oracle_mod.rdk_lz4_compress(b)[1] for b in inputs]
    fbuf, foffs = _pack(frames)
    d_in = torch.frombuffer(fbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(foffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(f) for f in frames], dtype=torch.int32, device="cuda")
    doffs, pos = [], 0
    for i, b in enumerate(inputs):
        pos += 1 + (i * 7) % 16          # a gap of 1..16 guard bytes: every alignment occurs
        doffs.append(pos)
        pos += len(b)
    total = pos + 64
    d_dec = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    dec_offs = torch.tensor(doffs, dtype=torch.int64, device="cuda")
    dec_caps = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    dec_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    status = torch.full((len(inputs),), 7, dtype=torch.int32, device="cuda")
    engine.lz4f_decompress_batch(d_in, in_offs, in_lens, d_dec, dec_offs, dec_caps, dec_lens, status)
    st, dl = status.cpu().numpy(), dec_lens.cpu().numpy()
    host = bytes(d_dec.cpu().numpy())
    want = bytearray(b"\xa5" * total)
    for o, b in zip(doffs, inputs):
        want[o:o + len(b)] = b
    assert (st == 0).all() and (dl == [len(b) for b in inputs]).all()
    assert host == bytes(want)


def test_batch_decompress_dst_too_small(engine, oracle_mod):
    import torch
    data = W.gen_json(200000)
    fr = oracle_mod.rdk_lz4_compress(data)[1]
    d_in = torch.frombuffer(bytearray(fr) + bytearray(256), dtype=torch.uint8).cuda()
    z64 = lambda v: torch.tensor([v], dtype=torch.int64, device="cuda")  # noqa: E731
    z32 = lambda v: torch.tensor([v], dtype=torch.int32, device="cuda")  # noqa: E731
    d_dec = torch.empty(300000, dtype=torch.uint8, device="cuda")
    lens, st = z32(0), z32(0)
    engine.lz4f_decompress_batch(d_in, z64(0), z32(len(fr)), d_dec, z64(0), z32(100000), lens, st)
    assert int(st.item()) == engine.LZ4F_E_DSTSIZE
    engine.lz4f_decompress_batch(d_in, z64(0), z32(len(fr)), d_dec, z64(0), z32(262144), lens, st)
    assert int(st.item()) == 0 and int(lens.item()) == len(data)
    assert bytes(d_dec[:len(data)].cpu().numpy()) == data


def test_batch_scale_roundtrip_property(engine):
    """config 4/5 shape at scale: 512 x 1 MiB JSON batches compressed on the
    device, decompressed on the device, compared whole (size-independent
    round-trip property); a sample is compared with the reference frames."""
    import torch
    n, size = 512, 1 << 20
    one = engine.gen_json(size * 4, 42)
    base = torch.frombuffer(bytearray(one), dtype=torch.uint8).cuda()
    d_in = torch.empty(n * size + 256, dtype=torch.uint8, device="cuda")
    for i in range(n):  # 4 distinct MiB, rotated
        d_in[i * size:(i + 1) * size] = base[(i % 4) * size:(i % 4 + 1) * size]
    in_offs = torch.arange(n, dtype=torch.int64, device="cuda") * size
    in_lens = torch.full((n,), size, dtype=torch.int32, device="cuda")
    bound = engine.lz4f_compress_bound(size)
    bound = (bound + 255) // 256 * 256
    d_out = torch.empty(n * bound + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * bound
    out_lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    d_dec = torch.empty(n * size + 256, dtype=torch.uint8, device="cuda")
    caps = torch.full((n,), size, dtype=torch.int32, device="cuda")
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    engine.lz4f_decompress_batch(d_out, out_offs, out_lens, d_dec, in_offs, caps, dl, st)
    assert int(st.abs().sum()) == 0 and bool((dl == size).all())
    assert bool(torch.equal(d_dec[:n * size], d_in[:n * size]))
    ol = out_lens.cpu().numpy()
    # equal inputs give equal frames (the same 4 MiB rotate through the batches) ...
    assert all(ol[i] == ol[i % 4] for i in range(n))
    # ... and the 4 distinct inputs compress like JSON does, not like a stored block
    assert all(size / 3.2 < int(ol[i]) < size / 2.2 for i in range(4)), ol[:4]


@pytest.mark.parametrize("n", [2300, 4400])
def test_thousands_of_multiblock_frames(engine, oracle_mod, n):
    """more than 2048 frames of several blocks each (the frame assembler then runs in small
    workgroups and still has to slide every block down to its place, raw blocks included;
    more than 4096: the block kernel visits as many block slots per frame as the longest
    frame has blocks): a sample of frames byte-identical to the reference's, every frame
    decoded back"""
    import numpy as np
    import torch
    sizes = [150000, 65536, 65537, 200001, 131072, 70000, 13, 0]
    pieces = [engine.gen_json(sz, 900 + j) if j != 3 else bytes(random.Random(5).randbytes(sz))
              for j, sz in enumerate(sizes)]  # (j == 3: incompressible, its blocks are stored raw)
    slot = 200704
    host = np.zeros(len(sizes) * slot, dtype=np.uint8)
    for j, p in enumerate(pieces):
        host[j * slot:j * slot + len(p)] = np.frombuffer(p, dtype=np.uint8)
    base = torch.from_numpy(host).cuda().view(len(sizes), slot)
    d_in = torch.empty(n * slot + 256, dtype=torch.uint8, device="cuda")
    idx = torch.arange(n, device="cuda") % len(sizes)
    d_in[:n * slot].view(n, slot).copy_(base[idx])
    in_offs = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    in_lens = torch.tensor([sizes[i % len(sizes)] for i in range(n)], dtype=torch.int32, device="cuda")
    bound = (engine.lz4f_compress_bound(max(sizes)) + 255) // 256 * 256
    d_out = torch.empty(n * bound + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * bound
    out_lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    ol = out_lens.cpu().numpy()
    want = [oracle_mod.rdk_lz4_compress(p)[1] for p in pieces]
    for i in list(range(16)) + [777, 1500, n - 3, n - 2, n - 1]:
        got = bytes(d_out[i * bound:i * bound + int(ol[i])].cpu().numpy())
        assert got == want[i % len(sizes)], i
    assert all(int(ol[i]) == len(want[i % len(sizes)]) for i in range(n))
    d_dec = torch.empty(n * slot + 256, dtype=torch.uint8, device="cuda")
    caps = torch.full((n,), slot, dtype=torch.int32, device="cuda")
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    engine.lz4f_decompress_batch(d_out, out_offs, out_lens, d_dec, in_offs, caps, dl, st)
    assert int(st.abs().sum()) == 0 and bool((dl == in_lens).all())
    for j, p in enumerate(pieces):
        for i in (j, j + 8 * 100, j + 8 * 280):
            assert bytes(d_dec[i * slot:i * slot + len(p)].cpu().numpy()) == p, i


# ------------------------------------------------ throughput-mode compressor
def _fast_compress(engine, inputs, units=False):
    import torch
    hbuf, hoffs = _pack(inputs)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    bounds = [engine.lz4f_compress_bound(len(b)) for b in inputs]
    ooffs = np.concatenate([[0], np.cumsum([(b + 63) // 64 * 64 for b in bounds])[:-1]])
    d_out = torch.empty(int(sum((b + 63) // 64 * 64 for b in bounds)) + 256, dtype=torch.uint8,
                        device="cuda")
    out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
    out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    comp = engine.lz4f_compress_units_batch if units else engine.lz4f_compress_fast_batch
    comp(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    host_out = bytes(d_out.cpu().numpy())
    flens = out_lens.cpu().numpy()
    return [host_out[ooffs[i]:ooffs[i] + flens[i]] for i in range(len(inputs))]


def _fast_inputs(seed, count):
    rnd = random.Random(seed)
    sizes = [0, 1, 12, 13, 14, 100, 4095, 65535, 65536, 65537, 1000000, 1 << 20] + \
            [rnd.randrange(1, 300000) for _ in range(count)]
    out = []
    for i, n in enumerate(sizes):
        kind = i % 5
        if kind == 0:
            out.append(W.gen_json(n, i))
        elif kind == 1:
            out.append(rnd.randbytes(n))
        elif kind == 2:
            out.append(bytes(n))
        elif kind == 3:
            base = rnd.randbytes(max(1, n // 50))
            out.append((base * 60)[:n])
        else:
            words = [rnd.randbytes(rnd.randrange(2, 9)) for _ in range(200)]
            out.append(b" ".join(rnd.choice(words) for _ in range(n // 4 + 1))[:n])
    return out


@pytest.mark.parametrize("units", [False, True], ids=["wave-engine", "units-engine"])
def test_fast_compress_decodes_with_reference(engine, oracle_mod, units):
    """Every throughput-mode frame decodes to its input with the reference's
    own decoder (oracle/_ref build of lz4frame.c via rd_kafka_lz4_decompress's
    loop when present here; the pinned restatement on the GPU box) and with
    the GPU decoder; frame structure is the reference's (header, 64 KiB
    independent blocks, raw fallback, end mark)."""
    inputs = _fast_inputs(41, 30)
    frames = _fast_compress(engine, inputs, units)
    use_ref = oracle_mod.ref_available()
    for i, (b, fr) in enumerate(zip(inputs, frames)):
        assert fr[:7] == bytes([0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82]), i
        assert fr[-4:] == b"\0\0\0\0", i
        e, out = oracle_mod.ref_rdk_lz4_decompress(fr, max_msg_size=1 << 30)[:2] if use_ref \
            else oracle_mod.rdk_lz4_decompress(fr)
        assert e == 0 and out == b, (i, len(b), e)
        e2, out2 = engine.rd_kafka_lz4_decompress(1, 0, fr)
        assert e2 == 0 and out2 == b, i
        # every block is no larger than the reference's worst case (raw + 4)
        assert len(fr) <= engine.lz4f_compress_bound(len(b)), i


@pytest.mark.parametrize("units", [False, True], ids=["wave-engine", "units-engine"])
def test_fast_compress_ratio_within_5pct(engine, oracle_mod, units):
    """north_star: compression ratio within 5 % of the reference's CPU lz4 on
    the same input (JSON records of configs[2], text-like and repetitive)."""
    rnd = random.Random(43)
    words = [bytes(rnd.choice(b"abcdefghij") for _ in range(rnd.randrange(2, 10)))
             for _ in range(500)]
    text = b" ".join(rnd.choice(words) for _ in range(300000))[:1 << 20]
    inputs = [W.gen_json(1 << 20, 42), W.gen_json(65536, 7), W.gen_json(1 << 20, 5), text,
              (rnd.randbytes(3000) * 400)[:1 << 20]]
    frames = _fast_compress(engine, inputs, units)
    for i, (b, fr) in enumerate(zip(inputs, frames)):
        ref = oracle_mod.rdk_lz4_compress(b)[1]
        r_gpu, r_ref = len(b) / len(fr), len(b) / len(ref)
        assert r_gpu >= 0.95 * r_ref, (i, r_gpu, r_ref)


def test_fast_compress_data_that_stops_and_starts_matching(engine, oracle_mod):
    """Stretches without matches (random bytes) put the wave engine's rounds at every eighth
    position, the first match seen brings the dense rounds back (from a round earlier):
    blocks that change between the two, at
    several stretch lengths and in both orders, decode to their input, and the ratio stays
    within 5 % of the reference's (whose own search step grows over such stretches)."""
    rnd = random.Random(46)
    inputs = []
    for stretch in (600, 1100, 1400, 2048, 5000, 20000, 70000):
        parts = []
        for j in range(12):
            parts.append(rnd.randbytes(stretch) if j % 2 == 0 else W.gen_json(stretch, 40 + j))
        inputs.append(b"".join(parts))
        inputs.append(b"".join(parts[1:]))
    # sparse matches: a 24-byte string every few hundred random bytes
    key = rnd.randbytes(24)
    inputs.append(b"".join(rnd.randbytes(rnd.randrange(100, 700)) + key for _ in range(400)))
    inputs.append(rnd.randbytes(300000))
    frames = _fast_compress(engine, inputs)
    for i, (b, fr) in enumerate(zip(inputs, frames)):
        e, out = oracle_mod.rdk_lz4_decompress(fr)
        assert e == 0 and out == b, (i, len(b), e)
        assert engine.rd_kafka_lz4_decompress(1, 0, fr) == (0, b), i
        ref = oracle_mod.rdk_lz4_compress(b)[1]
        assert len(b) / len(fr) >= 0.95 * (len(b) / len(ref)), (i, len(b), len(fr), len(ref))


def test_units_engine_equals_the_sequential_model(engine):
    """The workgroup-per-block engine's output is defined by tests/sim/lz4_units_sim.cpp (candidates
    in position order, units parsed on their own, stitched in order): the kernel's frames
    must be that model's frames byte for byte, on every input family and edge size."""
    import units_model
    rnd = random.Random(45)
    inputs = _fast_inputs(45, 20)
    inputs += [W.gen_json(n, n) for n in (895, 896, 897, 13439, 13440, 13441, 26880, 65536 + 896)]
    inputs += [bytes(70000), (rnd.randbytes(3000) * 400)[:1 << 20], (rnd.randbytes(70) * 3000)[:200000]]
    m = W.gen_perf_messages(3000)
    inputs.append(W.PERF_PATTERN * 4000)
    del m
    frames = _fast_compress(engine, inputs, units=True)
    for i, (b, fr) in enumerate(zip(inputs, frames)):
        want = units_model.frame(b)
        assert fr == want, (i, len(b), len(fr), len(want))


@pytest.mark.parametrize("units", [False, True], ids=["wave-engine", "units-engine"])
def test_fast_compress_deterministic(engine, units):
    inputs = _fast_inputs(44, 8)
    assert _fast_compress(engine, inputs, units) == _fast_compress(engine, inputs, units)


def test_batch_compress_window_engine_inputs(engine, oracle_mod):
    """The inputs that drive every path of the windowed exact engine (in-window
    candidates, matches and catch-ups longer than the register windows, searches that
    outlast the stride-1 probes, window hand-over after a match, stored blocks): frames
    byte-identical to the oracle's, as one batch."""
    import torch
    from test_window_sim import _inputs
    inputs = _inputs(1, 250)
    inputs += [b"".join(inputs[i] for i in range(k, k + 9)) for k in range(0, 90, 9)]  # multi-block
    hbuf, hoffs = _pack(inputs)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    bounds = [(engine.lz4f_compress_bound(len(b)) + 63) // 64 * 64 for b in inputs]
    ooffs = np.concatenate([[0], np.cumsum(bounds)[:-1]])
    d_out = torch.empty(int(sum(bounds)) + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
    out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    host_out = bytes(d_out.cpu().numpy())
    flens = out_lens.cpu().numpy()
    for i, b in enumerate(inputs):
        fr = host_out[ooffs[i]:ooffs[i] + flens[i]]
        assert fr == oracle_mod.rdk_lz4_compress(b)[1], (i, len(b))
