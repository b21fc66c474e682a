"""snappy on the GPU (csrc/snappy.hip): streams byte-identical to the restatement of
snappy.c's compress_fragment (oracle/snappy_oracle.c; its parity with snappy.c itself is
unpinned, see that file), decodable by an independent snappy (pyarrow's), and a decoder whose
verdicts (0 / -EIO) and payloads equal the oracle's on valid, foreign and damaged streams.
Through the drop-in symbols of src/snappy.h and through the batch API."""
import random
import struct

import numpy as np
import pytest

from librdkafka_amd import workload as W
from test_oracle_snappy import snappy_cases

pytestmark = pytest.mark.gpu


def _pack(items, align=64):
    offs, pos = [], 0
    for b in items:
        offs.append(pos)
        pos += (len(b) + align - 1) // align * align
    buf = bytearray(pos + 256)
    for o, b in zip(offs, items):
        buf[o:o + len(b)] = b
    return buf, offs


def _compress_batch(engine, inputs):
    import torch
    hbuf, hoffs = _pack(inputs)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    bounds = [engine.snappy_max_compressed_length(len(b)) for b in inputs]
    ooffs = np.concatenate([[0], np.cumsum([(b + 63) // 64 * 64 for b in bounds])[:-1]]).astype(np.int64)
    d_out = torch.zeros(int(ooffs[-1]) + bounds[-1] + 256, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
    out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    engine.snappy_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens)
    host = bytes(d_out.cpu().numpy())
    fl = out_lens.cpu().numpy()
    return [host[ooffs[i]:ooffs[i] + fl[i]] for i in range(len(inputs))]


def _uncompress_batch(engine, streams, caps=None):
    import torch
    hbuf, hoffs = _pack(streams)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in streams], dtype=torch.int32, device="cuda")
    if caps is None:
        caps = []
        for s in streams:   # the reader sizes its buffer from the preamble
            v, sh = 0, 0
            for b in s[:5]:
                v |= (b & 127) << sh
                sh += 7
                if b < 128:
                    break
            caps.append(min(v, 1 << 26))
    ooffs = np.concatenate([[0], np.cumsum([(c + 255) // 64 * 64 for c in caps])[:-1]]).astype(np.int64)
    d_out = torch.zeros(int(ooffs[-1]) + caps[-1] + 512, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
    out_caps = torch.tensor(caps, dtype=torch.int32, device="cuda")
    out_lens = torch.zeros(len(streams), dtype=torch.int32, device="cuda")
    status = torch.full((len(streams),), 77, dtype=torch.int32, device="cuda")
    engine.snappy_uncompress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_caps, out_lens, status)
    host = bytes(d_out.cpu().numpy())
    st, ol = status.cpu().numpy(), out_lens.cpu().numpy()
    return [(int(st[i]), host[ooffs[i]:ooffs[i] + ol[i]] if st[i] == 0 else b"") for i in range(len(streams))]


def test_batch_compress_matches_oracle_and_an_independent_decoder(engine, oracle_mod):
    pa = pytest.importorskip("pyarrow")
    inputs = snappy_cases(seed=21, extra=40)
    got = _compress_batch(engine, inputs)
    for i, (d, c) in enumerate(zip(inputs, got)):
        assert c == oracle_mod.snappy_compress(d), (i, len(d), len(c))
        if d:
            assert pa.decompress(c, decompressed_size=len(d), codec="snappy", asbytes=True) == d, i


def test_batch_compress_window_shapes(engine, oracle_mod):
    """the input families of the host model's test (tests/test_snappy_window_sim.py): in-window
    repeats, literal runs around the stride-1 limit, sparse matches, runs, every edge size --
    as single fragments and glued into multi-fragment streams"""
    from test_snappy_window_sim import _inputs
    frags = _inputs(7, 260)
    rnd = random.Random(8)
    glued = [b"".join(rnd.choice(frags) for _ in range(rnd.randrange(2, 6))) for _ in range(40)]
    inputs = frags + glued
    got = _compress_batch(engine, inputs)
    for i, (d, c) in enumerate(zip(inputs, got)):
        assert c == oracle_mod.snappy_compress(d), (i, len(d), len(c))


def test_dropin_compress_iov_segments(engine, oracle_mod):
    rnd = random.Random(3)
    data = W.gen_json(300001, 3)
    cuts = sorted(rnd.sample(range(1, len(data)), 9))
    segs = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
    err, c = engine.rd_kafka_snappy_compress_iov(segs)
    assert err == 0 and c == oracle_mod.snappy_compress(data)
    for d in (b"", b"x", b"hello world" * 3, bytes(70000)):
        assert engine.rd_kafka_snappy_compress_iov(d) == (0, oracle_mod.snappy_compress(d))


def test_batch_uncompress_own_and_foreign_streams(engine, oracle_mod):
    pa = pytest.importorskip("pyarrow")
    inputs = snappy_cases(seed=22, extra=30)
    own = [oracle_mod.snappy_compress(d) for d in inputs]
    foreign = [pa.compress(d, codec="snappy", asbytes=True) if d else b"\x00" for d in inputs]
    for streams in (own, foreign):
        res = _uncompress_batch(engine, streams)
        for i, (d, (st, out)) in enumerate(zip(inputs, res)):
            assert st == 0 and out == d, (i, st, len(d), len(out))


def test_uncompress_streams_that_do_not_split(engine, oracle_mod):
    """valid streams no compressor of 64 KiB fragments would make: a copy that reaches into the
    previous 64 KiB of output, an element that crosses a multiple of 64 KiB, more than 64
    fragments -- the parse-only pass must hand them to the serial decoder -- next to split ones"""
    pa = pytest.importorskip("pyarrow")
    rnd = random.Random(31)

    def varint(n):
        out = bytearray()
        while n >= 128:
            out.append((n & 127) | 128)
            n >>= 7
        out.append(n)
        return bytes(out)

    def literal(b):
        n = len(b) - 1
        if n < 60:
            return bytes([n << 2]) + b
        k = (n.bit_length() + 7) // 8
        return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + b

    a = rnd.randbytes(65536)
    b = W.gen_json(70000, 5)
    reach = varint(65536 + 8) + literal(a) + bytes([2 | (7 << 2), 100, 0])          # copy2 len 8 off 100
    cross = varint(70000) + literal(b)                                               # one literal over the boundary
    cross2 = varint(65536 + 40) + literal(a[:65530]) + bytes([2 | (45 << 2), 9, 0])  # copy over the boundary
    big = oracle_mod.snappy_compress(W.gen_json(65 * 65536 + 5, 6))                  # 66 fragments
    ok = oracle_mod.snappy_compress(W.gen_json(5 * 65536 + 77, 7))                   # splits
    streams = [reach, cross, cross2, big, ok]
    want = [oracle_mod.snappy_uncompress(x) for x in streams]
    assert all(w[0] == 0 for w in want)
    assert want[0][1] == a + a[65436:65444] and want[1][1] == b
    for x, w in zip(streams[:3], want[:3]):
        assert pa.decompress(x, decompressed_size=len(w[1]), codec="snappy", asbytes=True) == w[1]
    assert _uncompress_batch(engine, streams) == want


def test_uncompress_element_streams(engine, oracle_mod):
    """streams assembled element by element (tests/snappy_streams.py): every tag kind and
    literal-length encoding, lengths and offsets at their limits; fenced ones keep every element
    and copy inside a 64 KiB fragment of the output (they decode by fragments), the others do
    not, a quarter are damaged or cut short -- one batch, verdict and payload as the oracle's"""
    from snappy_streams import FRAG, stream
    rnd = random.Random(41)
    streams = []
    for it in range(240):
        total = rnd.choice([rnd.randrange(1, 3000), rnd.randrange(FRAG - 300, FRAG + 300),
                            rnd.randrange(FRAG, 4 * FRAG), 2 * FRAG, 3 * FRAG + 1])
        st, _ = stream(rnd, total, rnd.random() < 0.6, rnd.random() < 0.2)
        if it % 8 == 6:
            b = bytearray(st)
            for _ in range(rnd.randrange(1, 4)):
                b[rnd.randrange(3, len(b)) if len(b) > 3 else 0] = rnd.getrandbits(8)
            st = bytes(b)
        elif it % 8 == 7 and len(st) > 4:
            st = st[:rnd.randrange(3, len(st))]
        n = oracle_mod.snappy_uncompressed_length(st)
        if n is not None and n <= (1 << 23):
            streams.append(st)
    want = [oracle_mod.snappy_uncompress(s) for s in streams]
    assert sum(w[0] == 0 for w in want) > 150 and sum(w[0] != 0 for w in want) > 20
    res = _uncompress_batch(engine, streams)
    for i, ((st, out), (err, exp)) in enumerate(zip(res, want)):
        assert (st == 0) == (err == 0), (i, st, err)
        if err == 0:
            assert out == exp, i
        else:
            assert st == engine.SNAPPY_E_IO, (i, st)


def test_uncompress_copies_around_the_history_ring_edge(engine, oracle_mod):
    """copies whose sources lie just inside and just outside the decoder's on-chip history
    (4 KiB per wavefront, written out in 1 KiB pieces): offsets 4096 +- a few and down to a
    piece written moments ago; the oracle decides what each stream decodes to"""
    from snappy_streams import copy, literal, varint
    rnd = random.Random(78)
    streams = []
    for base in (3000, 4096, 5000, 9000, 20000):
        body = bytearray(literal(rnd, rnd.randbytes(base), False))
        pos = base
        for off in (4090, 4094, 4095, 4096, 4097, 4098, 4100, 4160, 3072, 3071, 3073, 5120, 2048, 1024,
                    1025, 1023, 8191, 8192, 12000):
            for length in (1, 4, 7, 19, 63, 64):
                if off > pos:
                    continue
                if rnd.random() < 0.5:
                    lit = rnd.randbytes(rnd.choice((1, 3, 17)))
                    body += literal(rnd, lit, False)
                    pos += len(lit)
                body += copy(rnd, length, off, 2)
                pos += length
        streams.append(varint(pos) + bytes(body))
    want = [oracle_mod.snappy_uncompress(st) for st in streams]
    assert all(w[0] == 0 for w in want)
    for i, ((st, out), (err, exp)) in enumerate(zip(_uncompress_batch(engine, streams), want)):
        assert st == 0 and out == exp, i


def test_uncompress_unaligned_destinations(engine, oracle_mod):
    """outputs at every byte alignment with guard bytes between them (single- and
    multi-fragment streams): the bytes arrive and nothing next to them is touched"""
    import torch
    rnd = random.Random(78)
    sizes = [1, 15, 16, 17, 1023, 1024, 1025, 4097, 65535, 65536, 65537, 131072, 200003, 3 * 65536 + 9] + \
            [rnd.randrange(1, 300000) for _ in range(26)]
    inputs = [W.gen_json(n, 200 + i) if i % 4 else (rnd.randbytes(5) * (n // 5 + 1))[:n]
              for i, n in enumerate(sizes)]
    streams = [oracle_mod.snappy_compress(b) for b in inputs]
    hbuf, hoffs = _pack(streams)
    d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    in_offs = torch.tensor(hoffs, dtype=torch.int64, device="cuda")
    in_lens = torch.tensor([len(b) for b in streams], dtype=torch.int32, device="cuda")
    doffs, pos = [], 0
    for i, b in enumerate(inputs):
        pos += 1 + (i * 7) % 16
        doffs.append(pos)
        pos += len(b)
    total = pos + 64
    d_out = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    out_offs = torch.tensor(doffs, dtype=torch.int64, device="cuda")
    out_caps = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
    out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
    status = torch.full((len(inputs),), 77, dtype=torch.int32, device="cuda")
    engine.snappy_uncompress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_caps, out_lens, status)
    st, ol = status.cpu().numpy(), out_lens.cpu().numpy()
    host = bytes(d_out.cpu().numpy())
    want = bytearray(b"\xa5" * total)
    for o, b in zip(doffs, inputs):
        want[o:o + len(b)] = b
    assert (st == 0).all() and (ol == [len(b) for b in inputs]).all()
    assert host == bytes(want)


def test_uncompress_verdicts_on_damaged_streams(engine, oracle_mod):
    rnd = random.Random(9)
    base = [W.gen_json(5000, 4), bytes(3000) + W.gen_json(2000, 1), (rnd.randbytes(100) * 60)]
    streams = []
    for d in base:
        c = oracle_mod.snappy_compress(d)
        for _ in range(150):
            m = bytearray(c)
            k = rnd.randrange(4)
            if k == 0:
                m = m[:rnd.randrange(len(m))]
            elif k == 1:
                m += rnd.randbytes(rnd.randrange(1, 4))
            else:
                for _ in range(rnd.randrange(1, 4)):
                    m[rnd.randrange(len(m))] = rnd.randrange(256)
            streams.append(bytes(m))
    # hand-made: every element form, and every way to fail
    streams += [bytes([70]) + bytes([60 << 2, 69]) + bytes(range(70)),
                bytes([8, 0]) + b"a" + bytes([1 | (3 << 2), 1]),
                bytes([12, 3 << 2]) + b"abcd" + bytes([2 | (7 << 2), 4, 0]),
                bytes([12, 3 << 2]) + b"abcd" + bytes([3 | (7 << 2), 4, 0, 0, 0]),
                bytes([8, 0]) + b"a" + bytes([1 | (3 << 2), 0]),
                bytes([8, 0]) + b"a" + bytes([1 | (3 << 2), 2]),
                bytes([8, 0]) + b"a" + bytes([1 | (3 << 2)]),
                bytes([9, 0]) + b"a" + bytes([1 | (3 << 2), 1]),
                bytes([7, 0]) + b"a" + bytes([1 | (3 << 2), 1]),
                bytes([2, 1 << 2]) + b"a", bytes([0]), bytes([0, 0, 0x61])]
    caps = []
    want = []
    for s in streams:
        n = oracle_mod.snappy_uncompressed_length(s)
        caps.append(min(n, 1 << 24) if n is not None else 0)
        err, out = oracle_mod.snappy_uncompress(s)
        want.append((err, out))
    keep = [i for i, s in enumerate(streams) if len(s) and caps[i] <= (1 << 23)]
    res = _uncompress_batch(engine, [streams[i] for i in keep], [caps[i] for i in keep])
    bad = 0
    for j, i in enumerate(keep):
        st, out = res[j]
        err, exp = want[i]
        assert (st == 0) == (err == 0), (i, streams[i][:40].hex(), st, err)
        if err == 0:
            assert out == exp, i
        else:
            assert st == engine.SNAPPY_E_IO, (i, st)
            bad += 1
    assert bad > 100


def test_dropin_reader_case_bare_and_snappy_java(engine, oracle_mod):
    a, b, c3 = W.gen_json(70000, 1), W.gen_json(123, 2), W.gen_json(40000, 3)
    ca, cb, cc = (oracle_mod.snappy_compress(x) for x in (a, b, c3))
    assert engine.rd_kafka_snappy_decompress(ca) == (0, a)
    hdr = b"\x82SNAPPY\x00" + struct.pack(">II", 1, 1)
    framed = hdr + b"".join(struct.pack(">I", len(x)) + x for x in (ca, cb, cc))
    assert engine.rd_kafka_snappy_decompress(framed) == (0, a + b + c3)
    for damaged in (framed + b"\x00", framed[:-1], hdr + struct.pack(">I", 1) + b"\x00",
                    b"\xff\xff\xff\xff\xff", framed[:40] + b"\x00" + framed[41:]):
        got = engine.rd_kafka_snappy_decompress(damaged)
        assert got == oracle_mod.rdk_snappy_decompress(damaged), damaged[:24].hex()


def test_roundtrip_at_scale(engine):
    """64 x 1 MiB JSON through compress -> uncompress on the device (property check at the
    bench's size; the oracle comparison above covers the bytes)."""
    import torch
    n = 64
    src, offs, lens = (None, None, None)
    data = [W.gen_json(1 << 20, 100 + i) for i in range(4)]
    inputs = [data[i % 4] for i in range(n)]
    streams = _compress_batch(engine, inputs)
    res = _uncompress_batch(engine, streams)
    for i in range(n):
        assert res[i] == (0, inputs[i]), i
    assert torch.cuda.is_available()
