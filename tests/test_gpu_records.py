"""GPU parity for MsgVersion 2 record serialisation (csrc/records.hip) against
the oracle restatement of rdkafka_msgset_writer.c, byte for byte."""
import numpy as np
import pytest

import librdkafka_amd as E
from librdkafka_amd import workload as W

pytestmark = pytest.mark.gpu


def _dev(m):
    import torch
    d = {}
    for k, v in m.items():
        a = v.view(np.int64) if v.dtype == np.uint64 else (v.view(np.int32) if v.dtype == np.uint32 else v)
        d[k] = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return d


def _batches(spec):
    b = np.zeros(len(spec), dtype=E.V2_BATCH_DTYPE)
    for i, (first, cnt) in enumerate(spec):
        b[i] = (first, cnt, 1000 + i, 7 * i - 1, i % 3, 0)
    return b


@pytest.mark.parametrize("headers", [True, False])
def test_v2_build_matches_oracle(engine, oracle_mod, headers):
    m = W.gen_messages(5000, seed=3, headers=headers)
    if not headers:
        m.pop("hdr_off"); m.pop("hdr_len"); m.pop("hdr_cnt")
    spec = [(0, 1), (1, 2), (3, 300), (303, 1), (304, 64), (368, 65), (433, 1000),
            (1433, 257), (1690, 3310)]
    b = _batches(spec)
    out, offs, sizes, crcs = E.msgset_v2_build(_dev(m), b, crc=True)
    host = bytes(out.cpu().numpy())
    offs, sizes, crcs = offs.cpu().numpy(), sizes.cpu().numpy(), crcs.cpu().numpy().view(np.uint32)
    for i, (first, cnt) in enumerate(spec):
        exp = oracle_mod.msgset_v2_write(m, first, cnt, 1000 + i, i % 3, 7 * i - 1, 0)
        got = host[offs[i]:offs[i] + sizes[i]]
        assert len(got) == len(exp), (i, len(got), len(exp))
        assert got == exp, (i, next(j for j in range(len(exp)) if got[j] != exp[j]))
        assert crcs[i] == int.from_bytes(exp[17:21], "big")


def test_v2_build_record_size_mix(engine, oracle_mod):
    """keys, values and header blocks of every length around the 16-byte copy unit, and records
    large enough that a chunk of 256 takes many passes of the on-chip tile (values of 1000 to
    70000 bytes, one of 1.5 MB that is many tiles long by itself), at every alignment of the
    arena and of the batch in the output"""
    rnd = np.random.default_rng(5)
    n = 2200
    sizes_v = [0, 1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 49, 100, 255, 256, 1000, 4096, 20000, 70000]
    arena = bytearray(rnd.integers(0, 256, 3, dtype=np.uint8).tobytes())
    m = {k: np.zeros(n, t) for k, t in (("ts", np.int64), ("key_off", np.uint64), ("key_len", np.int32),
                                        ("val_off", np.uint64), ("val_len", np.int32),
                                        ("hdr_off", np.uint64), ("hdr_len", np.uint32),
                                        ("hdr_cnt", np.int32))}
    for i in range(n):
        m["ts"][i] = 1600000000000 + int(rnd.integers(-5, 40))
        # the first 700 records stay small (chunks inside the tile), the rest mix in large ones
        pool = sizes_v[:13] if i < 700 else sizes_v
        kl = int(rnd.choice([-1, 0, 3, 15, 16, 17, 40, 200]))
        vl = int(rnd.choice(pool)) if i % 9 else -1
        if i == 1600:
            vl = 1500007
        m["key_len"][i] = kl
        if kl > 0:
            m["key_off"][i] = len(arena)
            arena += rnd.integers(0, 256, kl, dtype=np.uint8).tobytes()
        m["val_len"][i] = vl
        if vl > 0:
            m["val_off"][i] = len(arena)
            arena += rnd.integers(0, 256, vl, dtype=np.uint8).tobytes()
        if i % 4 == 0:  # one header, name "h", value of hv bytes (varint lengths as on the wire)
            hv = int(rnd.choice([0, 5, 12, 13, 14, 60]))
            h = bytes([2, ord("h"), hv << 1]) + rnd.integers(0, 256, hv, dtype=np.uint8).tobytes()
            m["hdr_off"][i] = len(arena)
            m["hdr_len"][i] = len(h)
            m["hdr_cnt"][i] = 1
            arena += h
    m["arena"] = np.frombuffer(bytes(arena), np.uint8).copy()
    spec = [(0, 1), (1, 255), (256, 257), (513, 187), (700, 300), (1000, 1), (1001, 513), (1514, 686)]
    b = _batches(spec)
    out, offs, sizes, crcs = E.msgset_v2_build(_dev(m), b, crc=True)
    host = bytes(out.cpu().numpy())
    offs, sizes, crcs = offs.cpu().numpy(), sizes.cpu().numpy(), crcs.cpu().numpy().view(np.uint32)
    for i, (first, cnt) in enumerate(spec):
        exp = oracle_mod.msgset_v2_write(m, first, cnt, 1000 + i, i % 3, 7 * i - 1, 0)
        got = host[offs[i]:offs[i] + sizes[i]]
        assert len(got) == len(exp), (i, len(got), len(exp))
        assert got == exp, (i, next(j for j in range(len(exp)) if got[j] != exp[j]))
        assert crcs[i] == int.from_bytes(exp[17:21], "big")


def test_v2_build_then_verify(engine):
    """The built batches pass the engine's own CRC verify (reader side)."""
    import torch
    m = W.gen_messages(20000, seed=9)
    spec = [(i * 1000, 1000) for i in range(20)]
    out, offs, sizes, _ = E.msgset_v2_build(_dev(m), _batches(spec), crc=True)
    st = torch.zeros(len(spec), dtype=torch.int32, device="cuda")
    E.msgset_v2_crc(out, offs, sizes, st, E.V2_CRC_VERIFY)
    assert int(st.abs().sum()) == 0


def _index(engine, batches_bytes, rec_lens=None, caps=None):
    """Index host-built v2 batches on the GPU; returns (count, rows) on the host."""
    import torch
    blob = b"".join(batches_bytes)
    offs = np.cumsum([0] + [len(b) for b in batches_bytes[:-1]]).astype(np.int64)
    lens = np.array([len(b) - 61 for b in batches_bytes], np.int64)
    if rec_lens is not None:
        lens = np.array(rec_lens, np.int64)
    dev = torch.frombuffer(bytearray(blob + b"\0" * 64), dtype=torch.uint8).cuda()
    n = len(batches_bytes)
    nrows = [max(1, int(l) // 6 + 1) for l in lens]
    if caps is None:
        caps = nrows
    row_offs = np.cumsum([0] + nrows[:-1]).astype(np.int64)
    tot = int(sum(nrows))
    rows = {k: torch.zeros(tot, dtype=getattr(torch, t), device="cuda")
            for k, t in E.V2_ROW_FIELDS}
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    t = lambda a, dt: torch.from_numpy(np.asarray(a, dtype=dt)).cuda()  # noqa: E731
    E.msgset_v2_index(dev, t(offs, np.int64), dev, t(offs + 61, np.int64), t(lens, np.int32),
                      t(row_offs, np.int64), t(caps, np.int32), rows, cnt)
    host = {k: v.cpu().numpy() for k, v in rows.items()}
    return cnt.cpu().numpy(), host, row_offs


def _check_index(oracle_mod, b, cnt, host, r0, rec_len=None):
    import struct
    rec = b[61:61 + (rec_len if rec_len is not None else len(b) - 61)]
    bo, bts = struct.unpack(">q", b[:8])[0], struct.unpack(">q", b[27:35])[0]
    n, exp = oracle_mod.msgset_v2_index(rec, bo, bts)
    assert cnt == n, (cnt, n)
    for k in exp:
        assert (host[k][r0:r0 + max(n, 0)].astype(np.int64) ==
                exp[k].astype(np.int64)).all(), k


def test_v2_index_matches_oracle(engine, oracle_mod):
    m = W.gen_messages(6000, seed=11)
    spec = [(0, 1), (1, 500), (501, 2000), (2501, 3499)]
    bs = [oracle_mod.msgset_v2_write(m, f, c, 5, 1, 0, 0) for f, c in spec]
    bs[2] = bs[2][:8] + bytes(8) + bs[2][16:]  # header BaseOffset stays 0; arbitrary
    cnt, host, r0 = _index(engine, bs)
    for i, b in enumerate(bs):
        _check_index(oracle_mod, b, cnt[i], host, r0[i])


def test_v2_index_big_records_and_errors(engine, oracle_mod):
    m = W.gen_messages(40, seed=5)
    # one 20 KiB value (larger than the 8 KiB LDS window)
    big = np.frombuffer(bytes(range(256)) * 80, np.uint8)
    m["val_off"][7] = len(m["arena"]); m["val_len"][7] = len(big)
    m["arena"] = np.concatenate([m["arena"], big])
    ok = oracle_mod.msgset_v2_write(m, 0, 40)
    trunc = ok[:-5]                                    # last record cut short
    bad_len = bytearray(ok); bad_len[61] |= 0x80       # first Length varint runs on
    bad_len = bytes(bad_len)
    empty = oracle_mod.msgset_v2_write(m, 0, 1)[:61]   # no records at all
    bs = [ok, trunc, bad_len, empty, ok]
    cnt, host, r0 = _index(engine, bs, caps=[1000, 1000, 1000, 1, 10])
    for i in range(4):
        _check_index(oracle_mod, bs[i], cnt[i], host, r0[i])
    assert cnt[4] == -(1 + 10)                          # row capacity 10: record 10 fails


def test_v2_index_large_batches(engine, oracle_mod):
    """~1 MiB batches (many LDS windows, records ending exactly at window edges)."""
    m = W.gen_messages(19000, seed=21)
    bs = [oracle_mod.msgset_v2_write(m, 0, 9500), oracle_mod.msgset_v2_write(m, 9500, 9500)]
    cnt, host, r0 = _index(engine, bs)
    for i, b in enumerate(bs):
        _check_index(oracle_mod, b, cnt[i], host, r0[i])


def test_v2_index_adversarial_payloads(engine, oracle_mod):
    """Values that are themselves v2 record streams (or runs of 0x00 / 0x02 bytes): the
    speculative segment guesses land inside values and must be rejected by the path check,
    leaving rows identical to the oracle's."""
    inner = oracle_mod.msgset_v2_write(W.gen_messages(300, seed=2), 0, 300)[61:]
    vals = [inner, inner[:4000], bytes(700), b"\x02\x00" * 400, inner[17:9000]]
    arena = np.frombuffer(b"".join(vals * 30), dtype=np.uint8)
    n = len(vals) * 30
    lens = np.array([len(v) for v in vals] * 30, dtype=np.int32)
    m = {"arena": arena, "ts": np.arange(n, dtype=np.int64) * 3,
         "key_off": np.zeros(n, dtype=np.uint64), "key_len": np.full(n, -1, dtype=np.int32),
         "val_off": np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64),
         "val_len": lens}
    bs = [oracle_mod.msgset_v2_write(m, 0, n), oracle_mod.msgset_v2_write(m, 3, n - 3)]
    cnt, host, r0 = _index(engine, bs)
    for i, b in enumerate(bs):
        _check_index(oracle_mod, b, cnt[i], host, r0[i])
