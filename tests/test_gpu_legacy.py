"""GPU parity for the MsgVersion 0/1 CRC-32 path (csrc/legacy.hip, csrc/crc32c.hip with the
CRC-32 image) against the oracle and zlib (the reference's own CRC-32, rdcrc32.h WITH_ZLIB)."""
import struct
import zlib

import numpy as np
import pytest

import librdkafka_amd as E
from librdkafka_amd import workload as W

pytestmark = pytest.mark.gpu


def test_crc32_ranges_match_zlib(engine):
    import torch
    rng = np.random.default_rng(8)
    data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    lens = [0, 1, 3, 15, 16, 17, 255, 4096, 100000, 1 << 20, 65537] + \
        list(rng.integers(0, 20000, 300))
    offs = [int(rng.integers(0, len(data) - l)) for l in lens]
    base = torch.from_numpy(data).cuda()
    o = torch.tensor(offs, dtype=torch.int64, device="cuda")
    ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = torch.zeros(len(lens), dtype=torch.int32, device="cuda")
    E.crc32_ranges(base, o, ln, out)
    got = out.cpu().numpy().view(np.uint32)
    for i, (a, l) in enumerate(zip(offs, lens)):
        assert got[i] == zlib.crc32(data[a:a + l].tobytes()), i


def test_rd_slice_crc32_matches_zlib(engine):
    rng = np.random.default_rng(1)
    segs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (5, 0, 70000, 13, 1 << 18)]
    assert E.rd_slice_crc32(segs) == zlib.crc32(b"".join(segs))
    assert E.rd_slice_crc32([b""]) == 0


def _run(sets, mode, caps=None, align=None):
    """Lay the sets out in one device buffer (odd alignments), run the kernel, return
    (count, [(pos, out) per set], buffer after)."""
    import torch
    rng = np.random.default_rng(len(sets))
    offs, cur = [], 0
    for i, s in enumerate(sets):
        cur += int(rng.integers(0, 16)) if align is None else align
        offs.append(cur)
        cur += len(s)
    buf = np.zeros(cur + 64, dtype=np.uint8)
    for o, s in zip(offs, sets):
        buf[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    caps = caps or [max(1, len(s) // 18 + 1) for s in sets]
    roffs = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    d = torch.from_numpy(buf).cuda()
    t = lambda a, dt: torch.tensor(a, dtype=dt, device="cuda")
    pos = torch.zeros(int(sum(caps)), dtype=torch.int32, device="cuda")
    out = torch.zeros(int(sum(caps)), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(len(sets), dtype=torch.int32, device="cuda")
    E.msgset_v01_crc(d, t(offs, torch.int64), t([len(s) for s in sets], torch.int32),
                     t(roffs, torch.int64), t(caps, torch.int32), pos, out, cnt, mode)
    torch.cuda.synchronize()
    cnt, pos = cnt.cpu().numpy(), pos.cpu().numpy().view(np.uint32)
    out, after = out.cpu().numpy().view(np.uint32), d.cpu().numpy()
    rows = []
    for i in range(len(sets)):
        k = cnt[i] if cnt[i] >= 0 else -cnt[i] - 1
        rows.append((pos[roffs[i]:roffs[i] + k], out[roffs[i]:roffs[i] + k]))
    return cnt, rows, [bytes(after[o:o + len(s)]) for o, s in zip(offs, sets)], caps


def _check(oracle_mod, sets, mode, **kw):
    cnt, rows, after, caps = _run(sets, mode, **kw)
    for i, s in enumerate(sets):
        n, pos, out, exp_after = oracle_mod.msgset_v01_crc(s, mode, max_rows=caps[i])
        assert cnt[i] == n, (i, cnt[i], n)
        assert (rows[i][0] == pos).all(), i
        assert (rows[i][1] == out).all(), (i, np.nonzero(rows[i][1] != out)[0][:5])
        assert after[i] == exp_after, i
    return cnt


def _sets(oracle_mod, seed, n_sets=12, per=3000):
    m = W.gen_messages(n_sets * per, seed=seed)
    return [oracle_mod.msgset_v01_write(m, i * per, per, magic=i % 2, base_offset=i << 20)
            for i in range(n_sets)]


@pytest.mark.parametrize("mode", [E.V2_CRC_COMPUTE, E.V2_CRC_FINALIZE, E.V2_CRC_VERIFY])
def test_v01_sets_match_oracle(engine, oracle_mod, mode):
    sets = _sets(oracle_mod, 3)
    if mode == E.V2_CRC_FINALIZE:   # blank Crc fields: FINALIZE must restore them
        blank = []
        for s in sets:
            b, p = bytearray(s), 0
            while p < len(b):
                b[p + 12:p + 16] = b"\0\0\0\0"
                p += 12 + struct.unpack_from(">i", b, p + 8)[0]
            blank.append(bytes(b))
        cnt, _, after, _ = _run(blank, mode)
        assert after == sets
        sets = blank
    if mode == E.V2_CRC_VERIFY:     # corrupt a few Crc / payload bytes
        b = bytearray(sets[1])
        for p in (12, 40000, 70001):
            b[p] ^= 0x40
        sets[1] = bytes(b)
    _check(oracle_mod, sets, mode)


def test_v01_edges(engine, oracle_mod):
    m = W.gen_messages(5000, seed=6)
    s0 = oracle_mod.msgset_v01_write(m, 0, 2000, magic=0)
    s1 = oracle_mod.msgset_v01_write(m, 2000, 3000, magic=1)
    pos1 = oracle_mod.msgset_v01_crc(s1, 0)[1]
    sets = [b"", s0[:1], s0[:30], s1[:pos1[-1] + 20], s1[:131072], s1[:131072 + 7]]
    for k, v in ((0, 5), (1500, 13), (2999, -7), (100, 3)):
        b = bytearray(s1)
        struct.pack_into(">i", b, int(pos1[k]) + 8, v)
        sets.append(bytes(b))
    for cut in (16, 17, 25):
        sets.append(s1[:int(pos1[2500]) + cut])
    _check(oracle_mod, sets, E.V2_CRC_COMPUTE)
    # row caps
    _check(oracle_mod, [s0, s1, s1], E.V2_CRC_COMPUTE, caps=[2000, 1999, 1])


def test_v01_big_messages(engine, oracle_mod):
    """Messages larger than the 128 KiB window (whole-workgroup path) between small ones."""
    rng = np.random.default_rng(12)
    sizes = [40, 300000, 17, 131072 - 30, 131072 - 28, 131072, 1 << 20, 5, 200, 70000, 70000]
    arena = rng.integers(0, 256, sum(sizes) + 10, dtype=np.uint8)
    n = len(sizes)
    m = {"arena": arena, "ts": np.arange(n, dtype=np.int64) * 7,
         "key_off": np.zeros(n, dtype=np.uint64), "key_len": np.full(n, -1, dtype=np.int32),
         "val_off": np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64),
         "val_len": np.array(sizes, dtype=np.int32)}
    sets = [oracle_mod.msgset_v01_write(m, 0, n, magic=1),
            oracle_mod.msgset_v01_write(m, 3, 5, magic=0)]
    _check(oracle_mod, sets, E.V2_CRC_COMPUTE)
    _check(oracle_mod, sets, E.V2_CRC_VERIFY)


def test_v01_adversarial_payloads(engine, oracle_mod):
    """Values that are themselves valid MessageSets, all-zero, or all-0x01: the speculative
    segment guesses land inside payloads and must be rejected by the path check."""
    inner = oracle_mod.msgset_v01_write(W.gen_messages(400, seed=1), 0, 400, magic=1)
    vals = [inner[:n] for n in (len(inner), 5000, 301)] + [bytes(900), b"\x01" * 700,
                                                          inner[34:9000]]
    arena = np.frombuffer(b"".join(vals * 40), dtype=np.uint8)
    n = len(vals) * 40
    lens = np.array([len(v) for v in vals] * 40, dtype=np.int32)
    m = {"arena": arena, "ts": np.arange(n, dtype=np.int64),
         "key_off": np.zeros(n, dtype=np.uint64), "key_len": np.full(n, -1, dtype=np.int32),
         "val_off": np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64),
         "val_len": lens}
    sets = [oracle_mod.msgset_v01_write(m, 0, n, magic=1),
            oracle_mod.msgset_v01_write(m, 1, n - 1, magic=0)]
    _check(oracle_mod, sets, E.V2_CRC_VERIFY)
