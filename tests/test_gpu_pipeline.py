"""The writer's and the reader's device paths end to end, chained through the C ABI as a
broker thread would chain them:

  messages --rdk_hip_msgset_v2_sizes/_write--> MessageSets --rdk_hip_msgset_v2_finalize-->
  finished batches (rdkafka_msgset_writer.c:652-754, :1117-1207, :1229-1295)
  --rdk_hip_msgset_v2_crc VERIFY--> codec from Attributes --decompress--> records
  --rdk_hip_msgset_v2_index--> rows (rdkafka_msgset_reader.c:982-1015, :258-533, :715-927)

Every stage is compared with the oracle elsewhere; here the finished batches are compared
with the oracle's writer + codec + CRC as a whole, and the rows that come out at the far end
with the messages that went in."""
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


@pytest.mark.parametrize("mode", [E.PRODUCER_EXACT, E.PRODUCER_FAST, 2])
def test_messages_to_batches_to_rows(engine, oracle_mod, mode):
    import torch
    m = W.gen_messages(12000, seed=77)
    spec = [(0, 1), (1, 700), (701, 2999), (3700, 64), (3764, 8236)]
    b = np.zeros(len(spec), dtype=E.V2_BATCH_DTYPE)
    for i, (first, cnt) in enumerate(spec):
        b[i] = (first, cnt, 5000 + 10 * i, -1, -1, 0)  # ProducerId, BaseSequence, Epoch, Attributes
    n = len(spec)
    d = _dev(m)
    # ---- writer: records, then compress + header finalize + CRC32C
    sets, offs, sizes, _ = E.msgset_v2_build(d, b, crc=False)
    rec_offs = offs + 61
    rec_lens = sizes - 61
    bound = E.snappy_max_compressed_length if mode == 2 else E.lz4f_compress_bound
    caps = [(61 + bound(int(x)) + 255) // 256 * 256 for x in rec_lens.cpu().numpy()]
    out_offs = torch.tensor(np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64), device="cuda")
    out_caps = torch.tensor(np.asarray(caps, np.int32), device="cuda")
    out = torch.zeros(int(sum(caps)) + 256, dtype=torch.uint8, device="cuda")
    flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    E.msgset_v2_finalize(sets, rec_offs, rec_lens, out, out_offs, out_caps, flens, blens, crcs, mode=mode)
    host = bytes(out.cpu().numpy())
    oo, bl = out_offs.cpu().numpy(), blens.cpu().numpy()
    plain = bytes(sets.cpu().numpy())
    so, ss = offs.cpu().numpy(), sizes.cpu().numpy()
    for i, (first, cnt) in enumerate(spec):
        # the oracle's whole writer: records, codec, verdict, header, CRC
        want_set = oracle_mod.msgset_v2_write(m, first, cnt, 5000 + 10 * i, -1, -1, 0)
        assert plain[so[i] + 61:so[i] + ss[i]] == want_set[61:], i
        got = host[oo[i]:oo[i] + bl[i]]
        recs = want_set[61:]
        if mode == E.PRODUCER_EXACT:
            err, frame = oracle_mod.rdk_lz4_compress(recs)
            assert err == 0
            payload, codec = (frame, 3) if len(frame) <= len(recs) else (recs, 0)
            assert got[61:] == payload, i
        elif mode == 2:
            comp = oracle_mod.snappy_compress(recs)
            payload, codec = (comp, 2) if len(comp) <= len(recs) else (recs, 0)
            assert got[61:] == payload, i
        else:
            codec = int.from_bytes(got[21:23], "big") & 7
            assert codec in (0, 3)
        assert int.from_bytes(got[21:23], "big") & 7 == codec
        assert int.from_bytes(got[8:12], "big") == len(got) - 12
        assert int.from_bytes(got[17:21], "big") == oracle_mod.crc32c(0, got[21:]), i
    # ---- reader: verify, decompress by the header's codec, index
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    E.msgset_v2_crc(out, out_offs, out_caps, st, E.V2_CRC_VERIFY)
    assert int(st.abs().sum()) == 0
    attrs = [int.from_bytes(host[oo[i] + 21:oo[i] + 23], "big") & 7 for i in range(n)]
    rl = rec_lens.cpu().numpy().astype(np.int64)
    doffs = torch.tensor(np.concatenate([[0], np.cumsum((rl + 255) // 256 * 256)[:-1]]).astype(np.int64),
                         device="cuda")
    dcaps = torch.tensor(((rl + 255) // 256 * 256).astype(np.int32), device="cuda")
    dec = torch.zeros(int(((rl + 255) // 256 * 256).sum()) + 256, dtype=torch.uint8, device="cuda")
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    pay_offs, pay_lens = out_offs + 61, blens - 61
    for codec, fn in ((3, E.lz4f_decompress_batch), (2, E.snappy_uncompress_batch)):
        sel = [i for i in range(n) if attrs[i] == codec]
        if not sel:
            continue
        ix = torch.tensor(sel, device="cuda")
        sl = torch.zeros(len(sel), dtype=torch.int32, device="cuda")
        ss_ = torch.zeros(len(sel), dtype=torch.int32, device="cuda")
        fn(out, pay_offs[ix].contiguous(), pay_lens[ix].contiguous(), dec, doffs[ix].contiguous(),
           dcaps[ix].contiguous(), sl, ss_)
        assert int(ss_.abs().sum()) == 0
        dl[ix] = sl
    for i in range(n):
        if attrs[i] == 0:  # sent plain
            dec[int(doffs[i]):int(doffs[i]) + int(rl[i])] = out[oo[i] + 61:oo[i] + 61 + int(rl[i])]
            dl[i] = int(rl[i])
    assert bool((dl.cpu() == rec_lens.cpu()).all())
    row_offs = torch.tensor(np.asarray([s[0] for s in spec], np.int64), device="cuda")
    row_caps = torch.tensor(np.asarray([s[1] for s in spec], np.int32), device="cuda")
    total = sum(c for _, c in spec)
    rows = {k: torch.zeros(total, dtype=getattr(torch, t), device="cuda") for k, t in E.V2_ROW_FIELDS}
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    E.msgset_v2_index(out, out_offs, dec, doffs, dl, row_offs, row_caps, rows, cnt)
    assert cnt.cpu().tolist() == [c for _, c in spec]
    r = {k: v.cpu().numpy() for k, v in rows.items()}
    decoded = dec.cpu().numpy()
    arena = m["arena"]
    do = doffs.cpu().numpy()
    rnd = np.random.default_rng(1)
    for i, (first, cnt_) in enumerate(spec):
        base_ts = int(m["ts"][first])
        for j in ([0, cnt_ - 1] + list(rnd.integers(0, cnt_, 40))):
            g = first + j
            assert r["offset"][g] == j  # BaseOffset 0 (the broker assigns it) + OffsetDelta
            assert r["timestamp"][g] == int(m["ts"][g]), (i, j, base_ts)
            for f in ("key", "val"):
                want_len = int(m[f + "_len"][g])
                assert r[f + "_len"][g] == want_len
                if want_len > 0:
                    p = int(do[i]) + int(r[f + "_off"][g])
                    o = int(m[f + "_off"][g])
                    assert bytes(decoded[p:p + want_len]) == bytes(arena[o:o + want_len])


def test_perf_tool_messages_through_writer_and_reader(engine, oracle_mod):
    """The workload of `rdkafka_performance -P -s 100 -z lz4` (examples/rdkafka_performance.c:798,
    :1318-1325): 100-byte messages of the repeated pattern, no key, cut into MessageSets by
    write_msgq's rule (batch.num.messages 10000, message.max.bytes 1000000,
    rdkafka_msgset_writer.c:859-863).  Every finished batch must equal the oracle's writer +
    the reference-identical LZ4F frame + CRC32C byte for byte, and the reader side must hand
    back the messages."""
    import torch
    m = W.gen_perf_messages(30000)
    spec = W.perf_batches(m)
    assert len(spec) == 4 and spec[0][1] > 9000 and sum(c for _, c in spec) == 30000
    n = len(spec)
    b = np.zeros(n, dtype=E.V2_BATCH_DTYPE)
    for i, (first, cnt) in enumerate(spec):
        b[i] = (first, cnt, -1, -1, -1, 0)
    d = _dev(m)
    sets, offs, sizes, _ = E.msgset_v2_build(d, b, crc=False)
    rec_offs, rec_lens = offs + 61, sizes - 61
    caps = [(61 + E.lz4f_compress_bound(int(x)) + 255) // 256 * 256 for x in rec_lens.cpu().numpy()]
    out_offs = torch.tensor(np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64), device="cuda")
    out_caps = torch.tensor(np.asarray(caps, np.int32), device="cuda")
    out = torch.zeros(int(sum(caps)) + 256, dtype=torch.uint8, device="cuda")
    flens, blens, crcs = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    E.msgset_v2_finalize(sets, rec_offs, rec_lens, out, out_offs, out_caps, flens, blens, crcs,
                         mode=E.PRODUCER_EXACT)
    host = bytes(out.cpu().numpy())
    oo, bl = out_offs.cpu().numpy(), blens.cpu().numpy()
    got_crcs = crcs.cpu().numpy().view(np.uint32)
    for i, (first, cnt) in enumerate(spec):
        want_set = oracle_mod.msgset_v2_write(m, first, cnt, -1, -1, -1, 0)
        assert len(want_set) <= 1000000 + 61
        err, frame = oracle_mod.rdk_lz4_compress(want_set[61:])
        assert err == 0 and len(frame) < len(want_set) - 61
        got = host[oo[i]:oo[i] + bl[i]]
        assert got[61:] == frame, i
        hdr = bytearray(want_set[:61])
        hdr[8:12] = (len(got) - 12).to_bytes(4, "big")
        hdr[21:23] = (int.from_bytes(hdr[21:23], "big") | 3).to_bytes(2, "big")
        crc = oracle_mod.crc32c(0, bytes(hdr[21:]) + frame)
        hdr[17:21] = crc.to_bytes(4, "big")
        assert got[:61] == bytes(hdr), i
        assert int(got_crcs[i]) == crc
    # the throughput compressor on the same MessageSets: decodable by the reference, ratio in bound
    out2 = torch.zeros_like(out)
    fl2, bl2, cr2 = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    E.msgset_v2_finalize(sets, rec_offs, rec_lens, out2, out_offs, out_caps, fl2, bl2, cr2,
                         mode=E.PRODUCER_FAST)
    host2 = bytes(out2.cpu().numpy())
    for i, (first, cnt) in enumerate(spec):
        want_set = oracle_mod.msgset_v2_write(m, first, cnt, -1, -1, -1, 0)
        got = host2[oo[i]:oo[i] + int(bl2[i])]
        assert int.from_bytes(got[17:21], "big") == oracle_mod.crc32c(0, got[21:])
        dec_ref = (oracle_mod.ref_rdk_lz4_decompress(got[61:], max_msg_size=1 << 30)[:2]
                   if oracle_mod.ref_available() else oracle_mod.rdk_lz4_decompress(got[61:]))
        assert dec_ref == (0, want_set[61:]), i
        assert len(got) - 61 <= 1.05 * int(flens[i]), (i, len(got) - 61, int(flens[i]))
    # ---- reader: check.crcs, decompress, record index
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    E.msgset_v2_crc(out, out_offs, out_caps, st, E.V2_CRC_VERIFY)
    assert int(st.abs().sum()) == 0
    rl = rec_lens.cpu().numpy().astype(np.int64)
    dslot = (rl + 255) // 256 * 256
    doffs = torch.tensor(np.concatenate([[0], np.cumsum(dslot)[:-1]]).astype(np.int64), device="cuda")
    dcaps = torch.tensor(dslot.astype(np.int32), device="cuda")
    dec = torch.zeros(int(dslot.sum()) + 256, dtype=torch.uint8, device="cuda")
    dl, ds = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(2))
    E.lz4f_decompress_batch(out, out_offs + 61, flens, dec, doffs, dcaps, dl, ds)
    assert int(ds.abs().sum()) == 0 and bool((dl == rec_lens).all())
    row_offs = torch.tensor(np.asarray([s[0] for s in spec], np.int64), device="cuda")
    row_caps = torch.tensor(np.asarray([s[1] for s in spec], np.int32), device="cuda")
    rows = {k: torch.zeros(30000, dtype=getattr(torch, t), device="cuda") for k, t in E.V2_ROW_FIELDS}
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    E.msgset_v2_index(out, out_offs, dec, doffs, dl, row_offs, row_caps, rows, cnt)
    assert cnt.cpu().tolist() == [c for _, c in spec]
    r = {k: v.cpu().numpy() for k, v in rows.items()}
    assert (r["timestamp"] == m["ts"]).all() and (r["val_len"] == 100).all() and (r["key_len"] == -1).all()
    want_off = np.concatenate([np.arange(c) for _, c in spec])
    assert (r["offset"] == want_off).all()
    decoded = dec.cpu().numpy()
    do = doffs.cpu().numpy()
    value = bytes(m["arena"][:100])
    for i, (first, c) in enumerate(spec):
        for j in (0, 1, c // 2, c - 1):
            p = int(do[i]) + int(r["val_off"][first + j])
            assert bytes(decoded[p:p + 100]) == value


def test_finalize_fast_on_the_units_engine(oracle_mod):
    """RDK_HIP_LZ4_FAST_ENGINE=units: rdk_hip_msgset_v2_finalize's FAST mode on the
    workgroup-per-block compressor, whose CRC32C comes from the batched CRC pass over the
    finished batches instead of the compress epilogue.  Own process: the engine choice is read
    once from the environment.  Every batch: header fields, CRC against the oracle, frame
    decoded by the reference decoder."""
    import os
    import subprocess
    import sys
    import textwrap
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        import numpy as np, torch
        import librdkafka_amd as E, oracle
        from librdkafka_amd import workload as W
        E.init(0)
        recs = [W.gen_json(n, 3 + i) for i, n in enumerate((1 << 20, 70000, 13, 5, 300000))] + \\
               [bytes(np.random.default_rng(1).integers(0, 256, 90000, dtype=np.uint8))]
        n = len(recs)
        stride = (61 + max(map(len, recs)) + 255) // 256 * 256
        src = torch.zeros(n * stride + 256, dtype=torch.uint8)
        for i, r in enumerate(recs):
            src[i * stride:i * stride + 61] = torch.frombuffer(bytearray(W.v2_header(i, 61 + len(r))), dtype=torch.uint8)
            src[i * stride + 61:i * stride + 61 + len(r)] = torch.frombuffer(bytearray(r), dtype=torch.uint8)
        src = src.cuda()
        rec_offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride + 61
        rec_lens = torch.tensor([len(r) for r in recs], dtype=torch.int32, device="cuda")
        cap = (61 + E.lz4f_compress_bound(max(map(len, recs))) + 255) // 256 * 256
        out = torch.zeros(n * cap + 256, dtype=torch.uint8, device="cuda")
        out_offs = torch.arange(n, dtype=torch.int64, device="cuda") * cap
        out_caps = torch.full((n,), cap, dtype=torch.int32, device="cuda")
        fl, bl, cr = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
        E.msgset_v2_finalize(src, rec_offs, rec_lens, out, out_offs, out_caps, fl, bl, cr, mode=E.PRODUCER_FAST)
        host = bytes(out.cpu().numpy())
        crcs = cr.cpu().numpy().view(np.uint32)
        for i, r in enumerate(recs):
            got = host[i * cap:i * cap + int(bl[i])]
            codec = int.from_bytes(got[21:23], "big") & 7
            assert int.from_bytes(got[8:12], "big") == len(got) - 12, i
            assert int.from_bytes(got[17:21], "big") == oracle.crc32c(0, got[21:]) == int(crcs[i]), i
            if codec == 3:
                assert oracle.rdk_lz4_decompress(got[61:]) == (0, r), i
            else:
                assert codec == 0 and got[61:] == r, i
        assert (int.from_bytes(host[21:23], "big") & 7) == 3 and (int.from_bytes(host[5 * cap + 21:5 * cap + 23], "big") & 7) == 0
        print("ok")
    """ % root)
    env = dict(os.environ, RDK_HIP_LZ4_FAST_ENGINE="units")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, (r.returncode, r.stdout, r.stderr[-3000:])
