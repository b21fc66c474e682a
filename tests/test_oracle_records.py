"""CPU checks of the MsgVersion 2 record oracle (oracle/msgset_oracle.c): the
varint codec against the reference's own known answers (rdvarint.c
unittest_rdvarint), and writer -> parser round trips."""
import struct

import numpy as np

from librdkafka_amd import workload as W


def test_varint_known_answers(oracle_mod, golden):
    for v in golden("varint_kat.json")["vectors"]:
        assert oracle_mod.varint_enc(v["num"]).hex() == v["hex"]
        assert oracle_mod.varint_dec(bytes.fromhex(v["hex"])) == (v["num"], len(v["hex"]) // 2)
    # truncated input fails (rdvarint.h RD_UVARINT_UNDERFLOW)
    assert oracle_mod.varint_dec(bytes.fromhex("f08d"))[1] == 0


def test_writer_header_fields_and_crc(oracle_mod):
    m = W.gen_messages(300)
    b = oracle_mod.msgset_v2_write(m, 10, 200, producer_id=77, producer_epoch=3,
                                   base_sequence=9, attributes=0)
    (base_off, length, epoch, magic, crc, attrs, lod, bts, mts, pid, pep, bseq,
     cnt) = struct.unpack(">qiibIhiqqqhii", b[:61])
    assert (base_off, length, magic, attrs, lod, pid, pep, bseq, cnt) == \
        (0, len(b) - 12, 2, 0, 199, 77, 3, 9, 200)
    assert bts == m["ts"][10] and mts == max(0, int(m["ts"][10:210].max()))
    assert crc == oracle_mod.crc32c(0, b[21:])          # writer.c:1235-1245


def test_writer_parser_round_trip(oracle_mod):
    m = W.gen_messages(2000)
    for first, cnt in ((0, 1), (0, 2000), (333, 777), (1999, 1)):
        b = oracle_mod.msgset_v2_write(m, first, cnt)
        bts = struct.unpack(">q", b[27:35])[0]
        n, rows = oracle_mod.msgset_v2_index(b[61:], base_offset=1000, base_ts=bts)
        assert n == cnt
        sl = slice(first, first + cnt)
        assert (rows["offset"] == 1000 + np.arange(cnt)).all()
        assert (rows["timestamp"] == m["ts"][sl]).all()
        assert (rows["key_len"] == m["key_len"][sl]).all()
        assert (rows["val_len"] == m["val_len"][sl]).all()
        # binhdrs = HeaderCount varint + headers (reader.c:876-878)
        hc = [len(oracle_mod.varint_enc(int(c))) for c in m["hdr_cnt"][sl]]
        assert (rows["hdr_len"] == m["hdr_len"][sl] + np.array(hc)).all()
        rec = b[61:]
        for i in range(0, cnt, 97):
            j = first + i
            vl = int(m["val_len"][j])
            if vl > 0:
                vo, so = int(rows["val_off"][i]), int(m["val_off"][j])
                assert rec[vo:vo + vl] == m["arena"][so:so + vl].tobytes()


def test_parser_rejects_truncation(oracle_mod):
    m = W.gen_messages(50)
    b = oracle_mod.msgset_v2_write(m, 0, 50)[61:]
    n, _ = oracle_mod.msgset_v2_index(b[:-3])
    assert n == -50                                      # record 49 fails
