"""snappy restatement (oracle/snappy_oracle.c; snappy.c:957-1103 compress_fragment,
:1226-1406 decoder, :1588 snappy-java framing).  PARITY UNPINNED against snappy.c itself
(it cannot be compiled here and the reference holds no snappy fixtures); what is pinned is
the format: pyarrow's bundled snappy, an independent implementation, decodes every stream
made here to the input, and streams made by it decode here to its input."""
import random
import struct

import pytest

from librdkafka_amd import workload as W

pa = pytest.importorskip("pyarrow")
if not pa.Codec.is_available("snappy"):
    pytest.skip("pyarrow without snappy", allow_module_level=True)


def snappy_cases(seed=5, extra=30):
    rnd = random.Random(seed)
    cases = [b"", b"a", b"hello world", W.gen_json(1 << 20, 42), W.gen_json(65536, 1),
             W.gen_json(65537, 2), W.gen_json(14, 3), W.gen_json(15, 3), W.gen_json(16, 3),
             bytes(200000), b"ab" * 50000, rnd.randbytes(100000),
             (rnd.randbytes(700) * 300)[:150000], b"x" * 65535]
    for _ in range(extra):
        n = rnd.choice([1, 5, 14, 15, 16, 17, 60, 61, 100, 255, 256, 257, 4096, 65535, 65536,
                        65537, rnd.randrange(1, 300000)])
        k = rnd.randrange(4)
        if k == 0:
            d = W.gen_json(n, rnd.randrange(100))
        elif k == 1:
            alpha = rnd.choice([1, 2, 4, 16])
            d = bytes(rnd.randrange(alpha) for _ in range(n))
        elif k == 2:
            d = rnd.randbytes(n)
        else:
            d = (rnd.randbytes(max(1, n // 37)) * 40)[:n]
        cases.append(d)
    return cases


def pa_compress(d):
    return pa.compress(d, codec="snappy", asbytes=True) if d else b"\x00"


def test_streams_decode_with_an_independent_snappy(oracle_mod):
    for i, d in enumerate(snappy_cases()):
        c = oracle_mod.snappy_compress(d)
        assert len(c) <= oracle_mod.snappy_max_compressed_length(len(d))
        assert oracle_mod.snappy_uncompressed_length(c) == len(d)
        if d:
            assert pa.decompress(c, decompressed_size=len(d), codec="snappy", asbytes=True) == d, i
        assert oracle_mod.snappy_uncompress(c) == (0, d), i


def test_decoder_reads_an_independent_snappy(oracle_mod):
    for i, d in enumerate(snappy_cases(seed=6)):
        assert oracle_mod.snappy_uncompress(pa_compress(d)) == (0, d), i


def test_element_forms(oracle_mod):
    """hand-made streams: every tag form of snappy.c:645-650 / char_table (:1129)"""
    lit = bytes(range(70))
    s = bytes([70]) + bytes([60 << 2, 69]) + lit           # 1 extra length byte
    assert oracle_mod.snappy_uncompress(s) == (0, lit)
    s = bytes([8]) + bytes([0 << 2]) + b"a" + bytes([1 | (3 << 2), 1])      # copy1: len 7, off 1
    assert oracle_mod.snappy_uncompress(s) == (0, b"a" * 8)
    s = bytes([12]) + bytes([3 << 2]) + b"abcd" + bytes([2 | (7 << 2), 4, 0])   # copy2: len 8
    assert oracle_mod.snappy_uncompress(s) == (0, b"abcd" * 3)
    s = bytes([12]) + bytes([3 << 2]) + b"abcd" + bytes([3 | (7 << 2), 4, 0, 0, 0])  # copy4
    assert oracle_mod.snappy_uncompress(s) == (0, b"abcd" * 3)
    bad = [bytes([8]) + bytes([0]) + b"a" + bytes([1 | (3 << 2), 0]),        # offset 0
           bytes([8]) + bytes([0]) + b"a" + bytes([1 | (3 << 2), 2]),        # offset > produced
           bytes([8]) + bytes([0]) + b"a" + bytes([1 | (3 << 2)]),           # header cut short
           bytes([9]) + bytes([0]) + b"a" + bytes([1 | (3 << 2), 1]),        # too few bytes
           bytes([7]) + bytes([0]) + b"a" + bytes([1 | (3 << 2), 1]),        # too many bytes
           bytes([2]) + bytes([1 << 2]) + b"a",                               # literal cut short
           bytes([0x80, 0x80, 0x80, 0x80, 0x10]),                             # varint too long
           b""]
    for s in bad:
        assert oracle_mod.snappy_uncompress(s)[0] != 0, s.hex()


def test_mutated_streams_agree_with_an_independent_snappy_when_both_accept(oracle_mod):
    rnd = random.Random(9)
    d = W.gen_json(5000, 4)
    c = bytearray(oracle_mod.snappy_compress(d))
    both = 0
    for _ in range(400):
        m = bytearray(c)
        for _ in range(rnd.randrange(1, 4)):
            m[rnd.randrange(len(m))] = rnd.randrange(256)
        n = oracle_mod.snappy_uncompressed_length(bytes(m))
        err, out = oracle_mod.snappy_uncompress(bytes(m))
        if err or n is None or n == 0:
            continue
        try:
            ref = pa.decompress(bytes(m), decompressed_size=n, codec="snappy", asbytes=True)
        except Exception:
            continue
        both += 1
        assert ref == out
    assert both > 20


def test_reader_case_bare_and_snappy_java(oracle_mod):
    """rdkafka_msgset_reader.c:299-390 / rd_kafka_snappy_java_uncompress (snappy.c:1588)"""
    a, b = W.gen_json(70000, 1), W.gen_json(123, 2)
    ca, cb = oracle_mod.snappy_compress(a), oracle_mod.snappy_compress(b)
    assert oracle_mod.rdk_snappy_decompress(ca) == (0, a)
    hdr = b"\x82SNAPPY\x00" + struct.pack(">II", 1, 1)
    framed = hdr + struct.pack(">I", len(ca)) + ca + struct.pack(">I", len(cb)) + cb
    assert oracle_mod.rdk_snappy_decompress(framed) == (0, a + b)
    assert oracle_mod.rdk_snappy_decompress(framed + b"\x00")[0] == -198      # trailing bytes
    assert oracle_mod.rdk_snappy_decompress(framed[:-1])[0] == -198           # chunk cut short
    assert oracle_mod.rdk_snappy_decompress(hdr + struct.pack(">I", 1) + b"\x00")[0] == -198  # empty
    assert oracle_mod.rdk_snappy_decompress(b"\xff\xff\xff\xff\xff")[0] == -198
