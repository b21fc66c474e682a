"""CPU oracle for the record-batch hot path -- TEST INFRASTRUCTURE ONLY.

Loads ``oracle/liboracle.so`` (the C restatement in crc32c_oracle.c /
lz4_oracle.c) and, when it has been built, ``oracle/_ref/libreflz4.so`` (the
reference's own vendored lz4 1.9.2 + xxHash compiled in place from
/root/reference/src, driven by ref_glue.c).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline.
The product package ``librdkafka_amd`` never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_REFLIB = os.path.join(_HERE, "_ref", "libreflz4.so")

ERR_NO_ERROR = 0
ERR_BAD_MSG = -199
ERR_BAD_COMPRESSION = -198
ERR_CRIT_SYS_RESOURCE = -194


def build(ref: bool = True) -> None:
    """Compile the oracle (and, if /root/reference exists, the reference lz4)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    if ref and os.path.isdir("/root/reference/src"):
        subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build(ref=False)
        L = C.CDLL(_LIB)
        u8p, u32p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
        L.or_crc32c.restype = C.c_uint32
        L.or_crc32c.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.or_crc32c_bitwise.restype = C.c_uint32
        L.or_crc32c_bitwise.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.or_crc32c_hw.restype = C.c_uint32
        L.or_crc32c_hw.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.or_crc32c_hw_available.restype = C.c_int
        L.or_crc32c_combine.restype = C.c_uint32
        L.or_crc32c_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_size_t]
        L.or_crc32c_batches_mt.restype = None
        L.or_crc32c_batches_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_size_t, C.c_int]
        L.or_xxh32.restype = C.c_uint32
        L.or_xxh32.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
        L.or_snappy_max_compressed_length.restype = C.c_size_t
        L.or_snappy_max_compressed_length.argtypes = [C.c_size_t]
        L.or_snappy_compress.restype = C.c_int
        L.or_snappy_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(C.c_size_t)]
        L.or_snappy_uncompressed_length.restype = C.c_int
        L.or_snappy_uncompressed_length.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.or_snappy_uncompress.restype = C.c_int
        L.or_snappy_uncompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.or_snappy_batches_mt.restype = C.c_int
        L.or_snappy_batches_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.or_rdk_snappy_decompress.restype = C.c_int
        L.or_rdk_snappy_decompress.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p),
                                               C.POINTER(C.c_size_t)]
        L.or_lz4hc_compress_block.restype = C.c_int
        L.or_lz4hc_compress_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.or_lz4_compress_block.restype = C.c_int
        L.or_lz4_compress_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.or_lz4_decompress_block.restype = C.c_int
        L.or_lz4_decompress_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.or_rdk_lz4_compress.restype = C.c_int
        L.or_rdk_lz4_compress.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.or_rdk_lz4_decompress.restype = C.c_int
        L.or_rdk_lz4_decompress.argtypes = [C.c_int, C.c_void_p, C.c_size_t,
                                            C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.or_lz4f_compress_bound.restype = C.c_size_t
        L.or_lz4f_compress_bound.argtypes = [C.c_size_t]
        L.or_free.argtypes = [C.c_void_p]
        L.or_lz4f_compress_batches_mt.restype = C.c_int
        L.or_lz4f_compress_batches_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.or_lz4f_compress_batches_level_mt.restype = C.c_int
        L.or_lz4f_compress_batches_level_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p,
                                                        C.c_size_t, C.c_void_p, C.c_void_p,
                                                        C.c_void_p, C.c_int, C.c_int]
        L.or_lz4f_decompress_batches_mt.restype = C.c_int
        L.or_lz4f_decompress_batches_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                    C.c_int]
        vp = C.c_void_p
        L.or_varint_enc_i64.restype = C.c_size_t
        L.or_varint_enc_i64.argtypes = [vp, C.c_int64]
        L.or_varint_dec_i64.restype = C.c_size_t
        L.or_varint_dec_i64.argtypes = [vp, C.c_size_t, C.POINTER(C.c_int64)]
        L.or_msgset_v2_write.restype = C.c_size_t
        L.or_msgset_v2_write.argtypes = [vp] * 9 + [C.c_uint32, C.c_uint32, C.c_int64, C.c_int16,
                                                    C.c_int32, C.c_int16, vp]
        L.or_msgset_v2_index.restype = C.c_long
        L.or_msgset_v2_index.argtypes = [vp, C.c_size_t, C.c_int64, C.c_int64] + [vp] * 8 + [C.c_long]
        L.or_crc32.restype = C.c_uint32
        L.or_crc32.argtypes = [C.c_uint32, vp, C.c_size_t]
        L.or_msgset_v01_write.restype = C.c_size_t
        L.or_msgset_v01_write.argtypes = [vp] * 6 + [C.c_uint32, C.c_uint32, C.c_int, C.c_int64,
                                                    C.c_int8, vp]
        L.or_msgset_v01_crc.restype = C.c_long
        L.or_msgset_v01_crc.argtypes = [vp, C.c_size_t, C.c_int, vp, vp, C.c_long]
        L.or_msgset_v01_crc_zlib.restype = C.c_long
        L.or_msgset_v01_crc_zlib.argtypes = [vp, C.c_size_t, C.c_int, vp, vp, C.c_long]
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(_REFLIB)


def ref():
    """The reference's own lz4/xxhash build (None if not built)."""
    global _ref
    if _ref is None and ref_available():
        R = C.CDLL(_REFLIB)
        R.ref_xxh32.restype = C.c_uint32
        R.ref_xxh32.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
        R.ref_lz4_decompress_safe.restype = C.c_int
        R.ref_lz4_decompress_safe.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        R.ref_lz4_compress_block.restype = C.c_int
        R.ref_lz4_compress_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        R.ref_lz4hc_compress_block.restype = C.c_int
        R.ref_lz4hc_compress_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        R.ref_rdk_lz4_compress.restype = C.c_int
        R.ref_rdk_lz4_compress.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_char_p),
                                           C.POINTER(C.c_size_t), C.c_int,
                                           C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        R.ref_rdk_lz4_decompress.restype = C.c_int
        R.ref_rdk_lz4_decompress.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_size_t,
                                             C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                             C.POINTER(C.c_int)]
        R.ref_free.argtypes = [C.c_void_p]
        R.ref_lz4f_compress_prefs.restype = C.c_int
        R.ref_lz4f_compress_prefs.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                              C.c_int, C.c_int, C.c_int, C.c_size_t,
                                              C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        R.ref_lz4f_compress_batches_mt.restype = C.c_int
        R.ref_lz4f_compress_batches_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                   C.c_int]
        R.ref_lz4f_decompress_batches_mt.restype = C.c_int
        R.ref_lz4f_decompress_batches_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p,
                                                     C.c_size_t, C.c_size_t, C.c_void_p,
                                                     C.c_void_p, C.c_void_p, C.c_int]
        _ref = R
    return _ref


def _buf(data: bytes):
    return C.create_string_buffer(bytes(data), max(1, len(data)))


# ---------------------------------------------------------------- oracle API
def crc32c(crc: int, data: bytes) -> int:
    b = _buf(data)
    return lib().or_crc32c(crc, b, len(data))


def crc32c_bitwise(crc: int, data: bytes) -> int:
    b = _buf(data)
    return lib().or_crc32c_bitwise(crc, b, len(data))


def crc32c_hw(crc: int, data: bytes) -> int:
    b = _buf(data)
    return lib().or_crc32c_hw(crc, b, len(data))


def crc32c_combine(a: int, b: int, len_b: int) -> int:
    return lib().or_crc32c_combine(a, b, len_b)


def xxh32(data: bytes, seed: int = 0) -> int:
    b = _buf(data)
    return lib().or_xxh32(b, len(data), seed)


def lz4_compress_block(data: bytes, acceleration: int = 1) -> bytes | None:
    """LZ4F block compression (cap = n-1); None means 'stored raw'."""
    n = len(data)
    src = _buf(data)
    dst = C.create_string_buffer(max(16, n + 16))
    r = lib().or_lz4_compress_block(src, n, dst, max(0, n - 1), acceleration)
    return None if r == 0 else dst.raw[:r]


def lz4hc_compress_block(data: bytes, level: int = 9) -> bytes | None:
    """LZ4HC block (hash chain 3..9, optimal parser 10..12; cap = n-1); None means 'stored raw'."""
    n = len(data)
    src = _buf(data)
    dst = C.create_string_buffer(max(16, n + 16))
    r = lib().or_lz4hc_compress_block(src, n, dst, max(0, n - 1), level)
    assert r >= 0, "level not restated"
    return None if r == 0 else dst.raw[:r]


def snappy_max_compressed_length(n: int) -> int:
    return lib().or_snappy_max_compressed_length(n)


def snappy_compress(data: bytes) -> bytes:
    """rd_kafka_snappy_compress_iov restated: varint length + 64 KiB fragments."""
    n = len(data)
    src = _buf(data)
    dst = C.create_string_buffer(snappy_max_compressed_length(n))
    out = C.c_size_t(0)
    assert lib().or_snappy_compress(src, n, dst, C.byref(out)) == 0
    return dst.raw[:out.value]


def snappy_uncompressed_length(data: bytes) -> int | None:
    b = _buf(data)
    r = C.c_size_t(0)
    return r.value if lib().or_snappy_uncompressed_length(b, len(data), C.byref(r)) else None


def snappy_uncompress(data: bytes) -> tuple[int, bytes]:
    """rd_kafka_snappy_uncompress restated: (0, payload) or (-EIO, b"")."""
    n = snappy_uncompressed_length(data)
    if n is None:
        return -5, b""
    b = _buf(data)
    out = C.create_string_buffer(max(1, n))
    r = lib().or_snappy_uncompress(b, len(data), out)
    return (0, out.raw[:n]) if r == 0 else (r, b"")


def rdk_snappy_decompress(data: bytes) -> tuple[int, bytes]:
    """The reader's snappy case (snappy-java framing or bare): (err, payload)."""
    b = _buf(data)
    out = C.c_void_p()
    n = C.c_size_t(0)
    err = lib().or_rdk_snappy_decompress(b, len(data), C.byref(out), C.byref(n))
    if err:
        return err, b""
    payload = C.string_at(out, n.value)
    lib().or_free(out)
    return 0, payload


def lz4_decompress_block(block: bytes, capacity: int, history: bytes = b"") -> tuple[int, bytes]:
    buf = C.create_string_buffer(len(history) + capacity + 64)
    C.memmove(buf, history, len(history))
    src = _buf(block)
    dst = C.cast(C.addressof(buf) + len(history), C.c_void_p)
    r = lib().or_lz4_decompress_block(src, len(block), dst, capacity, len(history))
    if r < 0:
        return r, b""
    return r, buf.raw[len(history):len(history) + r]


def rdk_lz4_compress(data: bytes, proper_hc: int = 1, comp_level: int = 0) -> tuple[int, bytes]:
    src = _buf(data)
    out = C.c_void_p()
    n = C.c_size_t()
    err = lib().or_rdk_lz4_compress(proper_hc, comp_level, src, len(data), C.byref(out), C.byref(n))
    if err:
        return err, b""
    res = C.string_at(out, n.value)
    lib().or_free(out)
    return 0, res


def rdk_lz4_decompress(frame: bytes, proper_hc: int = 1) -> tuple[int, bytes]:
    src = _buf(frame)
    out = C.c_void_p()
    n = C.c_size_t()
    err = lib().or_rdk_lz4_decompress(proper_hc, src, len(frame), C.byref(out), C.byref(n))
    if err:
        return err, b""
    res = C.string_at(out, n.value) if n.value else b""
    lib().or_free(out)
    return 0, res


# ------------------------------------------------------- reference (compiled)
def ref_rdk_lz4_compress(segments, proper_hc: int = 1, comp_level: int = 0) -> tuple[int, bytes]:
    if isinstance(segments, (bytes, bytearray)):
        segments = [bytes(segments)]
    R = ref()
    n = len(segments)
    ptrs = (C.c_char_p * max(1, n))(*[bytes(s) for s in segments])
    lens = (C.c_size_t * max(1, n))(*[len(s) for s in segments])
    out = C.c_void_p()
    olen = C.c_size_t()
    err = R.ref_rdk_lz4_compress(proper_hc, comp_level, ptrs, lens, n, C.byref(out), C.byref(olen))
    if err:
        return err, b""
    res = C.string_at(out, olen.value)
    R.ref_free(out)
    return 0, res


def ref_rdk_lz4_decompress(frame: bytes, proper_hc: int = 1,
                           max_msg_size: int = 1000000) -> tuple[int, bytes, int]:
    R = ref()
    src = _buf(frame)
    out = C.c_void_p()
    olen = C.c_size_t()
    grow = C.c_int()
    err = R.ref_rdk_lz4_decompress(proper_hc, src, len(frame), max_msg_size, C.byref(out),
                                   C.byref(olen), C.byref(grow))
    if err:
        return err, b"", grow.value
    res = C.string_at(out, olen.value) if olen.value else b""
    R.ref_free(out)
    return 0, res, grow.value


def ref_lz4_decompress_safe(block: bytes, capacity: int) -> tuple[int, bytes]:
    R = ref()
    src = _buf(block)
    dst = C.create_string_buffer(capacity + 64)
    r = R.ref_lz4_decompress_safe(src, dst, len(block), capacity)
    return (r, dst.raw[:r]) if r >= 0 else (r, b"")


def ref_lz4_compress_block(data: bytes, acceleration: int = 1) -> bytes | None:
    R = ref()
    n = len(data)
    src = _buf(data)
    dst = C.create_string_buffer(max(16, n + 16))
    r = R.ref_lz4_compress_block(src, n, dst, max(0, n - 1), acceleration)
    return None if r == 0 else dst.raw[:r]


def ref_lz4hc_compress_block(data: bytes, level: int = 9) -> bytes | None:
    R = ref()
    n = len(data)
    src = _buf(data)
    dst = C.create_string_buffer(max(16, n + 16))
    r = R.ref_lz4hc_compress_block(src, n, dst, max(0, n - 1), level)
    return None if r == 0 else dst.raw[:r]


def ref_xxh32(data: bytes, seed: int = 0) -> int:
    b = _buf(data)
    return ref().ref_xxh32(b, len(data), seed)


def ref_lz4f_compress_prefs(data: bytes, linked=0, block_size_id=4, block_checksum=0,
                            content_checksum=0, content_size=0, level=0, flush_every=0) -> bytes:
    """A frame from the reference LZ4F encoder with non-default preferences."""
    R = ref()
    src = _buf(data)
    out = C.c_void_p()
    n = C.c_size_t()
    err = R.ref_lz4f_compress_prefs(src, len(data), linked, block_size_id, block_checksum,
                                    content_checksum, content_size, level, flush_every,
                                    C.byref(out), C.byref(n))
    assert err == 0, err
    res = C.string_at(out, n.value)
    R.ref_free(out)
    return res


# ---- MsgVersion 2 records (msgset_oracle.c) ---------------------------------
def varint_enc(num: int) -> bytes:
    """rdvarint.h:67 rd_uvarint_enc_i64 (zig-zag + LEB128)."""
    b = C.create_string_buffer(16)
    n = lib().or_varint_enc_i64(b, num)
    return b.raw[:n]


def varint_dec(data: bytes) -> tuple[int, int]:
    """rdvarint.h:132 rd_varint_dec_i64 -> (value, bytes read); bytes read 0 = failure."""
    v = C.c_int64()
    n = lib().or_varint_dec_i64(_buf(data), len(data), C.byref(v))
    return v.value, n


def _np_ptr(a):
    return None if a is None else a.ctypes.data


def msgset_v2_write(msgs: dict, first: int, cnt: int, producer_id: int = -1,
                    producer_epoch: int = -1, base_sequence: int = -1, attributes: int = 0) -> bytes:
    """One uncompressed MsgVersion 2 batch of messages [first, first+cnt), as
    rdkafka_msgset_writer.c writes it.  `msgs`: numpy arrays arena (u8), ts (i64),
    key_off (u64), key_len (i32, -1 null), val_off, val_len, and optionally
    hdr_off (u64), hdr_len (u32), hdr_cnt (i32)."""
    import numpy as np
    kl, vl = msgs["key_len"], msgs["val_len"]
    hl = msgs.get("hdr_len")
    cap = 61 + int(cnt) * 40 + int(np.maximum(kl[first:first + cnt], 0).sum()) + \
        int(np.maximum(vl[first:first + cnt], 0).sum()) + \
        (int(hl[first:first + cnt].sum()) if hl is not None else 0)
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().or_msgset_v2_write(
        _np_ptr(msgs["arena"]), _np_ptr(msgs["ts"]), _np_ptr(msgs["key_off"]), _np_ptr(kl),
        _np_ptr(msgs["val_off"]), _np_ptr(vl), _np_ptr(msgs.get("hdr_off")), _np_ptr(hl),
        _np_ptr(msgs.get("hdr_cnt")), first, cnt, producer_id, producer_epoch, base_sequence,
        attributes, _np_ptr(out))
    return bytes(out[:n])


def msgset_v2_index(records: bytes, base_offset: int = 0, base_ts: int = 0, max_rows=None):
    """rdkafka_msgset_reader.c:715-927 over a batch's records -> (n, rows dict);
    n < 0: record -n-1 failed to parse."""
    import numpy as np
    m = max_rows if max_rows is not None else max(1, len(records) // 7 + 1)
    rows = {k: np.zeros(m, dtype=t) for k, t in (("offset", np.int64), ("timestamp", np.int64),
                                                  ("key_off", np.uint32), ("key_len", np.int32),
                                                  ("val_off", np.uint32), ("val_len", np.int32),
                                                  ("hdr_off", np.uint32), ("hdr_len", np.uint32))}
    rec = np.frombuffer(records, dtype=np.uint8) if records else np.zeros(1, dtype=np.uint8)
    n = lib().or_msgset_v2_index(
        _np_ptr(rec), len(records), base_offset, base_ts, *(_np_ptr(rows[k]) for k in
        ("offset", "timestamp", "key_off", "key_len", "val_off", "val_len", "hdr_off", "hdr_len")), m)
    return n, {k: v[:max(n, 0)] for k, v in rows.items()}


# ------------------------------------------------------------ MsgVersion 0/1
def crc32(crc: int, data: bytes) -> int:
    """zlib crc32() as the reference uses it (rdcrc32.h:93-131, WITH_ZLIB)."""
    return lib().or_crc32(crc & 0xFFFFFFFF, _buf(data), len(data))


def msgset_v01_write(msgs: dict, first: int, cnt: int, magic: int = 1, base_offset: int = 0,
                     attributes: int = 0) -> bytes:
    """Uncompressed MsgVersion 0/1 MessageSet of messages [first, first+cnt)
    (rdkafka_msgset_writer.c:583-645), CRCs filled in."""
    import numpy as np
    kl, vl = msgs["key_len"], msgs["val_len"]
    cap = int(cnt) * 34 + int(np.maximum(kl[first:first + cnt], 0).sum()) + \
        int(np.maximum(vl[first:first + cnt], 0).sum())
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    n = lib().or_msgset_v01_write(
        _np_ptr(msgs["arena"]), _np_ptr(msgs["ts"]), _np_ptr(msgs["key_off"]), _np_ptr(kl),
        _np_ptr(msgs["val_off"]), _np_ptr(vl), first, cnt, magic, base_offset, attributes,
        _np_ptr(out))
    return bytes(out[:n])


def msgset_v01_crc(mset: bytes, mode: int = 0, max_rows=None):
    """Reader walk + check.crcs (rdkafka_msgset_reader.c:538-628) over one MessageSet ->
    (n, pos, out, set_after); n < 0: message -n-1 failed the header checks."""
    import numpy as np
    m = max_rows if max_rows is not None else max(1, len(mset) // 18 + 1)
    buf = np.frombuffer(bytes(mset) + b"\0", dtype=np.uint8).copy()
    pos = np.zeros(max(m, 1), dtype=np.uint32)
    out = np.zeros(max(m, 1), dtype=np.uint32)
    n = lib().or_msgset_v01_crc(_np_ptr(buf), len(mset), mode, _np_ptr(pos), _np_ptr(out), m)
    k = max(n, 0) if n >= 0 else -n - 1
    return n, pos[:k], out[:k], bytes(buf[:len(mset)])
