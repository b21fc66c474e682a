"""librdkafka_amd -- MI355X (gfx950) engine for librdkafka's record-batch hot path.

Host-side mirror of the reference interface for this path (CRC32C over
MsgVersion 2 record batches, LZ4F frame compression / decompression), bound
to the C-ABI library ``librdkafka_hip.so`` built in-tree from ``csrc/``.

Two layers, as in ``include/librdkafka_hip.h``:

* drop-in functions with the reference's names, argument meaning and error
  codes: :func:`crc32c`, :func:`rd_slice_crc32c`, :func:`rd_kafka_lz4_compress`,
  :func:`rd_kafka_lz4_decompress` (host buffers in, host bytes out);
* the device-resident batch engine (``*_batch`` functions on torch device
  tensors) used by bench.py and the multi-partition producer/consumer paths.

There is no CPU fallback: if the library or a gfx950 device is missing every
call raises :class:`EngineError`.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import numpy as np

try:  # share torch's HIP runtime (same SONAME) when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always installed here
    torch = None

from . import workload  # noqa: E402,F401

_HERE = os.path.dirname(os.path.abspath(__file__))
# RDK_HIP_LIB: an alternative build of the same library (kernel A/B experiments)
LIB_PATH = os.environ.get("RDK_HIP_LIB") or os.path.join(_HERE, "librdkafka_hip.so")

RESP_ERR_NO_ERROR = 0
RESP_ERR__BAD_MSG = -199
RESP_ERR__BAD_COMPRESSION = -198
RESP_ERR__CRIT_SYS_RESOURCE = -194
LZ4F_E_DSTSIZE = -1000

V2_CRC_COMPUTE, V2_CRC_FINALIZE, V2_CRC_VERIFY = 0, 1, 2

# every symbol include/librdkafka_hip.h declares (checked by tests)
EXPORTED_SYMBOLS = (
    "crc32c", "crc32c_global_init", "rd_slice_crc32c", "rd_kafka_lz4_compress",
    "rd_kafka_lz4_decompress", "rdk_hip_init", "rdk_hip_last_error", "rdk_hip_version",
    "rdk_hip_crc32c_ranges", "rdk_hip_msgset_v2_crc", "rdk_hip_lz4f_compress_bound",
    "rdk_hip_lz4f_compress", "rdk_hip_lz4f_compress_fast", "rdk_hip_lz4f_decompress",
    "rdk_hip_gen_v2_batches", "rdk_hip_producer_new", "rdk_hip_producer_produce",
    "rdk_hip_producer_flush", "rdk_hip_producer_poll", "rdk_hip_producer_destroy",
    "rdk_hip_gen_json", "rdk_hip_msgset_v2_sizes", "rdk_hip_msgset_v2_write",
    "rdk_hip_msgset_v2_index", "rd_slice_crc32", "rdk_hip_crc32_ranges",
    "rdk_hip_msgset_v01_crc", "rdk_hip_lz4f_decompress_noalloc", "rdk_hip_msgset_v2_finalize",
    "rdk_hip_dropin_calls", "rdk_hip_snappy_max_compressed_length", "rdk_hip_snappy_compress",
    "rdk_hip_snappy_uncompress", "rd_kafka_snappy_init_env", "rd_kafka_snappy_init_env_sg",
    "rd_kafka_snappy_free_env", "rd_kafka_snappy_max_compressed_length",
    "rd_kafka_snappy_uncompressed_length", "rd_kafka_snappy_compress_iov",
    "rd_kafka_snappy_compress", "rd_kafka_snappy_uncompress", "rd_kafka_snappy_java_uncompress",
    "rdk_hip_snappy_dropin_calls", "rdk_hip_dropin_host_crcs", "rdk_hip_ctx_counts",
    "rdk_hip_dropin_combined",
    "rdk_hip_lz4f_compress_units",
)


class EngineError(RuntimeError):
    pass


def build(jobs: int = 8) -> str:
    """Compile librdkafka_hip.so for gfx950 in-tree (hipcc)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", _HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    """Load librdkafka_hip.so (raises EngineError when it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} not built (run librdkafka_amd.build())")
    L = C.CDLL(LIB_PATH)
    vp, sz, u32, i32, i64 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_int, C.c_int64
    L.crc32c.restype = u32
    L.crc32c.argtypes = [u32, vp, sz]
    L.crc32c_global_init.restype = None
    L.rd_slice_crc32c.restype = u32
    L.rd_slice_crc32c.argtypes = [vp]
    L.rd_slice_crc32.restype = u32
    L.rd_slice_crc32.argtypes = [vp]
    L.rd_kafka_lz4_compress.restype = i32
    L.rd_kafka_lz4_compress.argtypes = [vp, i32, i32, vp, C.POINTER(vp), C.POINTER(sz)]
    L.rd_kafka_lz4_decompress.restype = i32
    L.rd_kafka_lz4_decompress.argtypes = [vp, i32, i64, vp, sz, C.POINTER(vp), C.POINTER(sz)]
    L.rdk_hip_init.restype = i32
    L.rdk_hip_init.argtypes = [i32]
    L.rdk_hip_last_error.restype = C.c_char_p
    L.rdk_hip_version.restype = C.c_char_p
    L.rdk_hip_crc32c_ranges.restype = i32
    L.rdk_hip_crc32c_ranges.argtypes = [vp, vp, vp, vp, vp, u32, vp]
    L.rdk_hip_crc32_ranges.restype = i32
    L.rdk_hip_crc32_ranges.argtypes = [vp, vp, vp, vp, vp, u32, vp]
    L.rdk_hip_msgset_v01_crc.restype = i32
    L.rdk_hip_msgset_v01_crc.argtypes = [vp] * 8 + [u32, i32, vp]
    L.rdk_hip_msgset_v2_crc.restype = i32
    L.rdk_hip_msgset_v2_crc.argtypes = [vp, vp, vp, vp, u32, i32, vp]
    if hasattr(L, "rdk_hip_lz4f_compress"):
        L.rdk_hip_lz4f_compress_bound.restype = sz
        L.rdk_hip_lz4f_compress_bound.argtypes = [sz]
        L.rdk_hip_lz4f_compress.restype = i32
        L.rdk_hip_lz4f_compress.argtypes = [vp, vp, vp, vp, vp, vp, u32, i32, vp]
        L.rdk_hip_lz4f_compress_fast.restype = i32
        L.rdk_hip_lz4f_compress_fast.argtypes = [vp, vp, vp, vp, vp, vp, u32, vp]
        L.rdk_hip_lz4f_compress_units.restype = i32
        L.rdk_hip_lz4f_compress_units.argtypes = [vp, vp, vp, vp, vp, vp, u32, vp]
        L.rdk_hip_lz4f_decompress.restype = i32
        L.rdk_hip_lz4f_decompress.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]
        L.rdk_hip_lz4f_decompress_noalloc.restype = i32
        L.rdk_hip_lz4f_decompress_noalloc.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]
    L.rdk_hip_msgset_v2_finalize.restype = i32
    L.rdk_hip_msgset_v2_finalize.argtypes = [vp] * 9 + [u32, i32, vp]
    L.rdk_hip_producer_new.restype = vp
    L.rdk_hip_producer_new.argtypes = [i32, sz, i32, i32]
    L.rdk_hip_producer_produce.restype = i32
    L.rdk_hip_producer_produce.argtypes = [vp, vp, vp, u32, C.c_uint64]
    L.rdk_hip_producer_flush.restype = i32
    L.rdk_hip_producer_flush.argtypes = [vp]
    L.rdk_hip_producer_poll.restype = i32
    L.rdk_hip_producer_poll.argtypes = [vp, vp, i32, i32]
    L.rdk_hip_producer_destroy.restype = None
    L.rdk_hip_producer_destroy.argtypes = [vp]
    L.rdk_hip_gen_v2_batches.restype = i32
    L.rdk_hip_gen_v2_batches.argtypes = [vp, u32, u32, C.c_uint64, vp]
    L.rdk_hip_gen_json.restype = None
    L.rdk_hip_gen_json.argtypes = [vp, sz, u32]
    L.rdk_hip_msgset_v2_sizes.restype = i32
    L.rdk_hip_msgset_v2_sizes.argtypes = [C.POINTER(_Msgs), vp, u32, vp, vp, vp, vp]
    L.rdk_hip_msgset_v2_write.restype = i32
    L.rdk_hip_msgset_v2_write.argtypes = [C.POINTER(_Msgs), vp, u32, vp, vp, vp, vp, vp, vp, vp]
    L.rdk_hip_msgset_v2_index.restype = i32
    L.rdk_hip_msgset_v2_index.argtypes = [vp] * 7 + [C.POINTER(_Rows), vp, u32, vp]
    L.rdk_hip_dropin_host_crcs.restype = C.c_uint64
    L.rdk_hip_dropin_host_crcs.argtypes = []
    L.rdk_hip_ctx_counts.restype = None
    L.rdk_hip_ctx_counts.argtypes = [vp]
    L.rdk_hip_dropin_combined.restype = None
    L.rdk_hip_dropin_combined.argtypes = [vp]
    _lib = L
    return L


class _Msgs(C.Structure):
    """rdk_hip_msgs_t (include/librdkafka_hip.h): device pointers, one entry per message."""
    _fields_ = [(n, C.c_void_p) for n in ("arena", "timestamp", "key_off", "key_len", "value_off",
                                          "value_len", "headers_off", "headers_len",
                                          "header_count")]


class _Rows(C.Structure):
    """rdk_hip_v2_rows_t: device arrays of the record index."""
    _fields_ = [(n, C.c_void_p) for n in ("offset", "timestamp", "key_off", "key_len",
                                          "value_off", "value_len", "headers_off",
                                          "headers_len")]


V2_ROW_FIELDS = (("offset", "int64"), ("timestamp", "int64"), ("key_off", "int32"),
                 ("key_len", "int32"), ("val_off", "int32"), ("val_len", "int32"),
                 ("hdr_off", "int32"), ("hdr_len", "int32"))


# rdk_hip_v2_batch_t
V2_BATCH_DTYPE = np.dtype([("first_msg", "<u4"), ("msg_count", "<u4"), ("producer_id", "<i8"),
                           ("base_sequence", "<i4"), ("producer_epoch", "<i2"),
                           ("attributes", "<i2")])


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().rdk_hip_last_error().decode(errors="replace")
        raise EngineError(f"{what} failed ({rc}): {msg}")


def init(device: int = -1) -> None:
    """Bind the calling thread's engine context to `device` (default 0)."""
    _check(lib().rdk_hip_init(device), "rdk_hip_init")


def version() -> str:
    return lib().rdk_hip_version().decode()


# ------------------------------------------------------------------ drop-in
class _Segment(C.Structure):
    pass


_Segment._fields_ = [
    ("tqe_next", C.POINTER(_Segment)), ("tqe_prev", C.c_void_p),
    ("seg_p", C.c_void_p), ("seg_of", C.c_size_t), ("seg_size", C.c_size_t),
    ("seg_absof", C.c_size_t), ("seg_free", C.c_void_p), ("seg_flags", C.c_int),
]


class _Slice(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("seg", C.POINTER(_Segment)), ("rof", C.c_size_t),
                ("start", C.c_size_t), ("end", C.c_size_t)]


class RdSlice:
    """An rd_slice_t over a list of byte segments (rdbuf.h:63-115 layout),
    the boundary type the writer hands to rd_slice_crc32c / lz4_compress.
    `start`/`end` are absolute offsets into the concatenated segments."""

    def __init__(self, segments, start: int = 0, end: int | None = None):
        self._bufs = [C.create_string_buffer(bytes(s), max(1, len(s))) for s in segments]
        n = len(segments)
        self._segs = (_Segment * max(1, n))()
        absof = 0
        for i, s in enumerate(segments):
            g = self._segs[i]
            g.seg_p = C.addressof(self._bufs[i])
            g.seg_of = len(s)
            g.seg_size = len(s)
            g.seg_absof = absof
            absof += len(s)
            if i + 1 < n:
                g.tqe_next = C.pointer(self._segs[i + 1])
        total = absof
        end = total if end is None else end
        self.slice = _Slice()
        self.slice.start, self.slice.end = start, end
        # rd_slice_init: position the reader at `start`
        seg_i, rof = 0, start
        while seg_i < n - 1 and rof >= len(segments[seg_i]) and len(segments[seg_i]) > 0:
            rof -= len(segments[seg_i])
            seg_i += 1
        if n:
            self.slice.seg = C.pointer(self._segs[seg_i])
        self.slice.rof = rof

    def remains(self) -> int:
        s = self.slice
        if not s.seg:
            return s.end
        return s.end - (s.seg.contents.seg_absof + s.rof)

    @property
    def ptr(self):
        return C.byref(self.slice)


def crc32c(crc: int, data: bytes) -> int:
    """crc32c() (src/crc32c.c:360) on the GPU."""
    b = C.create_string_buffer(bytes(data), max(1, len(data)))
    return lib().crc32c(crc & 0xFFFFFFFF, b, len(data))


def rd_slice_crc32c(slice_or_segments) -> int:
    """rd_slice_crc32c() (src/rdbuf.c:1113) on the GPU; consumes the slice."""
    s = slice_or_segments if isinstance(slice_or_segments, RdSlice) else RdSlice(slice_or_segments)
    return lib().rd_slice_crc32c(s.ptr)


def rd_slice_crc32(slice_or_segments) -> int:
    """rd_slice_crc32() (src/rdbuf.c:1093, zlib CRC-32) on the GPU; consumes the slice."""
    s = slice_or_segments if isinstance(slice_or_segments, RdSlice) else RdSlice(slice_or_segments)
    return lib().rd_slice_crc32(s.ptr)


def rd_kafka_lz4_compress(proper_hc: int, comp_level: int, slice_or_segments) -> tuple[int, bytes]:
    """rd_kafka_lz4_compress() (src/rdkafka_lz4.c:329): (err, frame)."""
    s = slice_or_segments if isinstance(slice_or_segments, RdSlice) else RdSlice(
        [slice_or_segments] if isinstance(slice_or_segments, (bytes, bytearray)) else slice_or_segments)
    out = C.c_void_p()
    n = C.c_size_t()
    err = lib().rd_kafka_lz4_compress(None, proper_hc, comp_level, s.ptr, C.byref(out), C.byref(n))
    if err:
        return err, b""
    res = C.string_at(out, n.value)
    _libc().free(out)
    return 0, res


def rd_kafka_lz4_decompress(proper_hc: int, offset: int, frame) -> tuple[int, bytes]:
    """rd_kafka_lz4_decompress() (src/rdkafka_lz4.c:167): (err, payload).
    `frame` may be a bytearray, which is patched in place when !proper_hc."""
    buf = C.create_string_buffer(bytes(frame), max(1, len(frame)))
    out = C.c_void_p()
    n = C.c_size_t()
    err = lib().rd_kafka_lz4_decompress(None, proper_hc, offset, buf, len(frame),
                                        C.byref(out), C.byref(n))
    if isinstance(frame, bytearray):
        frame[:] = buf.raw[:len(frame)]
    if err:
        return err, b""
    res = C.string_at(out, n.value) if n.value else b""
    _libc().free(out)
    return 0, res


def dropin_host_crcs() -> int:
    """CRC drop-in calls that finished on the host after the device path failed twice."""
    return int(lib().rdk_hip_dropin_host_crcs())


def dropin_combined() -> tuple[int, int, int, int]:
    """(batches of >= 2 drop-in requests, requests served in them, largest batch, batches that
    fell back to single requests after a device error)."""
    a = (C.c_uint64 * 4)()
    lib().rdk_hip_dropin_combined(a)
    return tuple(int(x) for x in a)


def ctx_counts() -> tuple[int, int]:
    """(created, destroyed) per-thread engine contexts."""
    a = (C.c_uint64 * 2)()
    lib().rdk_hip_ctx_counts(a)
    return int(a[0]), int(a[1])


_libc_h = None


def _libc():
    global _libc_h
    if _libc_h is None:
        _libc_h = C.CDLL(None)
        _libc_h.free.argtypes = [C.c_void_p]
    return _libc_h


# ------------------------------------------------------- device batch engine
def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(stream):
    """Default to torch's current stream so engine launches are ordered with
    the torch ops that produce / consume the same device tensors."""
    if stream is None:
        if torch is None:
            return None
        stream = torch.cuda.current_stream()
    h = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
    return C.c_void_p(h) if h else None  # 0 -> the null stream


def crc32c_ranges(base, offs, lens, out, init=None, stream=None) -> None:
    """CRC32C of device ranges base[offs[i]:offs[i]+lens[i]] -> out[i] (uint32)."""
    _check(lib().rdk_hip_crc32c_ranges(_ptr(base), _ptr(offs), _ptr(lens), _ptr(init), _ptr(out),
                                       int(offs.numel()), _stream(stream)), "crc32c_ranges")


def crc32_ranges(base, offs, lens, out, init=None, stream=None) -> None:
    """CRC-32 (zlib crc32(), MsgVersion 0/1) of device ranges -> out[i] (uint32)."""
    _check(lib().rdk_hip_crc32_ranges(_ptr(base), _ptr(offs), _ptr(lens), _ptr(init), _ptr(out),
                                      int(offs.numel()), _stream(stream)), "crc32_ranges")


def msgset_v01_crc(base, set_offs, set_lens, row_offs, row_caps, msg_pos, msg_out, count,
                   mode=V2_CRC_COMPUTE, stream=None) -> None:
    """MsgVersion 0/1 MessageSets on device: per-message CRC-32 compute / finalize / verify
    (rdkafka_msgset_reader.c:538-628, rdkafka_msgset_writer.c:583-645); see
    include/librdkafka_hip.h for the row / count layout."""
    _check(lib().rdk_hip_msgset_v01_crc(_ptr(base), _ptr(set_offs), _ptr(set_lens),
                                        _ptr(row_offs), _ptr(row_caps), _ptr(msg_pos),
                                        _ptr(msg_out), _ptr(count), int(set_offs.numel()), mode,
                                        _stream(stream)), "msgset_v01_crc")


def msgset_v2_crc(base, batch_offs, batch_caps, out, mode=V2_CRC_COMPUTE, stream=None) -> None:
    """CRC32C compute / finalize / verify of MsgVersion 2 batches on device."""
    _check(lib().rdk_hip_msgset_v2_crc(_ptr(base), _ptr(batch_offs), _ptr(batch_caps), _ptr(out),
                                       int(batch_offs.numel()), mode, _stream(stream)),
           "msgset_v2_crc")


def lz4f_compress_bound(n: int) -> int:
    return int(lib().rdk_hip_lz4f_compress_bound(n))


def lz4f_compress_batch(src, in_offs, in_lens, dst, out_offs, out_lens, level=0, stream=None):
    _check(lib().rdk_hip_lz4f_compress(_ptr(src), _ptr(in_offs), _ptr(in_lens), _ptr(dst),
                                       _ptr(out_offs), _ptr(out_lens), int(in_offs.numel()),
                                       level, _stream(stream)), "lz4f_compress")


def lz4f_compress_fast_batch(src, in_offs, in_lens, dst, out_offs, out_lens, stream=None):
    """Throughput-mode LZ4F compression (csrc/lz4_encode_fast.hip): same frame
    format and prefs as rd_kafka_lz4_compress, reference-decodable, ratio
    within 5 % of the reference's; not byte-identical to its frames."""
    _check(lib().rdk_hip_lz4f_compress_fast(_ptr(src), _ptr(in_offs), _ptr(in_lens), _ptr(dst),
                                            _ptr(out_offs), _ptr(out_lens), int(in_offs.numel()),
                                            _stream(stream)), "lz4f_compress_fast")


def lz4f_compress_units_batch(src, in_offs, in_lens, dst, out_offs, out_lens, stream=None):
    """rdk_hip_lz4f_compress_units: the throughput compressor's workgroup-per-block engine
    (csrc/lz4_encode_units.hip), same contract as lz4f_compress_fast_batch."""
    _check(lib().rdk_hip_lz4f_compress_units(_ptr(src), _ptr(in_offs), _ptr(in_lens), _ptr(dst),
                                             _ptr(out_offs), _ptr(out_lens), int(in_offs.numel()),
                                             _stream(stream)), "lz4f_compress_units")


def lz4f_decompress_batch(src, in_offs, in_lens, dst, out_offs, out_caps, out_lens, status,
                          stream=None):
    _check(lib().rdk_hip_lz4f_decompress(_ptr(src), _ptr(in_offs), _ptr(in_lens), _ptr(dst),
                                         _ptr(out_offs), _ptr(out_caps), _ptr(out_lens),
                                         _ptr(status), int(in_offs.numel()), _stream(stream)),
           "lz4f_decompress")


LZ4F_NOALLOC_MAX_FRAMES = 1024


# ------------------------------------------------------------------ snappy
SNAPPY_E_IO, SNAPPY_E_DSTSIZE = -5, -1001


def snappy_max_compressed_length(n: int) -> int:
    f = lib().rdk_hip_snappy_max_compressed_length
    f.restype, f.argtypes = C.c_size_t, [C.c_size_t]
    return f(n)


def snappy_compress_batch(src, in_offs, in_lens, dst, out_offs, out_lens, stream=None) -> None:
    """rdk_hip_snappy_compress: n device-resident inputs -> n snappy streams."""
    _check(lib().rdk_hip_snappy_compress(_ptr(src), _ptr(in_offs), _ptr(in_lens), _ptr(dst),
                                         _ptr(out_offs), _ptr(out_lens), int(in_offs.numel()),
                                         _stream(stream)), "snappy_compress")


def snappy_uncompress_batch(src, in_offs, in_lens, dst, out_offs, out_caps, out_lens, status,
                            stream=None) -> None:
    """rdk_hip_snappy_uncompress: n device-resident streams -> payloads + per-stream verdict."""
    _check(lib().rdk_hip_snappy_uncompress(_ptr(src), _ptr(in_offs), _ptr(in_lens), _ptr(dst),
                                           _ptr(out_offs), _ptr(out_caps), _ptr(out_lens),
                                           _ptr(status), int(in_offs.numel()), _stream(stream)),
           "snappy_uncompress")


class _Iovec(C.Structure):
    _fields_ = [("iov_base", C.c_void_p), ("iov_len", C.c_size_t)]


def rd_kafka_snappy_compress_iov(segments) -> tuple[int, bytes]:
    """Drop-in rd_kafka_snappy_compress_iov over host segments, driven as
    rd_kafka_msgset_writer_compress_snappy does (rdkafka_msgset_writer.c:1041-1083):
    (0, stream) or (negative errno, b"")."""
    L = lib()
    segs = [bytes(s) for s in ([segments] if isinstance(segments, (bytes, bytearray)) else segments)]
    total = sum(len(s) for s in segs)
    bufs = [C.create_string_buffer(s, max(1, len(s))) for s in segs]
    iov = (_Iovec * max(1, len(segs)))()
    for i, (b, s) in enumerate(zip(bufs, segs)):
        iov[i].iov_base, iov[i].iov_len = C.addressof(b), len(s)
    env = (C.c_void_p * 3)()
    L.rd_kafka_snappy_init_env_sg.argtypes = [C.c_void_p, C.c_bool]
    L.rd_kafka_snappy_init_env_sg(env, True)
    L.rd_kafka_snappy_max_compressed_length.restype = C.c_size_t
    L.rd_kafka_snappy_max_compressed_length.argtypes = [C.c_size_t]
    cap = L.rd_kafka_snappy_max_compressed_length(total)
    out = C.create_string_buffer(cap)
    ciov = _Iovec(C.addressof(out), cap)
    L.rd_kafka_snappy_compress_iov.restype = C.c_int
    L.rd_kafka_snappy_compress_iov.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                               C.c_void_p]
    r = L.rd_kafka_snappy_compress_iov(env, iov, len(segs), total, C.byref(ciov))
    L.rd_kafka_snappy_free_env.argtypes = [C.c_void_p]
    L.rd_kafka_snappy_free_env(env)
    return (0, out.raw[:ciov.iov_len]) if r == 0 else (r, b"")


def rd_kafka_snappy_decompress(data: bytes) -> tuple[int, bytes]:
    """The reader's snappy case (rdkafka_msgset_reader.c:299-390) over the drop-in symbols:
    snappy-java framing or a bare stream.  (0, payload) or (RESP_ERR__BAD_COMPRESSION, b"")."""
    L = lib()
    data = bytes(data)
    buf = C.create_string_buffer(data, max(1, len(data)))
    if len(data) > 16 + 4 and data[:8] == b"\x82SNAPPY\x00":
        L.rd_kafka_snappy_java_uncompress.restype = C.c_void_p
        L.rd_kafka_snappy_java_uncompress.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                                      C.c_char_p, C.c_size_t]
        n = C.c_size_t(0)
        err = C.create_string_buffer(128)
        p = L.rd_kafka_snappy_java_uncompress(C.addressof(buf) + 16, len(data) - 16, C.byref(n),
                                              err, 128)
        if not p:
            return RESP_ERR__BAD_COMPRESSION, b""
        out = C.string_at(p, n.value)
        _libc().free(p)
        return 0, out
    L.rd_kafka_snappy_uncompressed_length.restype = C.c_bool
    L.rd_kafka_snappy_uncompressed_length.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    n = C.c_size_t(0)
    if not L.rd_kafka_snappy_uncompressed_length(buf, len(data), C.byref(n)):
        return RESP_ERR__BAD_COMPRESSION, b""
    out = C.create_string_buffer(max(1, n.value))
    L.rd_kafka_snappy_uncompress.restype = C.c_int
    L.rd_kafka_snappy_uncompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
    if L.rd_kafka_snappy_uncompress(buf, len(data), out):
        return RESP_ERR__BAD_COMPRESSION, b""
    return 0, out.raw[:n.value]


def lz4f_decompress_batch_noalloc(src, in_offs, in_lens, dst, out_offs, out_caps, out_lens,
                                  status, stream=None):
    """rdk_hip_lz4f_decompress_noalloc: the batch decoder on the library's fixed device
    scratch (no allocation; at most LZ4F_NOALLOC_MAX_FRAMES frames; init() first)."""
    _check(lib().rdk_hip_lz4f_decompress_noalloc(_ptr(src), _ptr(in_offs), _ptr(in_lens),
                                                 _ptr(dst), _ptr(out_offs), _ptr(out_caps),
                                                 _ptr(out_lens), _ptr(status),
                                                 int(in_offs.numel()), _stream(stream)),
           "lz4f_decompress_noalloc")


PRODUCER_EXACT, PRODUCER_FAST, PRODUCER_SNAPPY = 0, 1, 2
E_BUSY = -5


def msgset_v2_finalize(src, rec_offs, rec_lens, dst, out_offs, out_caps, frame_lens, batch_lens,
                       crcs, mode=PRODUCER_EXACT, stream=None) -> None:
    """rdk_hip_msgset_v2_finalize: the writer's compress + header finalize + CRC32C
    (rdkafka_msgset_writer.c:1335) for device-resident MessageSets."""
    _check(lib().rdk_hip_msgset_v2_finalize(_ptr(src), _ptr(rec_offs), _ptr(rec_lens), _ptr(dst),
                                            _ptr(out_offs), _ptr(out_caps), _ptr(frame_lens),
                                            _ptr(batch_lens), _ptr(crcs), int(rec_offs.numel()),
                                            mode, _stream(stream)), "msgset_v2_finalize")


class _Batch(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_uint32), ("crc", C.c_uint32),
                ("cookie", C.c_uint64)]


class Producer:
    """Producer batching front-end (include/librdkafka_hip.h rdk_hip_producer_*):
    a pinned staging ring whose slots run H2D -> LZ4F compress -> v2 header
    finalize -> CRC32C -> D2H on their own streams.  One per broker thread."""

    def __init__(self, device: int = 0, slot_bytes: int = 64 << 20, nslots: int = 4,
                 mode: int = PRODUCER_FAST):
        self._p = lib().rdk_hip_producer_new(device, slot_bytes, nslots, mode)
        if not self._p:
            raise EngineError("rdk_hip_producer_new: " + lib().rdk_hip_last_error().decode())
        self._out = (_Batch * 4096)()

    def produce(self, header61, records, cookie: int = 0) -> int:
        """0, or E_BUSY when every slot is in flight (poll() first)."""
        rc = lib().rdk_hip_producer_produce(self._p, header61, records, len(records), cookie)
        if rc not in (0, E_BUSY):
            _check(rc, "rdk_hip_producer_produce")
        return rc

    def flush(self) -> None:
        _check(lib().rdk_hip_producer_flush(self._p), "rdk_hip_producer_flush")

    def poll(self, block: bool = True, copy: bool = True):
        """[(cookie, batch_bytes, crc)] of the finished batches (copies), or
        [(cookie, (ptr, len), crc)] with copy=False (valid until the next
        produce()/flush())."""
        n = lib().rdk_hip_producer_poll(self._p, self._out, len(self._out), int(block))
        if n < 0:
            _check(n, "rdk_hip_producer_poll")
        res = []
        for b in self._out[:n]:
            res.append((b.cookie, C.string_at(b.data, b.len) if copy else (b.data, b.len), b.crc))
        return res

    def close(self) -> None:
        if self._p:
            lib().rdk_hip_producer_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gen_v2_batches(base, n: int, batch_size: int, seed: int = 0x5EED, stream=None) -> None:
    _check(lib().rdk_hip_gen_v2_batches(_ptr(base), n, batch_size, seed, _stream(stream)),
           "gen_v2_batches")


def gen_json(n: int, seed: int = 42) -> bytes:
    """Native JSON-like record generator (same bytes as workload.gen_json)."""
    b = C.create_string_buffer(max(1, n))
    lib().rdk_hip_gen_json(b, n, seed)
    return b.raw[:n]


def msgset_v2_build(msgs: dict, batches: np.ndarray, crc: bool = True, stream=None):
    """MsgVersion 2 record serialisation on the device (rdkafka_msgset_writer.c:352-403,
    :652-754, :1251-1295).  `msgs`: cuda tensors arena (u8), ts (i64), key_off (i64),
    key_len (i32), val_off (i64), val_len (i32) and optionally hdr_off (i64),
    hdr_len (i32), hdr_cnt (i32); `batches`: numpy array of V2_BATCH_DTYPE.
    Returns (out u8 tensor, out_offs i64 tensor, batch_sizes i32 tensor, crcs i32 tensor
    or None)."""
    n = len(batches)
    dev = msgs["arena"].device
    m = _Msgs(*(None if msgs.get(k) is None else msgs[k].data_ptr() for k in
                ("arena", "ts", "key_off", "key_len", "val_off", "val_len", "hdr_off", "hdr_len",
                 "hdr_cnt")))
    hb = np.ascontiguousarray(batches, V2_BATCH_DTYPE)
    nmsg = int(msgs["ts"].numel())
    rec_offs = torch.empty(max(nmsg, 1), dtype=torch.int32, device=dev)
    sizes = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    max_ts = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    s = _stream(stream)
    _check(lib().rdk_hip_msgset_v2_sizes(C.byref(m), hb.ctypes.data, n, _ptr(rec_offs), _ptr(sizes),
                                         _ptr(max_ts), s), "msgset_v2_sizes")
    sz64 = sizes[:n].to(torch.int64)
    offs = torch.cumsum(sz64, 0) - sz64
    total = int(sz64.sum()) if n else 0
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    crcs = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if crc else None
    _check(lib().rdk_hip_msgset_v2_write(C.byref(m), hb.ctypes.data, n, _ptr(rec_offs),
                                         _ptr(sizes), _ptr(max_ts), _ptr(offs), _ptr(out),
                                         _ptr(crcs), s), "msgset_v2_write")
    return out, offs, sizes[:n], (crcs[:n] if crc else None)


def msgset_v2_index(hdr_base, hdr_offs, rec_base, rec_offs, rec_lens, row_offs, row_caps,
                    rows: dict, count, stream=None) -> None:
    """MsgVersion 2 record index on the device (rdkafka_msgset_reader.c:715-927): `rows`
    holds cuda tensors named as V2_ROW_FIELDS; count[i] = records of batch i or
    -(1+j) when record j fails to parse."""
    r = _Rows(*(rows[k].data_ptr() for k, _ in V2_ROW_FIELDS))
    _check(lib().rdk_hip_msgset_v2_index(_ptr(hdr_base), _ptr(hdr_offs), _ptr(rec_base),
                                         _ptr(rec_offs), _ptr(rec_lens), _ptr(row_offs),
                                         _ptr(row_caps), C.byref(r), _ptr(count),
                                         int(hdr_offs.numel()), _stream(stream)),
           "msgset_v2_index")
