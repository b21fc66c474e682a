"""Deterministic synthetic workloads (DESIGN.md "Workloads").

* JSON-like record stream (BASELINE configs 3-5): records
  ``{"id":N,"user":"uUUUUU","ts":T,"event":"E","value":V.FF}\\n`` drawn from
  the LCG ``s = s*1103515245 + 12345 (mod 2^32)``, each draw using ``s >> 8``;
  seed 42.  Byte-identical to the native ``rdk_hip_gen_json``.
* MsgVersion 2 record batches (BASELINE config 2): 61-byte big-endian v2
  header (rdkafka_msgset_writer.c:352-403) + splitmix64 bytes; every 8-byte
  word w of the buffer is ``splitmix64(seed + w)`` (seed 0x5EED), identical
  to the device generator ``rdk_hip_gen_v2_batches``.
"""
from __future__ import annotations

import struct

import numpy as np

EVENTS = ("click", "view", "purchase", "scroll")
V2_HEADER = 61          # RD_KAFKAP_MSGSET_V2_SIZE, rdkafka_proto.h:540
V2_OF_LENGTH = 8
V2_OF_CRC = 17
V2_OF_ATTRIBUTES = 21


def gen_json(n: int, seed: int = 42) -> bytes:
    out = bytearray()
    s = seed & 0xFFFFFFFF
    rid = 0
    while len(out) < n:
        vals = []
        for _ in range(5):
            s = (s * 1103515245 + 12345) & 0xFFFFFFFF
            vals.append(s >> 8)
        user, ts, ev, v, f = vals
        out += (f'{{"id":{rid},"user":"u{user % 100000:05d}","ts":{1600000000 + ts % 86400},'
                f'"event":"{EVENTS[ev & 3]}","value":{v % 10000}.{f % 100:02d}}}\n').encode()
        rid += 1
    return bytes(out[:n])


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def v2_header(batch_index: int, batch_size: int) -> bytes:
    records = (batch_size - 61) // 100 + 1
    return struct.pack(">qiibIhiqqqhii", batch_index * records, batch_size - 12, 0, 2, 0, 0,
                       records - 1, 1600000000000 + batch_index, 1600000000000 + batch_index + 1,
                       -1, -1, -1, records)


def gen_v2_batches(n: int, batch_size: int, seed: int = 0x5EED) -> bytearray:
    """Host twin of rdk_hip_gen_v2_batches (CRC field 0)."""
    assert batch_size % 8 == 0 and batch_size >= V2_HEADER
    with np.errstate(over="ignore"):
        words = splitmix64(np.arange(n * batch_size // 8, dtype=np.uint64) + np.uint64(seed))
    buf = bytearray(words.astype("<u8").tobytes())
    for b in range(n):
        buf[b * batch_size:b * batch_size + V2_HEADER] = v2_header(b, batch_size)
    return buf


def json_v2_batch(payload: bytes, base_offset: int = 0) -> bytearray:
    """An uncompressed-looking v2 batch whose record area is `payload`."""
    hdr = bytearray(v2_header(0, V2_HEADER + len(payload) + ((8 - (V2_HEADER + len(payload)) % 8) % 8)))
    struct.pack_into(">i", hdr, V2_OF_LENGTH, V2_HEADER + len(payload) - 12)
    return hdr + payload
