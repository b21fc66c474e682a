"""Deterministic synthetic workloads.

* JSON-like record stream (the compress / decompress / producer configurations): records
  ``{"id":N,"user":"uUUUUU","ts":T,"event":"E","value":V.FF}\\n`` drawn from
  the LCG ``s = s*1103515245 + 12345 (mod 2^32)``, each draw using ``s >> 8``;
  seed 42.  Byte-identical to the native ``rdk_hip_gen_json``.
* MsgVersion 2 record batches (the CRC32C-only configuration): 61-byte big-endian v2
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


def gen_messages(n: int, seed: int = 42, headers: bool = True) -> dict:
    """Synthetic producer messages for the MsgVersion 2 record writer (numpy SoA).

    Values are JSON-like records (`gen_json` lines, ~95 B); keys are "k<id>"
    (every 7th null, every 11th empty); every 13th value is null; timestamps
    advance 0-3 ms with every 17th message stepping back (negative deltas);
    every 5th message carries 1-2 headers, serialised as on the wire
    (varint name length, name, varint value length, value;
    rdkafka_msgset_writer.c:558-568).
    """
    def zz(v):
        u = (v << 1) ^ (v >> 63)
        u &= (1 << 64) - 1
        out = bytearray()
        while True:
            out.append((u & 0x7F) | (0x80 if u > 0x7F else 0))
            u >>= 7
            if not u:
                return bytes(out)
    lines = gen_json(n * 100 + 4096, seed).split(b"\n")
    arena = bytearray()
    ts = np.zeros(n, np.int64)
    key_off = np.zeros(n, np.uint64); key_len = np.zeros(n, np.int32)
    val_off = np.zeros(n, np.uint64); val_len = np.zeros(n, np.int32)
    hdr_off = np.zeros(n, np.uint64); hdr_len = np.zeros(n, np.uint32)
    hdr_cnt = np.zeros(n, np.int32)
    t = 1600000000000
    s = seed & 0xFFFFFFFF
    for i in range(n):
        s = (s * 1103515245 + 12345) & 0xFFFFFFFF
        t += (s >> 8) % 4 if i % 17 else -((s >> 8) % 50)
        ts[i] = t
        if i % 7 == 0:
            key_len[i] = -1
        else:
            k = b"" if i % 11 == 0 else b"k%d" % i
            key_off[i] = len(arena); key_len[i] = len(k); arena += k
        if i % 13 == 0:
            val_len[i] = -1
        else:
            v = lines[i % len(lines)]
            val_off[i] = len(arena); val_len[i] = len(v); arena += v
        if headers and i % 5 == 0:
            h = bytearray()
            for j in range(1 + (i // 5) % 2):
                name, val = b"h%d" % j, (b"v%d" % i if j == 0 else None)
                h += zz(len(name)) + name
                h += zz(len(val)) + val if val is not None else zz(-1)
            hdr_off[i] = len(arena); hdr_len[i] = len(h); hdr_cnt[i] = 1 + (i // 5) % 2
            arena += h
    return {"arena": np.frombuffer(bytes(arena) or b"\0", np.uint8).copy(), "ts": ts,
            "key_off": key_off, "key_len": key_len, "val_off": val_off, "val_len": val_len,
            "hdr_off": hdr_off, "hdr_len": hdr_len, "hdr_cnt": hdr_cnt}


def msgset_v01_bytes(msgs: dict, first: int, cnt: int, magic: int = 1,
                     base_offset: int = 0, max_bytes: int | None = None) -> bytes:
    """Uncompressed MsgVersion 0/1 MessageSet of messages [first, first+cnt) in the layout of
    rd_kafka_msgset_writer_write_msg_v0_1 (rdkafka_msgset_writer.c:583-645), with the Crc
    fields left 0: the engine's FINALIZE mode fills them.  Stops before max_bytes."""
    arena = msgs["arena"]
    out = bytearray()
    for k in range(cnt):
        m = first + k
        kl, vl = int(msgs["key_len"][m]), int(msgs["val_len"][m])
        kb, vb = max(kl, 0), max(vl, 0)
        size = 4 + 1 + 1 + 4 + kb + 4 + vb + (8 if magic == 1 else 0)
        if max_bytes is not None and len(out) + 12 + size > max_bytes:
            break
        out += struct.pack(">qiIbb", base_offset + k, size, 0, magic, 0)
        if magic == 1:
            out += struct.pack(">q", int(msgs["ts"][m]))
        ko, vo = int(msgs["key_off"][m]), int(msgs["val_off"][m])
        out += struct.pack(">i", kl if kl >= 0 else -1) + arena[ko:ko + kb].tobytes()
        out += struct.pack(">i", vl if vl >= 0 else -1) + arena[vo:vo + vb].tobytes()
    return bytes(out)


PERF_PATTERN = b"librdkafka_performance testing!"   # examples/rdkafka_performance.c:798


def gen_perf_messages(n: int, msgsize: int = 100, msgs_per_ms: int = 800) -> dict:
    """The messages of `rdkafka_performance -P -s msgsize -c n`: every value is the pattern
    repeated to msgsize bytes (examples/rdkafka_performance.c:1318-1325; all messages share
    the one payload buffer), no key, no headers; timestamps are the produce() wall clock,
    here advancing one millisecond every `msgs_per_ms` messages."""
    value = (PERF_PATTERN * (msgsize // len(PERF_PATTERN) + 1))[:msgsize]
    z32, z64 = np.zeros(n, np.int32), np.zeros(n, np.uint64)
    return {"arena": np.frombuffer(value or b"\0", np.uint8).copy(),
            "ts": 1600000000000 + np.arange(n, dtype=np.int64) // msgs_per_ms,
            "key_off": z64.copy(), "key_len": np.full(n, -1, np.int32),
            "val_off": z64.copy(), "val_len": np.full(n, msgsize, np.int32),
            "hdr_off": z64.copy(), "hdr_len": np.zeros(n, np.uint32), "hdr_cnt": z32.copy()}


def _zz_width(v: int) -> int:
    u = ((v << 1) ^ (v >> 63)) & ((1 << 64) - 1)
    w = 1
    while u > 0x7F:
        u >>= 7
        w += 1
    return w


def perf_batches(msgs: dict, batch_num_messages: int = 10000, message_max_bytes: int = 1000000,
                 request_overhead: int = 55) -> list[tuple[int, int]]:
    """(first, count) of the MessageSets rd_kafka_msgset_writer_write_msgq
    (rdkafka_msgset_writer.c:804-902) cuts a toppar's queue into: a batch ends at
    batch.num.messages (rdkafka_conf.c:1155) or when the request buffer so far plus the next
    message's estimated wire size (value + key + RD_KAFKAP_MESSAGE_V2_OVERHEAD = 36,
    rdkafka_proto.h:508-524) would pass message.max.bytes (:859-863).  `request_overhead` is
    the ProduceRequest framing in front of the MessageSet (55 bytes for topic "perftest",
    client.id "rdkafka", ApiVersion 7)."""
    n = len(msgs["ts"])
    out, first = [], 0
    while first < n:
        length = request_overhead + V2_HEADER
        cnt = 0
        base_ts = int(msgs["ts"][first])
        while first + cnt < n and cnt < batch_num_messages:
            m = first + cnt
            kl, vl = int(msgs["key_len"][m]), int(msgs["val_len"][m])
            if cnt > 0 and length + 36 + max(kl, 0) + max(vl, 0) > message_max_bytes:
                break
            body = (1 + _zz_width(int(msgs["ts"][m]) - base_ts) + _zz_width(cnt) + _zz_width(kl) +
                    max(kl, 0) + _zz_width(vl) + max(vl, 0) + _zz_width(int(msgs["hdr_cnt"][m])) +
                    int(msgs["hdr_len"][m]))
            length += _zz_width(body) + body
            cnt += 1
        out.append((first, cnt))
        first += cnt
    return out
