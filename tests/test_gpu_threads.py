"""Concurrent drop-in calls from several host threads (the reference calls these symbols from
every broker thread at once, rdkafka_broker.c:5082; three in configs[0]).  Every result is
compared with the oracle and the run stops at the first mismatch.  Concurrent calls are
served together (one staging copy, one launch per batch kernel): the counters must show
that this happened, and the results must not depend on it."""
import ctypes as C
import os
import random
import subprocess
import sys
import threading

import pytest

import librdkafka_amd as L
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inputs():
    rnd = random.Random(5)
    sizes = [0, 1, 11, 12, 13, 61, 100, 4095, 4096, 4097, 16384, 65535, 65536, 65537, 200000, 1 << 20]
    out = []
    for i, n in enumerate(sizes):
        data = L.gen_json(n, 100 + i) if i % 3 else bytes(rnd.randrange(256 if i % 2 else 4) for _ in range(n))
        out.append(data)
    return out


def test_four_symbols_from_six_threads():
    L.init(0)
    inputs = _inputs()
    want = []
    for d in inputs:
        err, frame = oracle.rdk_lz4_compress(d)
        assert err == 0
        want.append((oracle.crc32c(0, d), oracle.crc32c(0x1234ABCD, d), frame))
    hc_frames = {}
    for i in (6, 10, 14):  # compression.level 9 and the legacy (!proper_hc) framing
        hc_frames[i] = (oracle.rdk_lz4_compress(inputs[i], comp_level=9)[1],
                        oracle.rdk_lz4_compress(inputs[i], proper_hc=0)[1])
    stop = threading.Event()
    errors = []
    before = L.dropin_combined()
    host_before = L.dropin_host_crcs()

    def fail(msg):
        errors.append(msg)
        stop.set()

    def worker(t):
        rnd = random.Random(t)
        L.init(0)
        for it in range(60):
            if stop.is_set():
                return
            i = rnd.randrange(len(inputs))
            d = inputs[i]
            crc0, crc1, frame = want[i]
            if L.crc32c(0, d) != crc0 or L.crc32c(0x1234ABCD, d) != crc1:
                return fail(f"crc32c thread {t} input {i}")
            cut = min(len(d), 61)
            mid = max(cut, len(d) // 2)
            if L.rd_slice_crc32c([d[:cut], d[cut:mid], d[mid:]]) != crc0:
                return fail(f"rd_slice_crc32c thread {t} input {i}")
            if L.rd_slice_crc32([d[:cut], d[cut:]]) != oracle.crc32(0, d):
                return fail(f"rd_slice_crc32 thread {t} input {i}")
            err, got = L.rd_kafka_lz4_compress(1, 0, [d[:cut], d[cut:]])
            if err or got != frame:
                return fail(f"rd_kafka_lz4_compress thread {t} input {i} err {err}")
            err, back = L.rd_kafka_lz4_decompress(1, 0, frame)
            if err or back != d:
                return fail(f"rd_kafka_lz4_decompress thread {t} input {i} err {err}")
            if i in hc_frames and it % 3 == 0:
                err, got = L.rd_kafka_lz4_compress(1, 9, d)
                if err or got != hc_frames[i][0]:
                    return fail(f"level 9 thread {t} input {i} err {err}")
                err, got = L.rd_kafka_lz4_compress(0, 0, d)
                if err or got != hc_frames[i][1]:
                    return fail(f"legacy framing thread {t} input {i} err {err}")
                err, back = L.rd_kafka_lz4_decompress(0, 0, bytearray(got))
                if err or back != d:
                    return fail(f"legacy framing decompress thread {t} input {i} err {err}")
            if it % 20 == 7:
                err, back = L.rd_kafka_lz4_decompress(1, 0, b"\x04\x22\x4d\x18" + b"\xff" * 40)
                if err != L.RESP_ERR__BAD_COMPRESSION and err != L.RESP_ERR__BAD_MSG:
                    return fail(f"bad frame thread {t}: err {err}")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[0]
    after = L.dropin_combined()
    assert after[0] > before[0], "no two calls were ever served together"
    assert after[1] - before[1] >= 2 * (after[0] - before[0])
    assert after[3] == before[3], "a combined batch fell back to single requests"
    assert L.dropin_host_crcs() == host_before


def test_native_threads_every_symbol():
    """8 native threads in a tight loop on each symbol (bench_native/dropin_threads.c): right
    results, and the calls were combined."""
    L.init(0)
    lib = L.lib()
    T = C.CDLL(os.path.join(ROOT, "bench_native", "libdropin_threads.so"))
    T.dropin_threads_run.restype = C.c_double
    T.dropin_threads_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_size_t,
                                     C.c_int, C.c_double]
    data = L.gen_json(16384, 7)
    err, frame = oracle.rdk_lz4_compress(data)
    buf = C.create_string_buffer(data, len(data))
    fbuf = C.create_string_buffer(frame, len(frame))
    crc = oracle.crc32c(0, data)
    before = L.dropin_combined()
    for which, fn, b, n, xl in ((0, lib.crc32c, buf, len(data), 0),
                                (1, lib.rd_slice_crc32c, buf, len(data), 0),
                                (2, lib.rd_kafka_lz4_compress, buf, len(data), len(frame)),
                                (3, lib.rd_kafka_lz4_decompress, fbuf, len(frame), len(data))):
        print(f"native threads: symbol {which}", flush=True)
        us = T.dropin_threads_run(which, C.cast(fn, C.c_void_p), b, n, crc, xl, 8, 0.2)
        assert us > 0, f"symbol {which}: wrong result under 8 threads"
    after = L.dropin_combined()
    assert after[0] > before[0] and after[2] >= 2
    assert after[3] == before[3]


def test_uncombined_switch():
    """RDK_HIP_COMBINE=0: the same calls, each on its own thread's stream."""
    code = (
        "import threading, librdkafka_amd as L, oracle\n"
        "L.init(0)\n"
        "d = L.gen_json(70000, 3); f = oracle.rdk_lz4_compress(d)[1]; bad = []\n"
        "def w():\n"
        "    for _ in range(20):\n"
        "        if L.crc32c(0, d) != oracle.crc32c(0, d): bad.append('crc')\n"
        "        if L.rd_kafka_lz4_compress(1, 0, d) != (0, f): bad.append('c')\n"
        "        if L.rd_kafka_lz4_decompress(1, 0, f) != (0, d): bad.append('d')\n"
        "ts = [threading.Thread(target=w) for _ in range(4)]\n"
        "[t.start() for t in ts]; [t.join() for t in ts]\n"
        "assert not bad, bad\n"
        "assert L.dropin_combined()[0] == 0\n"
        "print('ok')\n")
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, RDK_HIP_COMBINE="0", PYTHONPATH=ROOT),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-2000:]
