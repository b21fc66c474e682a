"""Soak of the combined drop-in path: 8 Python threads x N iterations over all symbols, mixed
sizes and levels, every result against the oracle; prints the combine counters."""
import os
import random
import sys
import threading
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import librdkafka_amd as L
import oracle

N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
L.init(0)
rnd0 = random.Random(11)
inputs = []
for i in range(40):
    n = rnd0.choice([0, 1, 12, 13, 100, 4096, 16384, 65536, 65537, 100000, 300000, rnd0.randrange(1, 200000)])
    inputs.append(L.gen_json(n, 500 + i) if i % 4 else bytes(rnd0.randrange(8) for _ in range(n)))
want = {}
for i, d in enumerate(inputs):
    want[i] = (oracle.crc32c(0, d), oracle.crc32(0, d), oracle.rdk_lz4_compress(d)[1],
               oracle.rdk_lz4_compress(d, comp_level=4)[1] if i % 5 == 0 else None)
bad = []
stop = threading.Event()


def worker(t):
    rnd = random.Random(100 + t)
    L.init(0)
    for it in range(N):
        if stop.is_set():
            return
        i = rnd.randrange(len(inputs))
        d = inputs[i]
        c32c, c32, frame, hc = want[i]
        op = rnd.randrange(6)
        ok = True
        if op == 0:
            ok = L.crc32c(0, d) == c32c
        elif op == 1:
            k = rnd.randrange(len(d) + 1)
            ok = L.rd_slice_crc32c([d[:k], d[k:]]) == c32c
        elif op == 2:
            ok = L.rd_slice_crc32([d]) == c32
        elif op == 3:
            ok = L.rd_kafka_lz4_compress(1, 0, d) == (0, frame)
        elif op == 4:
            ok = L.rd_kafka_lz4_decompress(1, 0, frame) == (0, d)
        elif hc is not None:
            ok = L.rd_kafka_lz4_compress(1, 4, d) == (0, hc)
        if not ok:
            bad.append((t, it, i, op))
            stop.set()


t0 = time.time()
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[t.start() for t in ths]
[t.join() for t in ths]
print("SOAK", "FAILED" if bad else "OK", bad[:3], "combined", L.dropin_combined(), "host_crcs", L.dropin_host_crcs(),
      f"{time.time() - t0:.1f} s", flush=True)
sys.exit(1 if bad else 0)
