"""Verdict soak on the GPU: frames and snappy streams made by the oracle, damaged (byte
edits, truncation, extension), through the drop-in decoders; error code and output must
equal the oracle's for every case.  Usage: gpu_soak_verdicts.py FIRST_SEED N_CASES."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import librdkafka_amd as L  # noqa: E402
from librdkafka_amd import workload as W  # noqa: E402
import oracle  # noqa: E402


def damage(rnd, fr, lo):
    fr = bytearray(fr)
    kind = rnd.randrange(5)
    if kind == 0 and len(fr) > lo + 2:
        del fr[rnd.randrange(lo, len(fr)):]
    elif kind == 1:
        fr += rnd.randbytes(rnd.randrange(1, 9))
    else:
        for _ in range(rnd.randrange(1, 5)):
            fr[rnd.randrange(lo, max(lo + 1, len(fr)))] = rnd.getrandbits(8)
    return bytes(fr)


def source(rnd, it):
    n = rnd.choice([rnd.randrange(20, 400), rnd.randrange(400, 9000), rnd.randrange(60000, 140000)])
    kind = it % 4
    if kind == 0:
        return W.gen_json(n, 7000 + it)
    if kind == 1:
        words = [rnd.randbytes(rnd.randrange(2, 9)) for _ in range(60)]
        return b" ".join(rnd.choice(words) for _ in range(n // 4 + 1))[:n]
    if kind == 2:
        p = rnd.randbytes(rnd.randrange(1, 40))
        return (p * (n // len(p) + 1))[:n]
    return W.gen_json(n // 2, it) + rnd.randbytes(n - n // 2)


def main():
    first, cases = int(sys.argv[1]), int(sys.argv[2])
    rnd = random.Random(first)
    bad = 0
    for it in range(cases):
        src = source(rnd, it)
        fr = damage(rnd, oracle.rdk_lz4_compress(src)[1], 4)
        e1, o1 = L.rd_kafka_lz4_decompress(1, 0, fr)
        e2, o2 = oracle.rdk_lz4_decompress(fr)
        assert e1 == e2 and o1 == o2, ("lz4", first, it, len(src), e1, e2)
        bad += e2 != 0
        st = damage(rnd, oracle.snappy_compress(src), 0)
        n = oracle.snappy_uncompressed_length(st)
        if n is None or n <= (64 << 20):  # (a damaged preamble may declare gigabytes)
            r1 = L.rd_kafka_snappy_decompress(st)
            r2 = oracle.rdk_snappy_decompress(st)
            assert r1 == r2, ("snappy", first, it, len(src), r1[0], r2[0])
        if (it + 1) % 500 == 0:
            print(f"{it + 1} cases ok ({bad} lz4 frames rejected so far)", flush=True)
    print(f"VERDICTS_OK {cases} cases, {bad} rejected lz4 frames")


if __name__ == "__main__":
    main()
