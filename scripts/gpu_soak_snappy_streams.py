"""Element-level soak of the snappy decoders on the GPU: streams assembled element by element
(every tag kind and every literal-length encoding, lengths and offsets at their limits), some
that keep every element and copy inside one 64 KiB fragment of the output and some that do
not, some damaged; error code and output must equal the oracle's.
Usage: gpu_soak_snappy_streams.py FIRST_SEED N_CASES."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import librdkafka_amd as L  # noqa: E402
import oracle  # noqa: E402

from snappy_streams import FRAG, stream  # noqa: E402


def main():
    first, cases = int(sys.argv[1]), int(sys.argv[2])
    rnd = random.Random(first)
    split = 0
    for it in range(cases):
        total = rnd.choice([rnd.randrange(1, 3000), rnd.randrange(FRAG - 300, FRAG + 300),
                            rnd.randrange(FRAG, 5 * FRAG), 2 * FRAG, 3 * FRAG + 1])
        fenced = rnd.random() < 0.6
        st, want = stream(rnd, total, fenced, rnd.random() < 0.2)
        mode = rnd.randrange(4)
        if mode == 0:  # damaged
            b = bytearray(st)
            for _ in range(rnd.randrange(1, 4)):
                b[rnd.randrange(len(b))] = rnd.getrandbits(8)
            st = bytes(b)
            n = oracle.snappy_uncompressed_length(st)
            if n is not None and n > (64 << 20):
                continue
        elif mode == 1 and len(st) > 4:
            st = st[:rnd.randrange(2, len(st))]
        r1 = L.rd_kafka_snappy_decompress(st)
        r2 = oracle.rdk_snappy_decompress(st)
        assert r1 == r2, ("snappy", first, it, total, fenced, mode, r1[0], r2[0])
        if mode >= 2:
            assert r2[0] == 0 and r2[1] == want, ("generator", first, it)
            split += fenced and total > FRAG
        if (it + 1) % 500 == 0:
            print(f"{it + 1} cases ok ({split} intact fenced multi-fragment streams)", flush=True)
    print(f"STREAMS_OK {cases} cases, {split} intact fenced multi-fragment streams")


if __name__ == "__main__":
    main()
