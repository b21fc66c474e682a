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

import librdkafka_amd as L  # noqa: E402
import oracle  # noqa: E402

FRAG = 1 << 16


def varint(n):
    out = bytearray()
    while n >= 128:
        out.append((n & 127) | 128)
        n >>= 7
    out.append(n)
    return bytes(out)


def literal(rnd, data, wide):
    n = len(data) - 1
    if n < 60 and not wide:
        return bytes([n << 2]) + data
    nb = max(1, (n.bit_length() + 7) // 8)
    if wide:
        nb = rnd.randrange(nb, 4)  # more length bytes than needed
    return bytes([(59 + nb) << 2]) + n.to_bytes(nb, "little") + data


def copy(rnd, length, off, kind):
    if kind == 1:
        return bytes([1 | ((length - 4) << 2) | ((off >> 8) << 5), off & 255])
    if kind == 2:
        return bytes([2 | ((length - 1) << 2)]) + off.to_bytes(2, "little")
    return bytes([3 | ((length - 1) << 2)]) + off.to_bytes(4, "little")


def stream(rnd, total, fenced, far):
    """fenced: no element or copy crosses a multiple of 64 KiB; far: 4-byte offsets appear"""
    out = bytearray()
    st = bytearray()
    while len(out) < total:
        room = total - len(out)
        if fenced:
            room = min(room, FRAG - len(out) % FRAG)
        reach = len(out) % FRAG if fenced else len(out)
        r = rnd.random()
        if reach == 0 or r < 0.3:
            n = rnd.choice([1, 2, rnd.randrange(1, 61), 60, 61, rnd.randrange(61, 300), 256, 257,
                            rnd.randrange(300, 70000)])
            n = min(n, room)
            data = rnd.randbytes(n)
            st += literal(rnd, data, n <= 1 << 16 and rnd.random() < 0.1)
            out += data
            continue
        kind = 1 if r < 0.6 else 2 if (r < 0.97 or not far) else 3
        if kind == 1:
            length = rnd.randrange(4, 12)
            off = rnd.choice([1, 2, rnd.randrange(1, 2048), 2047])
        else:
            length = rnd.choice([1, 2, 64, rnd.randrange(1, 65)])
            off = rnd.choice([1, rnd.randrange(1, 65536), 65535, reach])
        length = min(length, room)
        off = max(1, min(off, reach, 65535 if kind != 3 else reach))
        if kind == 1 and (length < 4 or off > 2047):
            kind = 2
        st += copy(rnd, length, off, kind)
        for _ in range(length):
            out.append(out[-off])
    return varint(len(out)) + bytes(st), bytes(out)


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
