"""Snappy streams assembled element by element for the decoder tests: every tag kind and
every literal-length encoding (snappy.c:652 emit_literal, :697 emit_copy_less_than64; the
4-byte-offset copy only a foreign writer makes), lengths and offsets at their limits."""

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
