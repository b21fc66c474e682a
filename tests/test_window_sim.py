"""The windowed exact LZ4 parse (host model of the HIP kernel's algorithm,
tests/sim/lz4_window_sim.cpp) against the oracle's restatement of LZ4_compress_generic:
byte-identical blocks on compressible, incompressible, repetitive and edge-size inputs."""
import ctypes as C
import os
import random
import subprocess

import pytest

from librdkafka_amd import workload as W

HERE = os.path.dirname(os.path.abspath(__file__))
SIM_SRC = os.path.join(HERE, "sim", "lz4_window_sim.cpp")
SIM_LIB = os.path.join(HERE, "sim", "libwindowsim.so")


@pytest.fixture(scope="module")
def sim():
    if not os.path.exists(SIM_LIB) or os.path.getmtime(SIM_LIB) < os.path.getmtime(SIM_SRC):
        subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", SIM_LIB, SIM_SRC], check=True)
    lib = C.CDLL(SIM_LIB)
    lib.sim_lz4_window_block.restype = C.c_int
    lib.sim_lz4_window_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    return lib


def _both(sim, oracle_mod, data):
    n = len(data)
    src = C.create_string_buffer(bytes(data), max(1, n))
    d1 = C.create_string_buffer(n + 64)
    d2 = C.create_string_buffer(n + 64)
    stats = (C.c_long * 6)()
    c1 = sim.sim_lz4_window_block(src, n, d1, n - 1, stats)
    c2 = oracle_mod.lib().or_lz4_compress_block(src, n, d2, n - 1, 1)
    return c1, d1.raw[:max(c1, 0)], c2, d2.raw[:max(c2, 0)], list(stats)


def _inputs(seed, count):
    rnd = random.Random(seed)
    out = []
    sizes = [13, 14, 15, 16, 17, 20, 63, 64, 65, 66, 67, 76, 77, 78, 79, 80, 127, 128, 129, 130,
             140, 141, 1000, 4095, 4096, 65535, 65536] + [rnd.randrange(13, 65537) for _ in range(count)]
    for i, n in enumerate(sizes):
        kind = i % 8
        if kind == 0:
            out.append(W.gen_json(n, i))
        elif kind == 1:
            out.append(rnd.randbytes(n))
        elif kind == 2:
            out.append(bytes(n))
        elif kind == 3:
            base = rnd.randbytes(max(1, n // 50))
            out.append((base * 60)[:n])
        elif kind == 4:
            words = [rnd.randbytes(rnd.randrange(2, 9)) for _ in range(200)]
            out.append(b" ".join(rnd.choice(words) for _ in range(n // 4 + 1))[:n])
        elif kind == 5:   # small alphabet: many short in-window repeats
            a = rnd.choice([2, 3, 4, 8])
            out.append(bytes(rnd.randrange(a) for _ in range(n)))
        elif kind == 6:   # sparse matches: long searches with strides above 1, then a match
            b = bytearray(rnd.randbytes(n))
            for _ in range(max(1, n // 3000)):
                if n > 200:
                    s = rnd.randrange(0, n - 100)
                    d = rnd.randrange(0, n - 100)
                    ln = rnd.randrange(4, 90)
                    b[d:d + ln] = b[s:s + ln]
            out.append(bytes(b[:n]))
        else:             # runs: period 1..7
            p = rnd.randbytes(rnd.randrange(1, 8))
            out.append((p * (n // len(p) + 1))[:n])
    return out


def test_window_parse_is_byte_identical_to_the_oracle(sim, oracle_mod):
    tot = [0] * 6
    for i, data in enumerate(_inputs(1, 400)):
        c1, b1, c2, b2, st = _both(sim, oracle_mod, data)
        assert c1 == c2 and b1 == b2, (i, len(data), c1, c2)
        tot = [a + b for a, b in zip(tot, st)]
    # every path of the model ran: windows, the stride>1 search, in-window candidates,
    # matches longer than the register window, catch-ups longer than the register window
    assert all(t > 0 for t in tot), tot


def test_window_parse_json_megabyte_blocks(sim, oracle_mod):
    data = W.gen_json(1 << 20, 42)
    for k in range(16):
        blk = data[k * 65536:(k + 1) * 65536]
        c1, b1, c2, b2, st = _both(sim, oracle_mod, blk)
        assert c1 == c2 and b1 == b2, k
        # on JSON nearly every sequence is found by the windows, not the stride>1 search
        assert st[1] < st[0] // 20
