"""CPU oracle pinned against the reference's KATs, golden frames made by the
reference's own LZ4F build, and (when oracle/_ref is built) live differential
fuzzing against the reference sources."""
import hashlib
import random

import pytest

from librdkafka_amd import workload as W


def sha(b):
    return hashlib.sha256(b).hexdigest()


# ----------------------------------------------------------------- CRC32C
def test_crc32c_reference_kat(oracle_mod, golden):
    kat = golden("crc32c_kat.json")
    text = golden(kat["license_text_file"])
    assert len(text) == 843
    for f in (oracle_mod.crc32c, oracle_mod.crc32c_bitwise, oracle_mod.crc32c_hw):
        assert f(0, text) == kat["license_text_crc"] == 0x7DCDE113
        assert f(0, b"123456789") == kat["check_123456789"]


def test_crc32c_vectors(oracle_mod, golden):
    for v in golden("crc32c_kat.json")["vectors"]:
        data = bytes.fromhex(v["hex"])
        assert oracle_mod.crc32c(v["init"], data) == v["crc"]
        assert oracle_mod.crc32c_hw(v["init"], data) == v["crc"]


def test_crc32c_chaining_and_combine(oracle_mod):
    rnd = random.Random(3)
    for _ in range(50):
        a = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 3000)))
        b = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 3000)))
        whole = oracle_mod.crc32c(0, a + b)
        assert oracle_mod.crc32c(oracle_mod.crc32c(0, a), b) == whole
        assert oracle_mod.crc32c_combine(oracle_mod.crc32c(0, a), oracle_mod.crc32c(0, b),
                                         len(b)) == whole


def test_crc32c_hw_3way_long(oracle_mod):
    rnd = random.Random(5)
    data = bytes(rnd.getrandbits(8) for _ in range(3 * 8192 * 2 + 3 * 256 * 3 + 13))
    assert oracle_mod.crc32c_hw(0, data) == oracle_mod.crc32c(0, data) == \
        oracle_mod.crc32c_bitwise(0, data)


# ------------------------------------------------------------------- LZ4F
def test_lz4f_frames_match_reference_golden(oracle_mod, golden):
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "mg", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    frames = golden("lz4f_frames.json")
    for name, data in mg.inputs():
        rec = frames[name]
        assert sha(data) == rec["input_sha256"], name
        err, fr = oracle_mod.rdk_lz4_compress(data)
        assert err == 0
        assert len(fr) == rec["frame_len"] and sha(fr) == rec["frame_sha256"], name
        if "frame_file" in rec:
            assert fr == golden(rec["frame_file"])
        err, out = oracle_mod.rdk_lz4_decompress(fr)
        assert err == 0 and out == data, name


def test_lz4f_decode_cases_match_reference_golden(oracle_mod, golden):
    for c in golden("lz4f_decode_cases.json"):
        f = bytes.fromhex(c["hex"])
        err, out = oracle_mod.rdk_lz4_decompress(f)
        assert err == c["err"], c["hex"][:80]
        if err == 0:
            assert len(out) == c["out_len"] and sha(out) == c["out_sha256"]


def test_header_bytes_constant(oracle_mod):
    err, fr = oracle_mod.rdk_lz4_compress(b"x" * 100)
    assert fr[:7] == bytes.fromhex("04224d18604082")       # LZ4F magic, FLG 0x60, BD 0x40, HC 0x82 (lz4frame.c:672-700)
    assert fr[-4:] == b"\x00\x00\x00\x00"


def test_legacy_framing_roundtrip(oracle_mod):
    data = W.gen_json(5000)
    err, fr = oracle_mod.rdk_lz4_compress(data, proper_hc=0)
    assert err == 0 and fr[6] != 0x82                      # broken HC (MsgVersion 0)
    buf = bytearray(fr)
    err, out = oracle_mod.rdk_lz4_decompress(bytes(buf), proper_hc=0)
    assert err == 0 and out == data


def test_acceleration_levels(oracle_mod):
    data = W.gen_json(70000)
    for level in (-1, -5, 0, 1, 2):
        err, fr = oracle_mod.rdk_lz4_compress(data, comp_level=level)
        assert err == 0
        assert oracle_mod.rdk_lz4_decompress(fr) == (0, data)


# ---------------------------------------- live differential vs the reference
needs_ref = pytest.mark.skipif("not __import__('oracle').ref_available()")


@needs_ref
def test_block_compress_matches_reference(oracle_mod):
    rnd = random.Random(11)
    srcs = [W.gen_json(65536, s) for s in range(3)] + [bytes(65536), bytes(rnd.getrandbits(8) for _ in range(5000))]
    for _ in range(40):
        src = rnd.choice(srcs)
        n = rnd.randrange(0, len(src) + 1)
        o = rnd.randrange(0, len(src) - n + 1)
        blk = src[o:o + n]
        for accel in (1, 2, 9):
            assert oracle_mod.lz4_compress_block(blk, accel) == \
                oracle_mod.ref_lz4_compress_block(blk, accel)


@needs_ref
def test_block_decompress_fuzz_matches_reference(oracle_mod):
    rnd = random.Random(12)
    for it in range(400):
        src = W.gen_json(rnd.randrange(20, 3000), it)
        blk = oracle_mod.lz4_compress_block(src)
        if blk is None:
            continue
        b = bytearray(blk)
        for _ in range(rnd.randrange(1, 4)):
            b[rnd.randrange(len(b))] = rnd.getrandbits(8)
        if rnd.random() < 0.3:
            b = b[:rnd.randrange(1, len(b) + 1)]
        cap = rnd.choice([len(src), len(src) + 30, 65536, 100])
        r1, o1 = oracle_mod.lz4_decompress_block(bytes(b), cap)
        r2, o2 = oracle_mod.ref_lz4_decompress_safe(bytes(b), cap)
        assert (r1 >= 0) == (r2 >= 0), (it, r1, r2)
        if r1 >= 0:
            assert r1 == r2 and o1 == o2, it


@needs_ref
def test_frame_segmentation_independent(oracle_mod):
    data = W.gen_json(200000)
    rnd = random.Random(4)
    cuts = sorted(rnd.sample(range(1, len(data)), 7))
    segs = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
    assert oracle_mod.ref_rdk_lz4_compress(segs)[1] == oracle_mod.rdk_lz4_compress(data)[1]


def _apply_edit(frame, edit):
    f = bytearray(frame)
    for pos, val in edit.get("flip", []):
        f[pos] = val
    if "truncate" in edit:
        f = f[:edit["truncate"]]
    if "append" in edit:
        f += bytes.fromhex(edit["append"])
    return bytes(f)


def test_lz4f_variant_frames_match_reference_golden(oracle_mod, golden):
    """Frames from other producers (linked blocks, 256 KB blocks, checksums,
    content size, flushed small blocks) and edits of them."""
    var = golden("lz4f_variants.json")
    frames = {k: golden(v["file"]) for k, v in var["frames"].items()}
    for k, v in var["frames"].items():
        err, out = oracle_mod.rdk_lz4_decompress(frames[k])
        assert err == 0 and sha(out) == v["payload_sha256"], k
    for c in var["cases"]:
        err, out = oracle_mod.rdk_lz4_decompress(_apply_edit(frames[c["base"]], c))
        assert err == c["err"], c
        if err == 0:
            assert len(out) == c["out_len"] and sha(out) == c["out_sha256"], c
