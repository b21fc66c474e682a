"""Regenerate tests/golden/ fixtures from the REFERENCE build (oracle/_ref).

Run in the build container (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py

Outputs (all data, no reference source):
  crc32c_kat.json          -- the reference's KAT (crc32c.c:388-438: license
                              text -> 0x7dcde113), the standard check value,
                              and seeded vectors (bit-serial definition).
  crc32c_kat_license.txt   -- the 843-byte KAT input of unittest_crc32c.
  lz4f_frames.json         -- for seeded inputs: length + sha256 of the frame
                              the reference's rd_kafka_lz4_compress path makes
                              (vendored lz4 1.9.2 LZ4F), and of its payload.
  frame_*.lz4              -- the frames themselves for inputs <= 64 KiB.
  lz4hc_frames.json        -- the same for compression.level 3..12 (LZ4HC hash
                              chain, lz4frame.c:782 -> lz4hc.c:532-746, and the
                              optimal parser of levels 10..12, lz4hc.c:1278).
  lz4f_decode_cases.json   -- deterministic malformed / edge-case frames and
                              the reference decoder's verdict (err, len,
                              sha256), exercising rdkafka_lz4.c:167-317.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402
from librdkafka_amd import workload as W  # noqa: E402

REF_CRC = "/root/reference/src/crc32c.c"


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def kat_text() -> bytes:
    src = open(REF_CRC).read()
    body = src[src.index("int unittest_crc32c"):src.index("const uint32_t expected_crc")]
    parts = re.findall(r'^"(.*)"', body, re.M)
    return "".join(p.encode().decode("unicode_escape") for p in parts).encode()


def inputs():
    """(name, bytes) pairs, all re-derivable from the generators in workload.py."""
    rnd = random.Random(1234)
    out = []
    for n in (16384, 65536, 65537, 262144, 1000000, 1 << 20):
        out.append((f"json_s42_{n}", W.gen_json(n, 42)))
    for n in (0, 1, 12, 13, 14, 100, 4095, 4096, 65535):
        out.append((f"json_s7_{n}", W.gen_json(n, 7)))
    out.append(("zeros_200000", bytes(200000)))
    out.append(("pattern_70000", (b"librdkafka_performance testing!" * 3000)[:70000]))
    rb = random.Random(99)
    out.append(("random_70000", bytes(rb.getrandbits(8) for _ in range(70000))))
    out.append(("random_20", bytes(rb.getrandbits(8) for _ in range(20))))
    # mostly-random with sparse repeats: exercises raw-vs-compressed decisions
    mix = bytearray(rb.getrandbits(8) for _ in range(65536))
    for i in range(0, 65536 - 64, 997):
        mix[i:i + 32] = mix[0:32]
    out.append(("mixed_65536", bytes(mix)))
    del rnd
    return out


def input_by_name(name: str) -> bytes:
    for n, b in inputs():
        if n == name:
            return b
    raise KeyError(name)


def mutate_cases(frame: bytes, rnd: random.Random, count: int):
    cases = []
    for i in range(count):
        f = bytearray(frame)
        kind = i % 6
        if kind == 0 and len(f) > 12:      # flip a byte in the block stream
            p = rnd.randrange(11, len(f) - 4)
            f[p] ^= 1 << rnd.randrange(8)
        elif kind == 1:                    # truncate
            f = f[:rnd.randrange(0, len(f))]
        elif kind == 2:                    # trailing garbage
            f += bytes([rnd.getrandbits(8) for _ in range(rnd.randrange(1, 9))])
        elif kind == 3 and len(f) > 12:    # random byte anywhere
            f[rnd.randrange(0, len(f))] = rnd.getrandbits(8)
        elif kind == 4 and len(f) > 15:    # corrupt a block size word
            f[7 + rnd.randrange(0, 4)] = rnd.getrandbits(8)
        else:                              # several flips
            for _ in range(4):
                p = rnd.randrange(0, len(f)) if f else 0
                if f:
                    f[p] ^= 0xFF
        cases.append(bytes(f))
    return cases


HC_INPUTS = ("json_s42_65536", "json_s42_65537", "json_s42_262144", "json_s7_13",
             "json_s7_4096", "zeros_200000", "pattern_70000", "random_70000", "mixed_65536")


def hc_frames() -> None:
    """LZ4HC (levels 3..12) frames of the reference's rd_kafka_lz4_compress path."""
    out = {}
    for name in HC_INPUTS:
        data = input_by_name(name)
        for level in range(3, 13):
            err, fr = O.ref_rdk_lz4_compress(data, comp_level=level)
            assert err == 0
            e2, payload, _ = O.ref_rdk_lz4_decompress(fr, max_msg_size=1 << 30)
            assert e2 == 0 and payload == data
            out[f"{name}@{level}"] = {"input": name, "level": level, "input_len": len(data),
                                      "frame_len": len(fr), "frame_sha256": sha(fr)}
    json.dump(out, open(os.path.join(HERE, "lz4hc_frames.json"), "w"), indent=1)


def main() -> None:
    O.build(ref=True)
    assert O.ref_available(), "oracle/_ref/libreflz4.so not built"
    # ---- CRC32C
    text = kat_text()
    open(os.path.join(HERE, "crc32c_kat_license.txt"), "wb").write(text)
    rnd = random.Random(0x5EED)
    vecs = []
    for n in (0, 1, 3, 4, 5, 15, 16, 17, 31, 63, 64, 65, 100, 1000, 1023, 1024, 1025, 4095, 16363):
        data = bytes(rnd.getrandbits(8) for _ in range(n))
        init = rnd.getrandbits(32) if n % 3 == 0 else 0
        vecs.append({"seed_index": len(vecs), "len": n, "init": init, "hex": data.hex(),
                     "crc": O.crc32c_bitwise(init, data)})
    kat = {"license_text_crc": 0x7DCDE113, "license_text_file": "crc32c_kat_license.txt",
           "check_123456789": 0xE3069283, "vectors": vecs}
    assert O.crc32c_bitwise(0, text) == 0x7DCDE113
    json.dump(kat, open(os.path.join(HERE, "crc32c_kat.json"), "w"), indent=1)

    # ---- LZ4F frames from the reference encoder
    frames = {}
    for name, data in inputs():
        err, fr = O.ref_rdk_lz4_compress(data)
        assert err == 0
        e2, payload, _ = O.ref_rdk_lz4_decompress(fr, max_msg_size=1 << 30)
        assert e2 == 0 and payload == data
        rec = {"input_len": len(data), "input_sha256": sha(data), "frame_len": len(fr),
               "frame_sha256": sha(fr)}
        if len(data) <= 65537:
            fn = f"frame_{name}.lz4"
            open(os.path.join(HERE, fn), "wb").write(fr)
            rec["frame_file"] = fn
        frames[name] = rec
    json.dump(frames, open(os.path.join(HERE, "lz4f_frames.json"), "w"), indent=1)
    hc_frames()

    # ---- decoder verdicts on malformed / edge frames
    rnd = random.Random(77)
    base = {n: O.ref_rdk_lz4_compress(input_by_name(n))[1]
            for n in ("json_s7_4096", "json_s42_16384", "random_20", "json_s7_100")}
    cases = []
    for n, fr in base.items():
        for f in mutate_cases(fr, rnd, 12 if len(fr) > 4096 else 80):
            err, out, _ = O.ref_rdk_lz4_decompress(f, max_msg_size=1 << 30)
            cases.append({"hex": f.hex(), "err": err, "out_len": len(out), "out_sha256": sha(out)})
    # hand-made edge frames
    hdr = bytes.fromhex("04224d18604082")
    extra = [b"", b"\x04\x22", hdr, hdr + b"\x00\x00\x00\x00", hdr + b"\x00\x00\x00\x00\x00",
             hdr + b"\x05\x00\x00\x80hello" + b"\x00" * 4,       # raw block
             hdr + b"\x05\x00\x00\x80hel",                       # truncated raw block
             bytes.fromhex("502a4d1804000000") + b"abcd",        # skippable frame
             bytes.fromhex("502a4d1804000000") + b"abcdXY",      # skippable + trailing
             bytes.fromhex("04224d18644082") + b"\x00\x00\x00\x00"]  # bad HC
    for f in extra:
        err, out, _ = O.ref_rdk_lz4_decompress(f, max_msg_size=1 << 30)
        cases.append({"hex": f.hex(), "err": err, "out_len": len(out), "out_sha256": sha(out)})
    json.dump(cases, open(os.path.join(HERE, "lz4f_decode_cases.json"), "w"))

    # ---- frames with non-default LZ4F preferences (other producers: linked
    # blocks, 256 KB blocks, checksums, content size, flushed small blocks),
    # and mutated copies described as edits of the base frame
    data = W.gen_json(40000, 5)
    variants = {
        "linked": dict(linked=1),
        "bsid5": dict(block_size_id=5),
        "checksums_csize": dict(block_checksum=1, content_checksum=1, content_size=1),
        "flush3000": dict(flush_every=3000),
        "linked_flush_bchk": dict(linked=1, flush_every=2500, block_checksum=1),
        "raw_random_cchk": dict(content_checksum=1),
    }
    rb = random.Random(5)
    var = {"input": "gen_json(40000, 5)", "input_sha256": sha(data), "frames": {}, "cases": []}
    rnd = random.Random(8)
    for name, kw in variants.items():
        src = bytes(rb.getrandbits(8) for _ in range(20000)) if name.startswith("raw") else data
        fr = O.ref_lz4f_compress_prefs(src, **kw)
        fn = f"variant_{name}.lz4"
        open(os.path.join(HERE, fn), "wb").write(fr)
        err, out, _ = O.ref_rdk_lz4_decompress(fr, max_msg_size=1 << 30)
        assert err == 0 and out == src
        var["frames"][name] = {"file": fn, "payload_sha256": sha(out), "payload_len": len(out)}
        for i in range(25):
            edit = {"base": name}
            kind = i % 4
            if kind == 0:
                edit["flip"] = [[rnd.randrange(7, len(fr)), rnd.getrandbits(8)] for _ in range(2)]
            elif kind == 1:
                edit["truncate"] = rnd.randrange(0, len(fr))
            elif kind == 2:
                edit["append"] = bytes(rnd.getrandbits(8) for _ in range(3)).hex()
            else:
                edit["flip"] = [[rnd.randrange(len(fr) - 12, len(fr)), rnd.getrandbits(8)]]
            f = apply_edit(fr, edit)
            err, out, _ = O.ref_rdk_lz4_decompress(f, max_msg_size=1 << 30)
            edit.update({"err": err, "out_len": len(out), "out_sha256": sha(out)})
            var["cases"].append(edit)
    json.dump(var, open(os.path.join(HERE, "lz4f_variants.json"), "w"), indent=0)
    print(f"wrote {len(vecs)} crc vectors, {len(frames)} frames, {len(cases)} decode cases, "
          f"{len(var['cases'])} variant cases")


def apply_edit(frame: bytes, edit: dict) -> bytes:
    f = bytearray(frame)
    for pos, val in edit.get("flip", []):
        f[pos] = val
    if "truncate" in edit:
        f = f[:edit["truncate"]]
    if "append" in edit:
        f += bytes.fromhex(edit["append"])
    return bytes(f)


if __name__ == "__main__":
    if sys.argv[1:] == ["--hc-only"]:
        O.build(ref=True)
        hc_frames()
    else:
        main()
