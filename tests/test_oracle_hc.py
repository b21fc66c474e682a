"""LZ4HC (compression.level 3..12) restatement (oracle/lz4hc_oracle.c) pinned
against frames made by the reference's own lz4hc.c build (tests/golden/
lz4hc_frames.json) and, when oracle/_ref is built, live block-level
differential tests against LZ4_compress_HC_extStateHC_fastReset
(lz4hc.c:896) -- including the level-9 pattern analysis (lz4hc.c:336-405) and
the optimal parser with its chain swap (levels 10..12, lz4hc.c:1278, :312-334)."""
import hashlib
import importlib.util
import os
import random

import pytest

from librdkafka_amd import workload as W


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _mg():
    spec = importlib.util.spec_from_file_location(
        "mg", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def test_lz4hc_frames_match_reference_golden(oracle_mod, golden):
    mg = _mg()
    recs = golden("lz4hc_frames.json")
    assert len(recs) == len(mg.HC_INPUTS) * 10
    for key, rec in recs.items():
        data = mg.input_by_name(rec["input"])
        err, fr = oracle_mod.rdk_lz4_compress(data, comp_level=rec["level"])
        assert err == 0
        assert len(fr) == rec["frame_len"] and sha(fr) == rec["frame_sha256"], key
        err, out = oracle_mod.rdk_lz4_decompress(fr)
        assert err == 0 and out == data, key


def _hc_cases():
    rnd = random.Random(11)
    js = W.gen_json(4 * 65536, 5)
    cases = [js[i * 65536:(i + 1) * 65536] for i in range(4)]
    cases += [bytes(65536), b"ab" * 30000, b"abcd" * 16000, b"abc" * 20000,
              (b"0000" + b"1" * 7 + b"\0" * 9) * 3000, b"x" * 13, b"hello world"]
    for _ in range(12):
        n = rnd.randint(1, 65536)
        alpha = rnd.choice([1, 2, 3, 4, 16, 256])
        cases.append(bytes(rnd.randrange(alpha) for _ in range(n)))
    return cases


@pytest.mark.parametrize("level", range(3, 13))
def test_lz4hc_block_differential_vs_reference(oracle_mod, level):
    if not oracle_mod.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference)")
    for i, d in enumerate(_hc_cases()):
        assert oracle_mod.lz4hc_compress_block(d, level) == \
            oracle_mod.ref_lz4hc_compress_block(d, level), (level, i, len(d))


def test_lz4hc_levels_above_12_clamp(oracle_mod):
    """MIN(LZ4HC_CLEVEL_MAX, cLevel), lz4hc.c:798"""
    d = W.gen_json(20000, 3)
    assert oracle_mod.lz4hc_compress_block(d, 13) == oracle_mod.lz4hc_compress_block(d, 12)
