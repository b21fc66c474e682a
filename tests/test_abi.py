"""C-ABI boundary checks that need no GPU: the library builds for gfx950,
exports exactly what include/librdkafka_hip.h declares, and links nothing
from the oracle."""
import os
import re
import subprocess

import librdkafka_amd as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "librdkafka_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", txt)) - {"sizeof"}


def dyn_symbols():
    if not os.path.exists(L.LIB_PATH):
        L.build()
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_header_declares_reference_dropins():
    fns = header_functions()
    for f in ("crc32c", "crc32c_global_init", "rd_slice_crc32c", "rd_kafka_lz4_compress",
              "rd_kafka_lz4_decompress"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    fns = header_functions()
    syms = dyn_symbols()
    missing = sorted(fns - syms)
    assert not missing, f"declared but not exported: {missing}"
    assert set(L.EXPORTED_SYMBOLS) <= syms
    # nothing else leaks (hidden visibility)
    extra = sorted(s for s in syms - fns if not s.startswith("_"))
    assert not extra, f"unexpected exports: {extra}"


def test_library_is_gfx950_code_object():
    """The fat binary carries a gfx950 code object (and no other target)."""
    blob = open(L.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_product_does_not_link_oracle():
    out = subprocess.run(["nm", "-D", L.LIB_PATH], capture_output=True, text=True).stdout
    assert " or_" not in out and "ref_" not in out
    ldd = subprocess.run(["ldd", L.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "libreflz4" not in ldd


def test_ctypes_load_without_gpu():
    lib = L.lib()
    assert lib.rdk_hip_version().decode().startswith("librdkafka_hip")


def test_json_generator_native_matches_python():
    from librdkafka_amd import workload as W
    for n in (0, 1, 77, 5000, 100003):
        assert L.gen_json(n, 42) == W.gen_json(n, 42)
        assert L.gen_json(n, 9) == W.gen_json(n, 9)


def test_v2_header_layout():
    from librdkafka_amd import workload as W
    h = W.v2_header(3, 16384)
    assert len(h) == 61 and h[16] == 2                     # Magic at 16
    assert int.from_bytes(h[8:12], "big") == 16384 - 12    # Length
    assert h[17:21] == b"\0\0\0\0"                          # CRC slot


def test_dropin_lz4_reports_reference_error_codes_without_a_device():
    """No device here: the LZ4 drop-ins must answer with the reference's own error codes
    (the writer then sends uncompressed, rdkafka_msgset_writer.c:1175; the reader raises a
    consumer error, rdkafka_msgset_reader.c:517), consume the slice, and never abort or
    hand the call to another definition of the symbol."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("a device is present")
    s = L.RdSlice([b"abc" * 100, b"def" * 50])
    err, out = L.rd_kafka_lz4_compress(1, 0, s)
    assert err == L.RESP_ERR__CRIT_SYS_RESOURCE and out == b"" and s.remains() == 0
    s = L.RdSlice([b"abc" * 100])
    err, out = L.rd_kafka_lz4_compress(1, 12, s)          # LZ4HC optimal: the same contract
    assert err == L.RESP_ERR__CRIT_SYS_RESOURCE and out == b"" and s.remains() == 0
    frame = bytes([0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82, 0, 0, 0, 0])
    assert L.rd_kafka_lz4_decompress(1, 0, frame) == (L.RESP_ERR__CRIT_SYS_RESOURCE, b"")


def test_product_never_forwards_to_another_definition():
    """The drop-in symbols never look up the next definition of themselves."""
    src = os.path.join(ROOT, "librdkafka_amd", "csrc")
    for f in os.listdir(src):
        txt = open(os.path.join(src, f)).read()
        assert "RTLD_NEXT" not in txt and "dlsym" not in txt, f
    out = subprocess.run(["nm", "-D", "--undefined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "dlsym" not in out
