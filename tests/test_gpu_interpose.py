"""The preload binding, exercised end to end: a program linked only
against a host library that defines crc32c / rd_slice_crc32c / rd_kafka_lz4_compress /
rd_kafka_lz4_decompress itself (default visibility, called through the PLT, like the
reference's CMake build) is run twice -- plainly, and with librdkafka_hip.so preloaded.
Preloaded, the host library's own call sites must reach the engine: results equal the
oracle's and the engine's call counters move while the host's own definitions stay idle.
(tests/interpose/ holds the fixture; the reference itself needs cmake and a generated
config.h to build, so it is not built here.)"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "interpose", "build")


def _run(tmp_path, preload):
    env = dict(os.environ, RDK_HIP_REPORT="1")
    if preload:
        import librdkafka_amd as L
        env["LD_PRELOAD"] = L.LIB_PATH
    data = tmp_path / ("data_%d.bin" % preload)
    r = subprocess.run([os.path.join(FIX, "driver"), "300000", str(data)], capture_output=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = dict(line.split(" ", 1) for line in r.stdout.decode().splitlines())
    return out, r.stderr, data.read_bytes()


def test_preload_binds_the_host_librarys_call_sites(tmp_path, oracle_mod):
    if not os.path.exists(os.path.join(FIX, "driver")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "interpose")], check=True)
    plain, _, data = _run(tmp_path, False)
    assert plain["compress_err"] == "-12345"                       # the host library's own stub
    assert plain["host_calls"] == "crc32c=2 slice=1 lz4c=1 lz4d=0"
    assert int(plain["crc"], 16) == oracle_mod.crc32c(0, data)     # its own bitwise crc32c

    pre, stderr, data2 = _run(tmp_path, True)
    assert data2 == data
    assert int(pre["crc"], 16) == oracle_mod.crc32c(0, data)
    assert pre["compress_err"] == "0" and pre["decompress_err"] == "0" and pre["roundtrip"] == "1"
    assert pre["host_calls"] == "crc32c=0 slice=0 lz4c=0 lz4d=0"   # never reached
    at = stderr.rfind(b"librdkafka_hip: calls")                    # printed at exit, after the frame
    report = stderr[at:] if at >= 0 else b""
    assert b"rd_slice_crc32c=1" in report and b"rd_kafka_lz4_compress=1" in report \
        and b"rd_kafka_lz4_decompress=1" in report, stderr[-500:]
    # the frame the host library's writer call site got back is the reference's frame
    frame = stderr[:int(pre["compress_len"])]
    assert frame == oracle_mod.rdk_lz4_compress(data)[1]
