"""The library's host files under ThreadSanitizer, without a GPU.

shim.cpp, combine.cpp, engine.cpp and lz4_host.cpp are built with -fsanitize=thread against
tests/tsan/hip_stub.cpp (a stand-in HIP runtime whose CRC entry points give right answers and
whose LZ4F entry points write stored-block frames).  tests/tsan/driver.cpp calls crc32c,
rd_slice_crc32c, rd_slice_crc32, rd_kafka_lz4_compress and rd_kafka_lz4_decompress from
broker-like threads at once (rdkafka_broker.c:5082) and checks every result.  The runs below
cover the combined path, forced device failures (retry, one-request-at-a-time fallback), no
pinned staging (CRC finished on the host, LZ4 symbols return __CRIT_SYS_RESOURCE) and the
uncombined path.
"""
import os
import re
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tsan")
BIN = os.path.join(HERE, "_build", "driver_tsan")


@pytest.fixture(scope="module")
def driver():
    subprocess.run(["make", "-s", "-C", HERE], check=True, timeout=300)
    return BIN


@pytest.fixture(scope="module")
def driver_asan():
    subprocess.run(["make", "-s", "-C", HERE, "_build/driver_asan"], check=True, timeout=300)
    return os.path.join(HERE, "_build", "driver_asan")


def run(driver, threads, iters, **env):
    p = subprocess.run([driver, str(threads), str(iters)], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=600)
    out = p.stdout + p.stderr
    assert "ThreadSanitizer" not in out and "AddressSanitizer" not in out and "runtime error" not in out, \
        out[-4000:]
    assert p.returncode == 0, out[-4000:]
    m = re.search(r"bad=(\d+) combined_batches=(\d+) requests=(\d+) largest=(\d+) fallbacks=(\d+) "
                  r"host_crcs=(\d+) ctx=(\d+)/(\d+)", out)
    assert m, out[-2000:]
    return [int(x) for x in m.groups()]


def test_combined_calls_are_race_free_and_right(driver):
    bad, batches, reqs, largest, fallbacks, host_crcs, made, gone = run(driver, 8, 60)
    assert bad == 0 and fallbacks == 0 and host_crcs == 0
    assert batches > 0 and reqs >= 2 * batches and 2 <= largest <= 8
    assert made == gone == 16  # two generations of 8 threads: every context ended with its thread


def test_forced_device_failures(driver):
    bad, batches, reqs, largest, fallbacks, host_crcs, made, gone = run(driver, 8, 40, STUB_FAIL_EVERY="5")
    assert bad == 0 and fallbacks > 0 and made == gone


def test_no_pinned_staging(driver):
    bad, batches, reqs, largest, fallbacks, host_crcs, made, gone = run(driver, 6, 30, STUB_FAIL_ALLOC="1")
    assert bad == 0 and host_crcs > 0 and made == gone


def test_uncombined(driver):
    bad, batches, reqs, largest, fallbacks, host_crcs, made, gone = run(driver, 6, 30, RDK_HIP_COMBINE="0")
    assert bad == 0 and batches == 0 and made == gone


def test_address_and_undefined_behaviour_sanitizers(driver_asan):
    """the same driver under ASan + UBSan with the leak check on: every malloc()ed result is
    freed by its owner, every context by its thread, on the good path and on the error paths"""
    for env in ({}, {"STUB_FAIL_EVERY": "5"}, {"STUB_FAIL_ALLOC": "1"}):
        bad, *_rest, made, gone = run(driver_asan, 6, 30, **env)
        assert bad == 0 and made == gone
