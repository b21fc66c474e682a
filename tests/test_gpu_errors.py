"""Failure handling of the drop-in symbols and stream ordering of the engine's scratch,
forced from the host (an allocation cap, two caller streams): every kernel still exits
normally."""
import os
import subprocess
import sys
import textwrap

import pytest

from librdkafka_amd import workload as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dropin_lz4_allocation_failure_is_an_error_code_not_an_abort():
    """RDK_HIP_MAX_SCRATCH_BYTES caps every device scratch region: a 1 MiB compress then
    fails to get its staging and must return __CRIT_SYS_RESOURCE (-194); the process lives
    on and smaller calls keep working.  Own process: the cap is read from the environment."""
    code = textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        import librdkafka_amd as L
        from librdkafka_amd import workload as W
        L.init(0)
        big = W.gen_json(1 << 20, 1)
        s = L.RdSlice([big])
        err, out = L.rd_kafka_lz4_compress(1, 0, s)
        assert err == L.RESP_ERR__CRIT_SYS_RESOURCE and out == b"" and s.remains() == 0, err
        err, fr = L.rd_kafka_lz4_compress(1, 0, W.gen_json(3000, 2))   # fits under the cap
        assert err == 0 and len(fr) > 11, err
        assert L.rd_kafka_lz4_decompress(1, 0, fr) == (0, W.gen_json(3000, 2))
        fr_big = bytes([0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82]) + \\
            b"".join((0x80010000).to_bytes(4, "little") + bytes(65536) for _ in range(40)) + bytes(4)
        err, out = L.rd_kafka_lz4_decompress(1, 0, fr_big)   # 2.5 MiB of output staging
        assert err == L.RESP_ERR__CRIT_SYS_RESOURCE and out == b"", err
        print("survived")
    """ % ROOT)
    env = dict(os.environ, RDK_HIP_MAX_SCRATCH_BYTES=str(1 << 20))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0 and "survived" in r.stdout, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "RDK_HIP_MAX_SCRATCH_BYTES" in r.stderr          # the first failure is reported


def _hc_compress(engine, inputs, level, stream):
    import numpy as np
    import torch
    with torch.cuda.stream(stream):
        offs, pos = [], 0
        for b in inputs:
            offs.append(pos)
            pos += (len(b) + 63) // 64 * 64
        hbuf = bytearray(pos + 256)
        for o, b in zip(offs, inputs):
            hbuf[o:o + len(b)] = b
        d_in = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
        in_offs = torch.tensor(offs, dtype=torch.int64, device="cuda")
        in_lens = torch.tensor([len(b) for b in inputs], dtype=torch.int32, device="cuda")
        bounds = [(engine.lz4f_compress_bound(len(b)) + 63) // 64 * 64 for b in inputs]
        ooffs = np.concatenate([[0], np.cumsum(bounds)[:-1]])
        d_out = torch.empty(int(sum(bounds)) + 256, dtype=torch.uint8, device="cuda")
        out_offs = torch.tensor(ooffs, dtype=torch.int64, device="cuda")
        out_lens = torch.zeros(len(inputs), dtype=torch.int32, device="cuda")
        engine.lz4f_compress_batch(d_in, in_offs, in_lens, d_out, out_offs, out_lens, level=level,
                                   stream=stream)
    return d_in, d_out, ooffs, out_lens


def test_lz4hc_two_streams_share_one_thread(engine, oracle_mod):
    """One host thread issues LZ4HC compressions on two streams back to back: the second
    must not touch the hash tables or the work counter while the first is running."""
    import torch
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = [W.gen_json(1 << 20, 10 + i) for i in range(6)]
    b = [W.gen_json(300000 + 1000 * i, 50 + i) for i in range(5)]
    ra = _hc_compress(engine, a, 9, s1)
    rb = _hc_compress(engine, b, 4, s2)
    torch.cuda.synchronize()
    for inputs, level, (_, d_out, ooffs, out_lens) in ((a, 9, ra), (b, 4, rb)):
        host = bytes(d_out.cpu().numpy())
        lens = out_lens.cpu().numpy()
        for i, data in enumerate(inputs):
            want = oracle_mod.rdk_lz4_compress(data, comp_level=level)[1]
            assert host[ooffs[i]:ooffs[i] + lens[i]] == want, (level, i)
