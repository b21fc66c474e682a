"""GPU parity for MsgVersion 2 record serialisation (csrc/records.hip) against
the oracle restatement of rdkafka_msgset_writer.c, byte for byte."""
import numpy as np
import pytest

import librdkafka_amd as E
from librdkafka_amd import workload as W

pytestmark = pytest.mark.gpu


def _dev(m):
    import torch
    d = {}
    for k, v in m.items():
        a = v.view(np.int64) if v.dtype == np.uint64 else (v.view(np.int32) if v.dtype == np.uint32 else v)
        d[k] = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return d


def _batches(spec):
    b = np.zeros(len(spec), dtype=E.V2_BATCH_DTYPE)
    for i, (first, cnt) in enumerate(spec):
        b[i] = (first, cnt, 1000 + i, 7 * i - 1, i % 3, 0)
    return b


@pytest.mark.parametrize("headers", [True, False])
def test_v2_build_matches_oracle(engine, oracle_mod, headers):
    m = W.gen_messages(5000, seed=3, headers=headers)
    if not headers:
        m.pop("hdr_off"); m.pop("hdr_len"); m.pop("hdr_cnt")
    spec = [(0, 1), (1, 2), (3, 300), (303, 1), (304, 64), (368, 65), (433, 1000),
            (1433, 257), (1690, 3310)]
    b = _batches(spec)
    out, offs, sizes, crcs = E.msgset_v2_build(_dev(m), b, crc=True)
    host = bytes(out.cpu().numpy())
    offs, sizes, crcs = offs.cpu().numpy(), sizes.cpu().numpy(), crcs.cpu().numpy().view(np.uint32)
    for i, (first, cnt) in enumerate(spec):
        exp = oracle_mod.msgset_v2_write(m, first, cnt, 1000 + i, i % 3, 7 * i - 1, 0)
        got = host[offs[i]:offs[i] + sizes[i]]
        assert len(got) == len(exp), (i, len(got), len(exp))
        assert got == exp, (i, next(j for j in range(len(exp)) if got[j] != exp[j]))
        assert crcs[i] == int.from_bytes(exp[17:21], "big")


def test_v2_build_then_verify(engine):
    """The built batches pass the engine's own CRC verify (reader side)."""
    import torch
    m = W.gen_messages(20000, seed=9)
    spec = [(i * 1000, 1000) for i in range(20)]
    out, offs, sizes, _ = E.msgset_v2_build(_dev(m), _batches(spec), crc=True)
    st = torch.zeros(len(spec), dtype=torch.int32, device="cuda")
    E.msgset_v2_crc(out, offs, sizes, st, E.V2_CRC_VERIFY)
    assert int(st.abs().sum()) == 0
