"""Two ranks, each bound to the engine (rdk_hip_init) and running CRC32C + LZ4F on its own
toppar shard with no data-path collective; the merged results equal the oracle's for all
partitions (= a 1-rank run).  On a 1-GPU box both ranks use device 0.  Also: bench.py
--gpus 2 started by hand launches two ranks itself and reports n_gpus 2."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N_PARTS = 23


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _part_records(p):
    from librdkafka_amd import workload as W
    return W.gen_json(70000 + 4099 * p, 500 + p)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    import librdkafka_amd as L
    from librdkafka_amd import workload as W
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = rank % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    L.init(dev)
    mine = bench.shard_partitions(N_PARTS, rank, world)
    recs = [_part_records(p) for p in mine]
    # this rank's shard: uncompressed v2 batches, then CRC finalize and LZ4F of the records
    batches = [W.v2_header(p, 61 + len(r)) + r for p, r in zip(mine, recs)]
    offs, pos = [], 0
    for b in batches:
        offs.append(pos)
        pos += (len(b) + 255) // 256 * 256
    hbuf = bytearray(pos + 256)
    for o, b in zip(offs, batches):
        hbuf[o:o + len(b)] = b
    d = torch.frombuffer(hbuf, dtype=torch.uint8).cuda()
    boffs = torch.tensor(offs, dtype=torch.int64, device="cuda")
    bcaps = torch.tensor([len(b) for b in batches], dtype=torch.int32, device="cuda")
    crcs = torch.zeros(len(mine), dtype=torch.int32, device="cuda")
    L.msgset_v2_crc(d, boffs, bcaps, crcs, L.V2_CRC_FINALIZE)
    roffs = boffs + 61
    rlens = bcaps - 61
    bound = (L.lz4f_compress_bound(max(len(r) for r in recs)) + 255) // 256 * 256
    out = torch.empty(len(mine) * bound + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(len(mine), dtype=torch.int64, device="cuda") * bound
    olens = torch.zeros(len(mine), dtype=torch.int32, device="cuda")
    L.lz4f_compress_batch(d, roffs, rlens, out, ooffs, olens)
    torch.cuda.synchronize()
    bench.barrier(world)                                   # gloo, CPU tensors only
    t = bench.max_over_ranks(float(rank + 1), world)
    host, ol = bytes(out.cpu().numpy()), olens.cpu().numpy()
    crc = crcs.cpu().numpy().view(np.uint32)
    res = {p: (int(crc[i]), host[i * bound:i * bound + ol[i]]) for i, p in enumerate(mine)}
    dist.destroy_process_group()
    q.put((rank, res, t))


@pytest.mark.timeout(600)
def test_two_ranks_run_the_engine_on_their_shards(oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=500) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert set(out[0][1]).isdisjoint(out[1][1])
    merged = {**out[0][1], **out[1][1]}
    assert sorted(merged) == list(range(N_PARTS))
    assert all(o[2] == 2.0 for o in out)                   # MAX over ranks
    for p in range(N_PARTS):
        rec = _part_records(p)
        crc, frame = merged[p]
        from librdkafka_amd import workload as W
        hdr = W.v2_header(p, 61 + len(rec))
        assert crc == oracle_mod.crc32c(0, hdr[21:] + rec), p
        assert frame == oracle_mod.rdk_lz4_compress(rec)[1], p


@pytest.mark.timeout(900)
def test_bench_gpus_2_launches_two_ranks():
    """bench.py --gpus 2 started by hand: the parent launches two ranks and rank 0 reports
    ranks 2 (weak scaling: 16 batches per rank).  On a box with one GPU the ranks share it:
    that takes --rehearsal, and the line then counts one GPU and says shared_device, so it
    cannot pass for a scaling point.  A --gpus that contradicts WORLD_SIZE is refused."""
    import torch
    ndev = torch.cuda.device_count()
    common = ["--steps", "3", "--warmup", "1", "--partitions", "16", "--no-legs", "--no-cpu-baseline"]
    if ndev < 2:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + common,
                           capture_output=True, text=True, timeout=800, cwd=ROOT)
        assert r.returncode != 0 and "--rehearsal" in r.stderr     # refused without the flag
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearsal"] + common,
                       capture_output=True, text=True, timeout=800, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks"] == 2 and line["n_gpus"] == min(2, ndev) and line["value"] > 0
    assert line.get("shared_device", False) == (ndev < 2) and line["scaling"] == "weak"
    assert line["config"]["batches_per_gpu"] == 16
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + common,
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
