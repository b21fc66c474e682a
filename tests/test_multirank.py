"""World-size-2 gloo rehearsal of the multi-GPU path on CPU: partitions shard
round-robin across ranks with no data-path collective; the only cross-rank
traffic is the barrier and the max-over-ranks step time bench.py reports."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    import bench
    import oracle
    from librdkafka_amd import workload as W
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_parts = 37
    mine = bench.shard_partitions(n_parts, rank, world)
    # each rank CRCs and compresses only its own partitions' batches
    res = {}
    for p in mine:
        data = W.gen_json(3000 + 17 * p, p)
        res[p] = (oracle.crc32c(0, data), oracle.rdk_lz4_compress(data)[1])
    bench.barrier(world)
    t = bench.max_over_ranks(float(rank + 1), world)
    dist.destroy_process_group()
    q.put((rank, mine, res, t))


@pytest.mark.timeout(300)
def test_two_rank_sharding_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out.sort()
    shards = [set(o[1]) for o in out]
    assert shards[0].isdisjoint(shards[1]) and shards[0] | shards[1] == set(range(37))
    assert all(o[3] == 2.0 for o in out)              # MAX over ranks
    import oracle
    from librdkafka_amd import workload as W
    merged = {**out[0][2], **out[1][2]}
    for p, (crc, frame) in merged.items():             # identical to a 1-rank run
        data = W.gen_json(3000 + 17 * p, p)
        assert crc == oracle.crc32c(0, data)
        assert frame == oracle.rdk_lz4_compress(data)[1]


def test_shard_balance():
    import bench
    for world in (1, 2, 4, 8):
        sizes = [len(bench.shard_partitions(1024, r, world)) for r in range(world)]
        assert sum(sizes) == 1024 and max(sizes) - min(sizes) <= 1
