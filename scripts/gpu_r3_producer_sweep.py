"""Producer front-end: threads x slot size x ring depth sweep (PCIe-inclusive GB/s), 2 GiB per step."""
import argparse
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import librdkafka_amd as L
import bench
L.init(0)
n = 2048
for ns, th, slot in ((8, 1, 128), (4, 1, 64), (8, 2, 128), (4, 2, 64), (2, 4, 64), (3, 4, 64), (4, 4, 32),
                     (2, 4, 128), (2, 8, 32), (3, 8, 32), (2, 8, 64), (4, 8, 16)):
    os.environ["RDK_BENCH_PRODUCER_NSLOTS"] = str(ns)
    r = bench.bench_producer(argparse.Namespace(steps=2, warmup=1, partitions=n), 0, 1, n=n, threads=th,
                             slot_mib=slot)
    print(f"queues={os.environ.get('GPU_MAX_HW_QUEUES', 'default')} slots={ns} threads={th} slot={slot}MiB: "
          f"{r['bytes'] / (r['ms'] / 1e3) / 1e9:.1f} GB/s", flush=True)
