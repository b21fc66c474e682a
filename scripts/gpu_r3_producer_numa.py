"""Producer front-end under CPU affinity: one run per NUMA node of the host."""
import argparse
import glob
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
    nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(d + "/cpulist").read())
print("nodes:", {k: (v[0], v[-1], len(v)) for k, v in nodes.items()}, flush=True)
for f in glob.glob("/sys/class/drm/card*/device/numa_node"):
    print(f, open(f).read().strip(), flush=True)
allowed = os.sched_getaffinity(0)
print("allowed cpus:", len(allowed), flush=True)
import librdkafka_amd as L
import bench
L.init(0)
n = 2048
for node, cpus in nodes.items():
    use = set(cpus) & allowed
    if not use:
        continue
    os.sched_setaffinity(0, use)   # the main thread; new threads inherit it
    for th, slot in ((1, 128), (2, 64), (4, 32)):
        r = bench.bench_producer(argparse.Namespace(steps=2, warmup=1, partitions=n), 0, 1, n=n, threads=th,
                                 slot_mib=slot)
        print(f"node {node}: threads={th} slot={slot}MiB: {r['bytes'] / (r['ms'] / 1e3) / 1e9:.1f} GB/s", flush=True)
