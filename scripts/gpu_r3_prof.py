"""Phase timing of the unit compressor (a -DRDK_UNITS_PROF build given by RDK_HIP_LIB):
runs the throughput compressor over 256 x 1 MiB JSON batches and prints the share of cycles
per phase and role."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import argparse
import torch
import librdkafka_amd as L
import bench
L.init(0)
src, offs, lens = bench.json_batches(256)
bound = (L.lz4f_compress_bound(bench.JSON_BATCH) + 255) // 256 * 256
dst = torch.empty(256 * bound + 256, dtype=torch.uint8, device="cuda")
ooffs = torch.arange(256, dtype=torch.int64, device="cuda") * bound
olens = torch.zeros(256, dtype=torch.int32, device="cuda")
for _ in range(3):
    L.lz4f_compress_fast_batch(src, offs, lens, dst, ooffs, olens)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(5):
    L.lz4f_compress_fast_batch(src, offs, lens, dst, ooffs, olens)
ev1.record()
torch.cuda.synchronize()
print("ms per 256 MiB:", ev0.elapsed_time(ev1) / 5, "ratio", 256 * bench.JSON_BATCH / int(olens.sum()))
if hasattr(L.lib(), "rdk_hip_units_prof_dump"):
    L.lib().rdk_hip_units_prof_dump()
