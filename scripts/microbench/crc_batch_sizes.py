# CRC32C headline kernel throughput vs batch size at a fixed 16 GiB (run on the GPU box).
import sys, torch
sys.path.insert(0, __import__("os").path.abspath(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "..")))
import librdkafka_amd as E
tot = 16 << 30
for size in (16384, 65536, 262144):
    n = tot // size
    buf = torch.empty(n * size + 64, dtype=torch.uint8, device="cuda")
    E.gen_v2_batches(buf, n, size, 7)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * size
    caps = torch.full((n,), size, dtype=torch.int32, device="cuda")
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    for _ in range(2): E.msgset_v2_crc(buf, offs, caps, out, E.V2_CRC_COMPUTE)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record()
    for _ in range(5): E.msgset_v2_crc(buf, offs, caps, out, E.V2_CRC_COMPUTE)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    print(size, n, "%.3f ms  %.0f GB/s" % (ms, n * (size - 21) / ms / 1e6), flush=True)
    del buf
