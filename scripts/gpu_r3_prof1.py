"""Phase timing of the unit compressor on ONE block / a few blocks (prof build via RDK_HIP_LIB)."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import librdkafka_amd as L
L.init(0)
for nframes, size in ((1, 65536), (256, 65536), (256, 1 << 20)):
    host = L.gen_json(size, 42)
    src = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda().repeat(nframes)
    offs = torch.arange(nframes, dtype=torch.int64, device="cuda") * size
    lens = torch.full((nframes,), size, dtype=torch.int32, device="cuda")
    bound = (L.lz4f_compress_bound(size) + 255) // 256 * 256
    dst = torch.empty(nframes * bound + 256, dtype=torch.uint8, device="cuda")
    ooffs = torch.arange(nframes, dtype=torch.int64, device="cuda") * bound
    olens = torch.zeros(nframes, dtype=torch.int32, device="cuda")
    L.lz4f_compress_fast_batch(src, offs, lens, dst, ooffs, olens)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        L.lz4f_compress_fast_batch(src, offs, lens, dst, ooffs, olens)
    ev1.record()
    torch.cuda.synchronize()
    print(f"{nframes} x {size}: {ev0.elapsed_time(ev1) / 10 * 1000:.1f} us per launch", flush=True)
    if hasattr(L.lib(), "rdk_hip_units_prof_dump"):
        L.lib().rdk_hip_units_prof_dump()
