"""Timing of the exact LZ4 and snappy compressors on 256 x 1 MiB of random bytes and of a
half random / half JSON mix (device-resident, HIP events), printed as GB/s."""
import sys
import numpy as np
import torch
import librdkafka_amd as L

N, B = 256, 1 << 20


def run(name, fn, steps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    print(f"{name}: {ms:.3f} ms  {N * B / ms / 1e6:.1f} GB/s", flush=True)


def main():
    rng = np.random.default_rng(5)
    rnd = rng.integers(0, 256, N * B, dtype=np.uint8)
    js = np.frombuffer(L.gen_json(B * 8, 42), dtype=np.uint8)
    mix = rnd.copy().reshape(N, B)
    for i in range(N):
        mix[i, B // 2:] = js[(i % 8) * B:(i % 8) * B + B // 2]
    for label, host in (("random", rnd), ("half random half json", mix.reshape(-1))):
        src = torch.from_numpy(host).cuda()
        offs = torch.arange(N, dtype=torch.int64, device="cuda") * B
        lens = torch.full((N,), B, dtype=torch.int32, device="cuda")
        bound = (max(L.lz4f_compress_bound(B), L.snappy_max_compressed_length(B)) + 255) // 256 * 256
        dst = torch.empty(N * bound + 256, dtype=torch.uint8, device="cuda")
        ooffs = torch.arange(N, dtype=torch.int64, device="cuda") * bound
        olens = torch.zeros(N, dtype=torch.int32, device="cuda")
        run(f"lz4 exact, {label}", lambda: L.lz4f_compress_batch(src, offs, lens, dst, ooffs, olens))
        print("  ratio", N * B / int(olens.sum()))
        run(f"lz4 fast, {label}", lambda: L.lz4f_compress_fast_batch(src, offs, lens, dst, ooffs, olens))
        run(f"snappy, {label}", lambda: L.snappy_compress_batch(src, offs, lens, dst, ooffs, olens))
        print("  ratio", N * B / int(olens.sum()))
        # decode what snappy made, then what lz4 makes
        out = torch.empty(N * B + 256, dtype=torch.uint8, device="cuda")
        caps = torch.full((N,), B, dtype=torch.int32, device="cuda")
        dl = torch.zeros(N, dtype=torch.int32, device="cuda")
        st = torch.zeros(N, dtype=torch.int32, device="cuda")
        run(f"snappy uncompress, {label}", lambda: L.snappy_uncompress_batch(dst, ooffs, olens, out, offs, caps, dl, st))
        assert int(st.abs().sum()) == 0 and torch.equal(out[:N * B], src)
        L.lz4f_compress_batch(src, offs, lens, dst, ooffs, olens)
        run(f"lz4 decompress, {label}", lambda: L.lz4f_decompress_batch(dst, ooffs, olens, out, offs, caps, dl, st))
        assert int(st.abs().sum()) == 0 and torch.equal(out[:N * B], src)


if __name__ == "__main__":
    sys.exit(main())
