// Read-pattern ceilings for the CRC v4 layout (scratch microbenchmark).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kNoLoad = 0x80000000u;

// G lanes per batch, V vectors (16 B) per lane per step, P steps in flight
template <int G, int V, int P>
__global__ __launch_bounds__(1024, 1) void rd_kernel(const uint8_t *base, uint32_t n, uint32_t bsz, uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const uint32_t l = lane % G;
  const uint32_t gpw = 64 / G;
  const uint32_t grp = (blockIdx.x * blockDim.x + threadIdx.x) / G;
  const uint32_t ngrp = gridDim.x * blockDim.x / G;
  uint32_t acc = 0;
  const uint32_t stepb = G * 16 * V;
  const uint32_t K = bsz / stepb;
  for (uint32_t i0 = (blockIdx.x * blockDim.x + (threadIdx.x & ~63)) / G; i0 < n; i0 += ngrp) {
    const uint32_t i = i0 + (lane / G);
    const uintptr_t sb = reinterpret_cast<uintptr_t>(base) + uint64_t(__builtin_amdgcn_readfirstlane(i0)) * bsz;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(sb), 0, int(kNoLoad), 0x00020000);
    const uint32_t o0 = (i - __builtin_amdgcn_readfirstlane(i0)) * bsz + 16 * V * l;
    const bool act = i < n;
    u32x4 buf[P][V];
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int v = 0; v < V; ++v)
        buf[j][v] = __builtin_amdgcn_raw_buffer_load_b128(rs, act ? o0 + stepb * j + 16 * v : kNoLoad, 0, 2);
    for (uint32_t k0 = 0; k0 < K; k0 += P) {
#pragma unroll
      for (int j = 0; j < P; ++j) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          u32x4 w = buf[j][v];
          const uint32_t k = k0 + j + P;
          buf[j][v] = __builtin_amdgcn_raw_buffer_load_b128(rs, (act && k < K) ? o0 + stepb * k + 16 * v : kNoLoad, 0, 2);
          acc ^= w.x ^ w.y ^ w.z ^ w.w;
        }
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int G, int V, int P>
void run(const char *name, const uint8_t *d, uint32_t n, uint32_t bsz, uint32_t *o, int grid) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((rd_kernel<G, V, P>), dim3(grid), dim3(1024), 0, 0, d, n, bsz, o);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((rd_kernel<G, V, P>), dim3(grid), dim3(1024), 0, 0, d, n, bsz, o);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
  printf("%-28s grid %4d  %.3f ms  %.0f GB/s\n", name, grid, ms, double(n) * bsz / ms / 1e6);
}

int main() {
  const uint32_t n = 1u << 20, bsz = 16384;
  uint8_t *d; uint32_t *o;
  if (hipMalloc(&d, size_t(n) * bsz) != hipSuccess) return 1;
  hipMalloc(&o, 64);
  hipMemset(d, 1, size_t(n) * bsz);
  for (int grid : {256, 512}) {
    run<16, 1, 8>("G16 V1 P8 (v4 pattern)", d, n, bsz, o, grid);
    run<16, 2, 4>("G16 V2 P4", d, n, bsz, o, grid);
    run<16, 4, 2>("G16 V4 P2", d, n, bsz, o, grid);
    run<32, 1, 8>("G32 V1 P8", d, n, bsz, o, grid);
    run<64, 1, 8>("G64 V1 P8 (v3-like)", d, n, bsz, o, grid);
    run<64, 1, 4>("G64 V1 P4", d, n, bsz, o, grid);
    run<16, 1, 16>("G16 V1 P16", d, n, bsz, o, grid);
  }
  return 0;
}
