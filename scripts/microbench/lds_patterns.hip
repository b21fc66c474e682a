// LDS access-pattern timing on gfx950: cycles per wave instruction (s_memtime around 64
// back-to-back instructions, one wave per SIMD, 4 waves on the CU), for the patterns the LZ4
// unit compressor uses.  Build: hipcc --offload-arch=gfx950 -O3 lds_patterns.hip -o lds_patterns
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x2_a1 __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32_a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;
#define LDSV4U(p) (*(__attribute__((address_space(3))) const u32x4_a1 *)(p))
#define LDSV2U(p) (*(__attribute__((address_space(3))) const u32x2_a1 *)(p))
#define LDSU32U(p) (*(__attribute__((address_space(3))) const u32_a1 *)(p))
#define LDSV4(p) (*(__attribute__((address_space(3))) const u32x4 *)(p))
#define LDSU16(p) (*(__attribute__((address_space(3))) const uint16_t *)(p))

template <int MODE>
__global__ __launch_bounds__(256) void k(const uint32_t *rnd, uint64_t *out, uint32_t *sink) {
  __shared__ __attribute__((aligned(16))) uint8_t mem[65536 + 256];
  lds_u8 *L = (lds_u8 *)mem;
  for (int i = threadIdx.x; i < 65536 / 4; i += 256) ((uint32_t *)mem)[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  uint32_t addr[8];
  for (int j = 0; j < 8; ++j) {
    const uint32_t r = rnd[(blockIdx.x * 256 + threadIdx.x) * 8 + j];
    switch (MODE) {
      case 0: addr[j] = 1024 * j + lane + 3; break;                 // b128, stride 1 byte (own window)
      case 1: addr[j] = (r % 65000u); break;                        // b128, random unaligned
      case 2: addr[j] = (r % 65000u) & ~15u; break;                 // b128, random 16-aligned
      case 3: addr[j] = 1024 * j + 16 * lane; break;                // b128, aligned consecutive
      case 4: addr[j] = 1024 * j + lane + 1; break;                 // b32, stride 1 byte
      case 5: addr[j] = (r % 65000u); break;                        // b32, random unaligned
      case 6: addr[j] = (r % 32000u) * 2; break;                    // u16 random
      case 7: addr[j] = (r % 16000u) * 4; break;                    // ds_max_u32 random
      case 8: addr[j] = (r % 65000u) & ~3u; break;                  // b128, random 4-aligned
      case 9: addr[j] = 1024 * j + 4 * lane; break;                 // b128 at stride 4 bytes (overlapping, dword aligned)
      case 10: addr[j] = (r % 65000u); break;                       // b64, random unaligned
      case 11: addr[j] = 1024 * j + 2 * lane; break;                // u16 consecutive (ring row)
    }
  }
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int rep = 0; rep < 8; ++rep) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MODE <= 3 || MODE == 8 || MODE == 9) { const u32x4_a1 v = LDSV4U(L + addr[j]); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
      else if (MODE == 4 || MODE == 5) acc ^= LDSU32U(L + addr[j]);
      else if (MODE == 6 || MODE == 11) acc ^= LDSU16(L + addr[j]);
      else if (MODE == 7) __hip_atomic_fetch_max((__attribute__((address_space(3))) uint32_t *)(L + addr[j]), acc + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else if (MODE == 10) { const u32x2_a1 v = LDSV2U(L + addr[j]); acc ^= v.x ^ v.y; }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE> void run(const char *name, uint32_t *rnd, uint64_t *out, uint32_t *sink) {
  k<MODE><<<256, 256>>>(rnd, out, sink);
  k<MODE><<<256, 256>>>(rnd, out, sink);
  hipDeviceSynchronize();
  uint64_t h[1024];
  hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 1024; ++i) s += double(h[i]);
  printf("%-40s %7.1f cycles per wave instruction (4 waves per CU issuing)\n", name, s / 1024 / 64);
}

int main() {
  uint32_t *rnd, *sink; uint64_t *out;
  hipMalloc(&rnd, 256 * 256 * 8 * 4); hipMalloc(&sink, 256 * 256 * 4); hipMalloc(&out, 1024 * 8);
  uint32_t *h = (uint32_t *)malloc(256 * 256 * 8 * 4);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < 256 * 256 * 8; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = uint32_t(s >> 16); }
  hipMemcpy(rnd, h, 256 * 256 * 8 * 4, hipMemcpyHostToDevice);
  run<3>("b128 aligned consecutive", rnd, out, sink);
  run<0>("b128 stride 1 byte (own window)", rnd, out, sink);
  run<9>("b128 stride 4 bytes (overlapping)", rnd, out, sink);
  run<1>("b128 random unaligned", rnd, out, sink);
  run<8>("b128 random 4-aligned", rnd, out, sink);
  run<2>("b128 random 16-aligned", rnd, out, sink);
  run<10>("b64 random unaligned", rnd, out, sink);
  run<4>("b32 stride 1 byte", rnd, out, sink);
  run<5>("b32 random unaligned", rnd, out, sink);
  run<6>("u16 random", rnd, out, sink);
  run<11>("u16 consecutive", rnd, out, sink);
  run<7>("ds_max_u32 random", rnd, out, sink);
  return 0;
}
