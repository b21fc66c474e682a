// lz4_wave.h -- wavefront helpers shared by the LZ4 block encoders (the throughput
// engine in lz4_encode_fast.hip and the windowed exact engine in lz4_encode.hip):
// bounds-checked block reads through a raw buffer resource, a DPP prefix sum, and the
// byte-granular pieces of the LZ4 sequence format (lz4.c:961-1073).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lz4_device.h"

namespace rdk {

// All block reads go through a raw buffer resource spanning the block's
// dwords [lo, hi): MUBUF range checking is per dword, so a dword outside the
// block (or a lane parked at kNoLoad) reads 0 and touches no memory.  Loads
// are issued unconditionally, which keeps the compiler's vmcnt bookkeeping
// exact and lets the next round's loads stay in flight.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kNoLoad = 0x80000000u;

__device__ __forceinline__ rsrc_t block_rsrc(uintptr_t lo, uintptr_t hi) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(lo), 0, int(hi - lo),
                                           0x00020000);
}

// nine dwords at block offset a-4 .. a+28 (a 4-aligned, relative to lo).
// The dword before a is its own load: a vector load that starts below the
// resource (a-4 wraps) reads as zero as a whole.
__device__ __forceinline__ void load9(rsrc_t r, uint32_t a, uint32_t d[9]) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  d[0] = __builtin_amdgcn_raw_buffer_load_b32(r, a - 4u, 0, 0);
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0);
  const u4 w = __builtin_amdgcn_raw_buffer_load_b128(r, a + 16u, 0, 0);
  d[1] = v.x; d[2] = v.y; d[3] = v.z; d[4] = v.w;
  d[5] = w.x; d[6] = w.y; d[7] = w.z; d[8] = w.w;
}

// five dwords at block offset a .. a+16
__device__ __forceinline__ void load5(rsrc_t r, uint32_t a, uint32_t d[5]) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0);
  d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  d[4] = __builtin_amdgcn_raw_buffer_load_b32(r, a + 16u, 0, 0);
}

// exclusive prefix sum over the wave by DPP row shifts and row broadcasts
// (no LDS round trips); `total` gets the wave sum
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t &total) {
  int x = int(v);
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false); // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false); // row_bcast:31
  total = uint32_t(__builtin_amdgcn_readlane(x, 63));
  return uint32_t(x) - v;
}

// exclusive running maximum over the wave of non-negative values (lane 0 gets 0): DPP row
// shifts and row broadcasts, then one wave shift
__device__ __forceinline__ int wave_excl_max(int v) {
  int x = v;
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true));   // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true));   // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true));   // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true));   // row_shr:8
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true);        // wave_shr:1
}

// equal bytes a[i]==b[i] for i in [0, limit), 64 per wave step
__device__ __forceinline__ int wave_count_fwd(uintptr_t a, uintptr_t b, int limit, int lane) {
  int cnt = 0;
  while (cnt < limit) {
    const int l = cnt + lane;
    const bool ok = l < limit && ldb(a + l) == ldb(b + l);
    const uint64_t m = ballot(ok);
    const int run = m == ~0ull ? 64 : __builtin_ctzll(~m);
    cnt += run;
    if (run < 64) break;
  }
  return cnt;
}

__device__ __forceinline__ void wave_copy_bytes(uintptr_t d, uintptr_t s, uint32_t len, int lane) {
  for (uint32_t base = 0; base < len; base += 256u) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // (clamped, not predicated: a load under a lane predicate is waited for at once, and
      // the four would be four round trips)
      const uint32_t i = base + lane + 64u * j;
      v[j] = ldb(s + (i < len ? i : len - 1u));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + lane + 64u * j;
      if (i < len) stb(d + i, v[j]);
    }
  }
}

__device__ __forceinline__ uint32_t ext_bytes(uint32_t v) {  // 255-run encoding length
  return v >= 15u ? (v - 15u) / 255u + 1u : 0u;
}

__device__ __forceinline__ uintptr_t put_len(uintptr_t p, uint32_t v) {  // v >= 15
  uint32_t r = v - 15u;
  for (; r >= 255u; r -= 255u) stb(p++, 255u);
  stb(p++, r);
  return p;
}

}  // namespace rdk
