// win_ring.h -- the source ring of the windowed exact block compressors (LZ4 in
// lz4_encode.hip, snappy in snappy.hip): a block's source streams once through a 4 KiB LDS
// ring in 1 KiB chunks, the next chunk's global load issued one chunk ahead, so a window's
// own bytes and candidates within the last 4 KiB never leave the CU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lz4_device.h"
#include "lz4_wave.h"

namespace rdk {

typedef __attribute__((address_space(3))) uint32_t ring_lds_u32;
typedef __attribute__((address_space(3))) uint8_t ring_lds_u8;
typedef uint32_t ring_u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kRingBytes = 4096, kRingChunk = 1024;

struct SrcRing {
  uintptr_t src;  // the block's first byte
  rsrc_t r;       // the block's dwords (reads outside return 0)
  uint32_t sa;    // src & 3: byte offset of position 0 inside the read resource
  // virtual positions (position + sa) [H - kRingBytes, H) are at ring[v & (kRingBytes-1)].
  // `pend` is the chunk at H, loaded one fill ahead.
  ring_lds_u32 *ring;
  int H;
  ring_u32x4 pend;
};

__device__ __forceinline__ void ring_init(SrcRing &b, uintptr_t src, uint32_t n, ring_lds_u32 *ring,
                                          int lane) {
  b.src = src;
  const uintptr_t lo = src & ~uintptr_t(3);
  b.r = block_rsrc(lo, (src + n + 3u) & ~uintptr_t(3));
  b.sa = uint32_t(src & 3u);
  b.ring = ring;
  b.H = 0;
  b.pend = __builtin_amdgcn_raw_buffer_load_b128(b.r, 16u * uint32_t(lane), 0, 0);
}

// ring[H, H+1 KiB) <- pend; the load of the following chunk is issued at once
__device__ __forceinline__ void ring_fill(SrcRing &b, int lane) {
  typedef __attribute__((address_space(3))) ring_u32x4 lds_u4v;
  const uint32_t at = (uint32_t(b.H) & (kRingBytes - 1u)) + 16u * uint32_t(lane);
  *(lds_u4v *)((ring_lds_u8 *)b.ring + at) = b.pend;
  b.H += int(kRingChunk);
  b.pend = __builtin_amdgcn_raw_buffer_load_b128(b.r, uint32_t(b.H) + 16u * uint32_t(lane), 0, 0);
  asm volatile("" ::: "memory");
}

// nine dwords around virtual position v (4-aligned a = v & ~3): a-4 .. a+28, from the ring.
// Eight consecutive dwords from the ring index of a; the few lanes whose window runs over
// the end of the ring read again with every index wrapped (the straight reads past the
// end land in the LDS behind the ring, which the callers place there: harmless).
__device__ __forceinline__ void ring_load9(const SrcRing &b, uint32_t a, uint32_t d[9]) {
  const uint32_t at = a & (kRingBytes - 1u);
  d[0] = *(ring_lds_u32 *)((ring_lds_u8 *)b.ring + ((a - 4u) & (kRingBytes - 1u)));
  ring_lds_u32 *p = (ring_lds_u32 *)((ring_lds_u8 *)b.ring + at);
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k + 1] = p[k];
  const bool wraps = at > kRingBytes - 32u;
  if (ballot(wraps)) {
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const uint32_t v =
          *(ring_lds_u32 *)((ring_lds_u8 *)b.ring + ((at + 4u * uint32_t(k)) & (kRingBytes - 1u)));
      if (wraps) d[k + 1] = v;
    }
  }
}

// The same nine dwords for a lane whose window lies inside the ring without running over
// either end (ring_straight(a)): one address, nine fixed offsets.  A lane for which that does
// not hold reads LDS it has no use for (its address is kept inside the allocation).
__device__ __forceinline__ bool ring_straight(uint32_t a) {
  const uint32_t at = a & (kRingBytes - 1u);
  return at - 4u <= kRingBytes - 36u - 4u;  // 4 <= at && at + 32 <= kRingBytes
}
__device__ __forceinline__ void ring_load9_straight(const SrcRing &b, uint32_t a, uint32_t d[9]) {
  uint32_t at = a & (kRingBytes - 1u);
  at = at < 4u ? 4u : at;
  ring_lds_u32 *p = (ring_lds_u32 *)((ring_lds_u8 *)b.ring + (at - 4u));
#pragma unroll
  for (int k = 0; k < 9; ++k) d[k] = p[k];
}

__device__ __forceinline__ bool ring_has(const SrcRing &b, int v_lo, int v_hi) {  // [v_lo, v_hi)
  return v_lo >= b.H - int(kRingBytes) && v_hi <= b.H;
}

// equal bytes a[i]==b[i], i < limit, 64 per wave step; a / c are block positions.  Steps
// whose bytes are all in the ring read LDS, the others global memory.
__device__ __forceinline__ int win_count_fwd(const SrcRing &b, int a, int c, int limit, int lane) {
  int cnt = 0;
  while (cnt < limit) {
    const int l = cnt + lane;
    const int va = a + cnt + int(b.sa), vc = c + cnt + int(b.sa);
    uint32_t x, y;
    if (ring_has(b, vc, vc + 64) && ring_has(b, va, va + 64)) {
      x = ((ring_lds_u8 *)b.ring)[uint32_t(va + lane) & (kRingBytes - 1u)];
      y = ((ring_lds_u8 *)b.ring)[uint32_t(vc + lane) & (kRingBytes - 1u)];
    } else {
      x = l < limit ? ldb(b.src + uint32_t(a + l)) : 0u;
      y = l < limit ? ldb(b.src + uint32_t(c + l)) : 1u;
    }
    const uint64_t m = ballot(l < limit && x == y);
    const int run = m == ~0ull ? 64 : __builtin_ctzll(~m);
    cnt += run;
    if (run < 64) break;
  }
  return cnt;
}

__device__ __forceinline__ uint64_t bits_below(int x) {  // lanes [0, x), x in 0..64
  return x >= 64 ? ~0ull : ((1ull << x) - 1ull);
}
__device__ __forceinline__ uint64_t bits_range(int a, int b) {  // lanes [a, b)
  return a >= b ? 0ull : (bits_below(b) & ~bits_below(a));
}

}  // namespace rdk
