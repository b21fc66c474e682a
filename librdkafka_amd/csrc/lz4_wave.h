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

// A block move by kThreads threads: sz bytes from `from` down to `to` (to < from in the same
// buffer, or another buffer).  The destination is cut at its 16-byte
// boundaries: up to 15 head bytes, whole 16-byte units, up to 15 tail bytes.  A unit is
// fetched as five dwords around its source (the source is not aligned to the destination; the
// fetch goes through a range-checked resource, so it never reads past the block) and stored
// as one aligned 16-byte word.  Each step reads four units per thread, then -- behind a
// barrier, because a step's destination may overlap its own source -- writes them; the head
// travels with the first step and the tail with the last, whose sources nothing before them
// overwrites (a step's destination ends below the next step's source).
// kBarrier = false: one wavefront moving between buffers that do not overlap.
template <uint32_t kAsmThreads, bool kBarrier = true>
__device__ __forceinline__ void asm_slide(uintptr_t to, uintptr_t from, uint32_t sz, int t) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) u4 g_u4;
  const uint32_t head0 = uint32_t(-intptr_t(to)) & 15u;
  const uint32_t head = head0 < sz ? head0 : sz;
  const uint32_t units = (sz - head) >> 4;
  const uint32_t tail = sz - head - (units << 4);
  const uint32_t fa = uint32_t(from & 3u);
  const rsrc_t rs = block_rsrc(from - fa, (from + sz + 3u) & ~uintptr_t(3));
  const uint32_t sh = (fa + head) & 3u;  // a unit's first byte inside its first dword
  constexpr uint32_t kPer = 4;
  for (uint32_t u0 = 0;; u0 += kAsmThreads * kPer) {
    const bool first = u0 == 0u, last = u0 + kAsmThreads * kPer >= units;
    u4 a[kPer];
    uint32_t e[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      const uint32_t u = u0 + uint32_t(t) + kAsmThreads * j;
      const uint32_t off = u < units ? ((fa + head + (u << 4)) & ~3u) : kNoLoad;
      a[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
      e[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 16u, 0, 0);
    }
    // head and tail bytes, one per thread (threads 0..14 and 16..30)
    uint32_t hb = 0, tb = 0;
    const bool do_h = first && uint32_t(t) < head;
    const bool do_t = last && uint32_t(t) >= 16u && uint32_t(t) - 16u < tail;
    if (do_h) hb = ldb(from + uint32_t(t));
    if (do_t) tb = ldb(from + head + (units << 4) + (uint32_t(t) - 16u));
    if (kBarrier) __syncthreads();  // the step is fully read before any of it is written
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      const uint32_t u = u0 + uint32_t(t) + kAsmThreads * j;
      if (u < units) {
        u4 v;
        v.x = __builtin_amdgcn_alignbyte(a[j].y, a[j].x, sh);
        v.y = __builtin_amdgcn_alignbyte(a[j].z, a[j].y, sh);
        v.z = __builtin_amdgcn_alignbyte(a[j].w, a[j].z, sh);
        v.w = __builtin_amdgcn_alignbyte(e[j], a[j].w, sh);
        *(g_u4 *)(to + head + (u << 4)) = v;
      }
    }
    if (do_h) stb(to + uint32_t(t), hb);
    if (do_t) stb(to + head + (units << 4) + (uint32_t(t) - 16u), tb);
    if (last) break;
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
