// crc32c.hip -- CRC32C kernels for gfx950 (MI355X).
//
// Replaces crc32c() (src/crc32c.c:360) / rd_slice_crc32c() (src/rdbuf.c:1113)
// as called by the MessageSet writer (rdkafka_msgset_writer.c:1229-1246) and
// reader (rdkafka_msgset_reader.c:982-1015).
//
// Design:
//   * one wavefront per byte range (a record batch), persistent grid;
//   * lane l of iteration k owns the 16-byte vector at V + 1024k + 16l, so
//     every global_load_dwordx4 of the wave reads 1 KiB contiguous (coalesced);
//   * v3 (default): a lane runs Horner over its 4-byte words, u = M(u ^ w),
//     where M (advance 4 bytes; 1012 bytes for the first word of a vector,
//     folding in the lane's 1008-byte gap) is evaluated as 8 lookups in
//     32-fold replicated nibble tables: conflict-free LDS banks and one
//     v_and_or_b32 per lookup address (crc32c_tables.h "v3 image");
//   * v1 (RDK_HIP_CRC_V1=1): 16 byte slicing tables + 4-lookup 1024-byte
//     operator; measured LDS-conflict bound (profiles/r01_crc_v1_*);
//   * the 64 lane registers are merged by a 6-level xor-shuffle tree whose
//     level m applies the "advance 16*2^m bytes" operator -- the GF(2)
//     combine of crc32c.c:144-231 generalised from 3 streams to 64 lanes;
//   * unaligned starts are zero-masked (leading zeros do not change a raw
//     CRC), the caller's running crc is injected by xor into the first four
//     message bytes, and the <16-byte tail is folded in by the last lane.
#include <hip/hip_runtime.h>

#include "common.h"
#include "crc32c_tables.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace rdk {

// threads per workgroup: v3's 57 KiB of tables fit twice per CU -> 2 x 16 waves;
// v1's 40 KiB fit four times -> 4 x 8 waves
template <int V> constexpr int crc_block() { return V == 3 ? 1024 : 512; }
constexpr int kCrcSmall = 64;        // ranges shorter than this: serial lane
constexpr uint32_t kCrcChunk = 65536; // split of long single ranges

// LDS-qualified pointer: keeps table lookups as ds_read_b32 with an immediate
// table offset instead of generic (flat) address arithmetic.
typedef __attribute__((address_space(3))) const uint32_t lds_u32;

__device__ __forceinline__ uint32_t L8(const lds_u32 *L, int table, uint32_t byte) {
  return L[(table << 8) + byte];
}

// raw CRC register advanced by 4 zero bytes... n bytes via a 4x256 operator
__device__ __forceinline__ uint32_t shift_op(const lds_u32 *L, int base, uint32_t x) {
  return L8(L, base, x & 0xffu) ^ L8(L, base + 1, (x >> 8) & 0xffu) ^
         L8(L, base + 2, (x >> 16) & 0xffu) ^ L8(L, base + 3, x >> 24);
}

// advance 16 bytes: state byte j is followed by 15-j bytes -> T[15-j]
__device__ __forceinline__ uint32_t shift16(const lds_u32 *L, uint32_t x) {
  return L8(L, 15, x & 0xffu) ^ L8(L, 14, (x >> 8) & 0xffu) ^
         L8(L, 13, (x >> 16) & 0xffu) ^ L8(L, 12, x >> 24);
}

// raw CRC (zero register) of one 16-byte vector, byte i -> T[15-i]
__device__ __forceinline__ uint32_t raw16(const lds_u32 *L, uint4 w) {
  uint32_t a = L8(L, 15, w.x & 0xffu) ^ L8(L, 14, (w.x >> 8) & 0xffu) ^
               L8(L, 13, (w.x >> 16) & 0xffu) ^ L8(L, 12, w.x >> 24);
  uint32_t b = L8(L, 11, w.y & 0xffu) ^ L8(L, 10, (w.y >> 8) & 0xffu) ^
               L8(L, 9, (w.y >> 16) & 0xffu) ^ L8(L, 8, w.y >> 24);
  uint32_t c = L8(L, 7, w.z & 0xffu) ^ L8(L, 6, (w.z >> 8) & 0xffu) ^
               L8(L, 5, (w.z >> 16) & 0xffu) ^ L8(L, 4, w.z >> 24);
  uint32_t d = L8(L, 3, w.w & 0xffu) ^ L8(L, 2, (w.w >> 8) & 0xffu) ^
               L8(L, 1, (w.w >> 16) & 0xffu) ^ L8(L, 0, w.w >> 24);
  return (a ^ b) ^ (c ^ d);
}

// Zero the bytes of dword [d, d+4) that precede `s`, and xor the 4-byte
// injected register `ninit` (placed at byte address s) into it.
__device__ __forceinline__ uint32_t head_fix(uint32_t v, uintptr_t d, uintptr_t s, uint32_t ninit) {
  if (d + 4 <= s) v = 0;
  else if (d < s) v &= 0xffffffffu << (8u * uint32_t(s - d));
  long rel = long(s) - long(d);
  if (rel >= 0 && rel < 4) v ^= ninit << (8u * uint32_t(rel));
  else if (rel < 0 && rel > -4) v ^= ninit >> (8u * uint32_t(-rel));
  return v;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gbl_u32x4;
__device__ __forceinline__ uint4 ldg16(uintptr_t a) {
  // streamed once: non-temporal hint keeps it from evicting L2-resident tables
  const u32x4 v = __builtin_nontemporal_load((gbl_u32x4 *)a);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// CRC32C of [s, e) by one wavefront.  `inject`: the range starts a message
// whose previous crc is `init` (crc32c() chaining); `final`: return the
// inverted crc32c() value, else the raw register (for later combining).
// The result is valid in every lane.
__device__ __attribute__((always_inline)) uint32_t wave_crc(uintptr_t s, uintptr_t e,
                                                           uint32_t init, bool inject,
                                                           bool final, const lds_u32 *L,
                                                           int lane) {
  const size_t len = e - s;
  uint32_t x;
  if (len < size_t(kCrcSmall)) {
    uint32_t c = inject ? ~init : 0u;
    if (lane == 0) {
      typedef __attribute__((address_space(1))) const uint8_t gbl_u8;
      gbl_u8 *p = (gbl_u8 *)s;
      for (size_t i = 0; i < len; ++i) c = L8(L, 0, (c ^ p[i]) & 0xffu) ^ (c >> 8);
    }
    x = __builtin_amdgcn_readfirstlane(c);
    return final ? ~x : x;
  }
  const uintptr_t A = s & ~uintptr_t(15), B = e & ~uintptr_t(15);
  const uint32_t nb = uint32_t((B - A) >> 4);
  const uint32_t K = (nb + 63u) >> 6;
  const uintptr_t V = B - uintptr_t(K) * 1024u;
  const uint32_t ninit = inject ? ~init : 0u;
  const int sh1024 = crc_shift_table(6);

  uintptr_t blk = V + uintptr_t(lane) * 16u;
  uint4 nxt = make_uint4(0, 0, 0, 0);
  if (blk >= A) nxt = ldg16(blk);
  uint32_t r = 0;
  for (uint32_t k = 0; k < K; ++k) {
    uint4 w = nxt;
    const uintptr_t cb = blk;
    blk += 1024u;
    if (k + 1 < K) nxt = ldg16(blk);  // software prefetch of the next 1 KiB
    if (cb < A + 32u) {
      w.x = head_fix(w.x, cb, s, ninit);
      w.y = head_fix(w.y, cb + 4, s, ninit);
      w.z = head_fix(w.z, cb + 8, s, ninit);
      w.w = head_fix(w.w, cb + 12, s, ninit);
    }
    if (k) r = shift_op(L, sh1024, r);
    r ^= raw16(L, w);
  }
  // 64-lane merge tree: lane l (bit m set) absorbs lane l-2^m, 16*2^m earlier
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    uint32_t y = (m == 0) ? shift16(L, r) : shift_op(L, crc_shift_table(m), r);
    y = __shfl_xor(y, 1 << m);
    if (lane & (1 << m)) r ^= y;
  }
  // lane 63 now holds the register for [A, B); fold the tail [B, e)
  const uint32_t t = uint32_t(e - B);
  if (lane == 63 && t) {
    const uint4 tw = ldg16(B);
    uint32_t y = (t < 4) ? (r >> (8u * t)) : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
      if (j < t) y ^= L8(L, int(t - 1 - j), (r >> (8 * j)) & 0xffu);
    const uint32_t tv[4] = {tw.x, tw.y, tw.z, tw.w};
#pragma unroll
    for (uint32_t i = 0; i < 15; ++i)
      if (i < t) y ^= L8(L, int(t - 1 - i), (tv[i >> 2] >> (8 * (i & 3))) & 0xffu);
    r = y;
  }
  x = __builtin_amdgcn_readlane(r, 63);
  return final ? ~x : x;
}


// ---------------------------------------------------------------- v3 path
// LDS read at absolute byte address `a` + immediate `off` (the dynamic LDS
// block is the kernel's only LDS, so it starts at 0 -- checked on the host
// side by the parity tests, any other base would fail every CRC).
__device__ __forceinline__ uint32_t lds_rd(uint32_t a, uint32_t off) {
  return *reinterpret_cast<const lds_u32 *>(size_t(a + off));
}

// a ^ b ^ c in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96 (the
// compiler emits two v_xor_b32 for it)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// M(x) ^ extra for map MAP (0: advance 1012 zero bytes, 1: advance 4), 8
// lookups whose addresses are one v_and_or_b32 each (crc32c_tables.h "v3 image")
template <int MAP>
__device__ __forceinline__ uint32_t map_v3(uint32_t x, uint32_t lc4, uint32_t extra = 0u) {
  const uint32_t y1 = __builtin_amdgcn_alignbit(x, x, 8);
  const uint32_t y2 = __builtin_amdgcn_alignbit(x, x, 16);
  const uint32_t y3 = __builtin_amdgcn_alignbit(x, x, 24);
  constexpr uint32_t s7 = kV3S7 + MAP * 4 * 2048, s11 = kV3S11 + MAP * 4 * 128;
  const uint32_t a0 = lds_rd((x & 0x780u) | lc4, s7), b0 = lds_rd((x & 0x7800u) | lc4, s11);
  const uint32_t a1 = lds_rd((y1 & 0x780u) | lc4, s7 + 2048), b1 = lds_rd((y1 & 0x7800u) | lc4, s11 + 128);
  const uint32_t a2 = lds_rd((y2 & 0x780u) | lc4, s7 + 4096), b2 = lds_rd((y2 & 0x7800u) | lc4, s11 + 256);
  const uint32_t a3 = lds_rd((y3 & 0x780u) | lc4, s7 + 6144), b3 = lds_rd((y3 & 0x7800u) | lc4, s11 + 384);
  return xor3(xor3(a0, b0, a1), xor3(b1, a2, b2), xor3(a3, b3, extra));
}

__device__ __forceinline__ uint32_t byte_tab(int i, uint32_t b) {
  return lds_rd(b << 2, uint32_t(v3_byte_table(i)));
}

__device__ __forceinline__ uint32_t shift_tree_v3(int m, uint32_t x) {
  return byte_tab(m * 4, x & 0xffu) ^ byte_tab(m * 4 + 1, (x >> 8) & 0xffu) ^
         byte_tab(m * 4 + 2, (x >> 16) & 0xffu) ^ byte_tab(m * 4 + 3, x >> 24);
}

// Absorb one lane's 16-byte vector (at cb) into its register: Horner over
// 4-byte words (the slicing-by-4 step of crc32c.c:110-125), with the 1008
// bytes owned by the other lanes folded into the first word's map.
template <bool HEAD>
__device__ __forceinline__ void absorb_vec(uint32_t &u, uint4 w, uintptr_t cb, uintptr_t A,
                                           uintptr_t s, uint32_t ninit, uint32_t lc4,
                                           bool first) {
  if (HEAD && cb < A + 32u) {  // head: zero bytes before s, inject the running crc
    w.x = head_fix(w.x, cb, s, ninit);
    w.y = head_fix(w.y, cb + 4, s, ninit);
    w.z = head_fix(w.z, cb + 8, s, ninit);
    w.w = head_fix(w.w, cb + 12, s, ninit);
  }
  u = first ? w.x : map_v3<0>(u, lc4, w.x);
  u = map_v3<1>(u, lc4, w.y);
  u = map_v3<1>(u, lc4, w.z);
  u = map_v3<1>(u, lc4, w.w);
}

constexpr int kCrcPrefetch = 4;  // 1 KiB wave steps in flight per wave

// steps k0 .. k0+kCrcPrefetch-1; buffer j is reloaded right after use (3 KiB
// per wave stay in flight while it is absorbed)
template <bool HEAD>
__device__ __forceinline__ void crc_round(uint32_t &u, uint4 (&buf)[kCrcPrefetch], uint32_t k0,
                                          uint32_t K, uintptr_t base, uintptr_t A, uintptr_t s,
                                          uint32_t ninit, uint32_t lc4) {
#pragma unroll
  for (int j = 0; j < kCrcPrefetch; ++j) {
    const uint32_t k = k0 + uint32_t(j);
    if (k < K) {
      const uintptr_t cb = base + uintptr_t(k) * kLaneStride;
      absorb_vec<HEAD>(u, buf[j], cb, A, s, ninit, lc4, HEAD && j == 0);
      if (k + kCrcPrefetch < K) buf[j] = ldg16(cb + kCrcPrefetch * kLaneStride);
    }
  }
}

__device__ __attribute__((always_inline)) uint32_t wave_crc_v3(uintptr_t s, uintptr_t e,
                                                              uint32_t init, bool inject,
                                                              bool final, int lane) {
  typedef __attribute__((address_space(1))) const uint8_t gbl_u8;
  const size_t len = e - s;
  uint32_t x;
  if (len < size_t(kCrcSmall)) {
    uint32_t c = inject ? ~init : 0u;
    if (lane == 0) {
      gbl_u8 *p = (gbl_u8 *)s;
      for (size_t i = 0; i < len; ++i) c = byte_tab(kV3T0, (c ^ p[i]) & 0xffu) ^ (c >> 8);
    }
    x = __builtin_amdgcn_readfirstlane(c);
    return final ? ~x : x;
  }
  const uintptr_t A = s & ~uintptr_t(15), B = e & ~uintptr_t(15);
  const uint32_t nb = uint32_t((B - A) >> 4);
  const uint32_t K = (nb + 63u) >> 6;  // 1 KiB wave steps
  const uintptr_t V = B - uintptr_t(K) * kLaneStride;
  const uint32_t ninit = inject ? ~init : 0u;
  const uint32_t lc4 = (uint32_t(lane) & 31u) << 2;

  // kCrcPrefetch register buffers rotate through the steps: buffer j holds
  // step k0+j and is reloaded with step k0+j+kCrcPrefetch as soon as it has
  // been absorbed (no register copies; up to 4 KiB per wave in flight).
  // Only step 0 can start below A, and the head ([s, s+4)) lies in steps 0-1.
  const uintptr_t base = V + uintptr_t(lane) * 16u;
  uint4 buf[kCrcPrefetch];
#pragma unroll
  for (int j = 0; j < kCrcPrefetch; ++j) {
    buf[j] = make_uint4(0, 0, 0, 0);
    const uintptr_t a = base + uintptr_t(j) * kLaneStride;
    if (uint32_t(j) < K && a >= A) buf[j] = ldg16(a);
  }
  uint32_t u = 0;
  crc_round<true>(u, buf, 0u, K, base, A, s, ninit, lc4);  // steps 0-3 (head)
  for (uint32_t k0 = kCrcPrefetch; k0 < K; k0 += kCrcPrefetch)
    crc_round<false>(u, buf, k0, K, base, A, s, ninit, lc4);
  uint32_t r = map_v3<1>(u, lc4);
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    uint32_t y = shift_tree_v3(m, r);
    y = __shfl_xor(y, 1 << m);
    if (lane & (1 << m)) r ^= y;
  }
  const uint32_t t = uint32_t(e - B);
  if (lane == 63 && t) {  // fold the <16-byte tail byte by byte (crc32c.c:131)
    gbl_u8 *p = (gbl_u8 *)B;
    for (uint32_t i = 0; i < t; ++i) r = byte_tab(kV3T0, (r ^ p[i]) & 0xffu) ^ (r >> 8);
  }
  x = __builtin_amdgcn_readlane(r, 63);
  return final ? ~x : x;
}

// ---------------------------------------------------------------- v4 path
// Four ranges per wavefront, one per 16-lane group (crc32c_tables.h "v4 image").
// Per 16-byte vector a lane does 16 LDS lookups whose addresses are one v_perm_b32
// each, and 8 xor3: half the LDS cycles of v3 per byte.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kNoLoad = 0x80000000u;  // buffer offset past num_records: reads 0
constexpr uint32_t kV4Span = 0x7f000000u;  // ranges of one pass lie within this of its base
#ifndef RDK_V4_AUX
#define RDK_V4_AUX 2  // nt: streamed once
#endif
#ifndef RDK_V4_PREFETCH
#define RDK_V4_PREFETCH 4
#endif
constexpr int kV4Prefetch = RDK_V4_PREFETCH;  // group steps in flight per lane (x kV4Vecs loads)

// selector: byte 0 <- C byte t (4c | 0x80t), byte 1 <- register byte q, byte 2 <- C byte 2
// (0x01) for the upper half, else 0; byte 3 <- 0
typedef __attribute__((address_space(3))) const uint8_t lds_c8;
// LDS read at byte offset a + off of the kernel's table image Lb (a static array, the
// kernel's only LDS object: reads through it keep the allocation alive and fold to
// absolute addresses)
__device__ __forceinline__ uint32_t lds4(const lds_u32 *Lb, uint32_t a, uint32_t off) {
  return *reinterpret_cast<const lds_u32 *>(reinterpret_cast<lds_c8 *>(Lb) + a + off);
}

template <int Q> constexpr uint32_t v4_sel() {
  return uint32_t(Q & 1) | (uint32_t(4 + Q) << 8) | (uint32_t((Q >> 1) ? 2 : 12) << 16) |
         (12u << 24);
}

__device__ __forceinline__ uint32_t v4_step(const lds_u32 *Lb, uint32_t r, uint32_t w, uint32_t C) {
#if defined(RDK_V4_ABL) && RDK_V4_ABL == 2  // timing ablation only: no table lookups
  return xor3(r, w, C);
#endif
  const uint32_t a = lds4(Lb, __builtin_amdgcn_perm(r, C, v4_sel<0>()), 0);
  const uint32_t b = lds4(Lb, __builtin_amdgcn_perm(r, C, v4_sel<1>()), 0);
  const uint32_t c = lds4(Lb, __builtin_amdgcn_perm(r, C, v4_sel<2>()), 0);
  const uint32_t d = lds4(Lb, __builtin_amdgcn_perm(r, C, v4_sel<3>()), 0);
  return xor3(xor3(a, b, c), d, w);
}

__device__ __forceinline__ uint32_t v4_z4(const lds_u32 *Lb, uint32_t x) {
  return lds4(Lb, (x & 0xffu) << 2, kV4Z4) ^ lds4(Lb, ((x >> 8) & 0xffu) << 2, kV4Z4 + 1024) ^
         lds4(Lb, ((x >> 16) & 0xffu) << 2, kV4Z4 + 2048) ^ lds4(Lb, (x >> 24) << 2, kV4Z4 + 3072);
}

__device__ __forceinline__ uint32_t v4_z256(const lds_u32 *Lb, uint32_t x) {
  return lds4(Lb, (x & 0xffu) << 2, kV4Z256) ^ lds4(Lb, ((x >> 8) & 0xffu) << 2, kV4Z256 + 1024) ^
         lds4(Lb, ((x >> 16) & 0xffu) << 2, kV4Z256 + 2048) ^
         lds4(Lb, (x >> 24) << 2, kV4Z256 + 3072);
}

__device__ __forceinline__ uint32_t v4_fin(const lds_u32 *Lb, uint32_t x, uint32_t lc4) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= lds4(Lb, (((x >> (4 * i)) & 15u) << 7) | lc4, kV4Fin + 2048 * i);
  return r;
}

__device__ __forceinline__ uint32_t v4_t0(const lds_u32 *Lb, uint32_t r, uint32_t byte) {
  return lds4(Lb, ((r ^ byte) & 0xffu) << 2, kV4T0) ^ (r >> 8);
}

// xor over the 16 lanes of a DPP row (= one group)
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x122, 0xf, 0xf, false);  // row_ror:2
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x121, 0xf, 0xf, false);  // row_ror:1
  return v;
}

__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(v), l);
  const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(v >> 32), l);
  return (uint64_t(hi) << 32) | lo;
}

// Raw CRC register (before the final inversion) of the group's range [s, e), whose
// running crc is injected as ninit = ~init; valid in every lane of the group.  `active`
// must be uniform within a group.  Groups whose ranges lie within kV4Span of each
// other share one pass over their longest range (shorter ones start with zero
// vectors, which leave a raw register unchanged); others take further passes.
__device__ __attribute__((always_inline)) uint32_t group_crc_v4(uintptr_t s, uintptr_t e,
                                                               uint32_t ninit, bool active,
                                                               int lane, const lds_u32 *Lb) {
  typedef __attribute__((address_space(1))) const uint8_t gbl_u8;
  const uint32_t l = uint32_t(lane) & uint32_t(kV4Lanes - 1);
  const uint32_t lc4 = (uint32_t(lane) & 31u) << 2;
  const uint32_t C = lc4 | ((lc4 | 0x80u) << 8) | (1u << 16);
  const size_t len = active ? e - s : 0;
  const bool big = active && len >= size_t(kCrcSmall);
  if (active && !big) {  // short range: byte-serial, every lane of the group alike
    uint32_t c = ninit;
    gbl_u8 *p = (gbl_u8 *)s;
    for (size_t i = 0; i < len; ++i) c = v4_t0(Lb, c, p[i]);
    return c;
  }
  const uintptr_t A = s & ~uintptr_t(15), B = e & ~uintptr_t(15);
  constexpr int NV = kV4Vecs;
  constexpr int P = kV4Prefetch;
  constexpr uint32_t VPS = uint32_t(kV4Lanes * NV);  // group vectors per step
  const uint32_t K = big ? uint32_t(((B - A) >> 4) + VPS - 1u) / VPS : 0u;  // steps
  uint32_t R[NV][4] = {};  // Horner registers; a lane only steps them in its own pass
  // groups still to do: one bit per group leader lane
  uint64_t todo = __builtin_amdgcn_ballot_w64(big && l == 0);
  while (todo) {
    // pass base: the lowest A among the remaining groups
    uintptr_t sb = ~uintptr_t(0);
    for (uint64_t t = todo; t; t &= t - 1) {
      const uintptr_t a = rdlane64(A, int(__builtin_ctzll(t)));
      sb = a < sb ? a : sb;
    }
    const bool inpass = big && ((todo >> (lane & (64 - kV4Lanes))) & 1u) && B - sb < kV4Span;
    const uint64_t pm = __builtin_amdgcn_ballot_w64(inpass && l == 0);
    todo &= ~pm;
    uint32_t Kmax = 0;
    for (uint64_t t = pm; t; t &= t - 1) {
      const uint32_t k = __builtin_amdgcn_readlane(K, int(__builtin_ctzll(t)));
      Kmax = k > Kmax ? k : Kmax;
    }
    // whole blocks of P steps: extra leading steps lie before every range and read zeros,
    // which leave a raw CRC register unchanged
    Kmax = (Kmax + P - 1) / P * P;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(sb), 0,
                                                        int(kNoLoad), 0x00020000);
    // lane offsets relative to sb: vector v of step k at o0 + kV4Step*k + 256v; below
    // lowA (before the range, including the shorter ranges' leading steps) the load is
    // parked and reads 0 (lanes outside the pass: o0 = INT32_MIN, every offset >= kNoLoad)
    const int32_t o0 =
        inpass ? int32_t(uint32_t(B - sb) - kV4Step * Kmax + 16u * l) : int32_t(kNoLoad);
    const int32_t lowA = inpass ? int32_t(uint32_t(A - sb)) : 0x7fffffff;
    const uint32_t srel = uint32_t(s - sb);
    auto voff = [&](uint32_t k, int v) -> int32_t { return o0 + int32_t(kV4Step * k + kV4Row * v); };
    auto off = [&](uint32_t k, int v) -> uint32_t {
      const int32_t o = voff(k, v);
      return (k < Kmax && o >= lowA) ? uint32_t(o) : kNoLoad;
    };
    // last step holding a head vector ([A, A+32) of some range in the pass): blocks after it
    // load unconditionally and skip the head check
    uint32_t khead = 0;
    {
      const int32_t kl = inpass ? (lowA + 31 - o0) / kV4Step : 0;  // per group leader (l = 0)
      for (uint64_t t = pm; t; t &= t - 1) {
        const int32_t k = __builtin_amdgcn_readlane(kl, int(__builtin_ctzll(t)));
        khead = uint32_t(k) > khead ? uint32_t(k) : khead;
      }
    }
    u32x4 buf[P][NV];
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v)
        buf[j][v] = __builtin_amdgcn_raw_buffer_load_b128(rs, off(uint32_t(j), v), 0, RDK_V4_AUX);
    // one block = P steps; CHK: its steps may hold heads and its loads may fall outside
    // the ranges.  Each slot is refilled right after it is consumed, so the load ring keeps
    // its registers across blocks and loops (no drains).
    auto block = [&](uint32_t k0, auto chk) __attribute__((always_inline)) {
      constexpr bool CHK = decltype(chk)::value;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const uint32_t k = k0 + uint32_t(j);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          u32x4 w = buf[j][v];
          if (CHK) {
            const int32_t oc = voff(k, v);
            if (oc >= lowA && oc < lowA + 32) {  // head: zero bytes before s, inject ninit
              const uintptr_t d = uintptr_t(uint32_t(oc));
              w.x = head_fix(w.x, d, srel, ninit);
              w.y = head_fix(w.y, d + 4, srel, ninit);
              w.z = head_fix(w.z, d + 8, srel, ninit);
              w.w = head_fix(w.w, d + 12, srel, ninit);
            }
          }
          R[v][0] = v4_step(Lb, R[v][0], w.x, C);
          R[v][1] = v4_step(Lb, R[v][1], w.y, C);
          R[v][2] = v4_step(Lb, R[v][2], w.z, C);
          R[v][3] = v4_step(Lb, R[v][3], w.w, C);
          const uint32_t kn = k + P;
          buf[j][v] = __builtin_amdgcn_raw_buffer_load_b128(
              rs, CHK ? off(kn, v) : uint32_t(voff(kn, v)), 0, RDK_V4_AUX);
        }
      }
    };
    if (inpass) {
      uint32_t k0 = 0;
      for (; k0 < Kmax && (k0 <= khead || k0 + 2 * P > Kmax); k0 += P)
        block(k0, std::true_type{});
      for (; k0 + 2 * P <= Kmax; k0 += P) block(k0, std::false_type{});
      for (; k0 < Kmax; k0 += P) block(k0, std::true_type{});
    }
  }
  // combine each vector's four dword streams, then the vectors, place lane l, reduce
  uint32_t r = 0;
#if defined(RDK_V4_ABL) && RDK_V4_ABL == 1  // timing ablation only: skip the combine
  if (big) return R[0][0] ^ R[0][1] ^ R[NV - 1][2] ^ R[NV - 1][3];
#endif
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const uint32_t x = v4_z4(Lb, v4_z4(Lb, v4_z4(Lb, R[v][0]) ^ R[v][1]) ^ R[v][2]) ^ R[v][3];
    r = v ? v4_z256(Lb, r) ^ x : x;
  }
  r = row_xor(v4_fin(Lb, r, lc4));
  if (kV4Lanes == 32) r ^= __builtin_amdgcn_ds_swizzle(r, 0x401f);  // xor lane 16
  // fold the <16-byte tail [B, e) byte by byte (crc32c.c:131)
  if (big) {
    gbl_u8 *p = (gbl_u8 *)B;
    for (uint32_t i = 0, t = uint32_t(e - B); i < t; ++i) r = v4_t0(Lb, r, p[i]);
  }
  return r;
}

template <int V>
__device__ __forceinline__ uint32_t wave_crc_v(uintptr_t s, uintptr_t e, uint32_t init,
                                               bool inject, bool final, const lds_u32 *L,
                                               int lane) {
  if constexpr (V == 3) return wave_crc_v3(s, e, init, inject, final, lane);
  else return wave_crc(s, e, init, inject, final, L, lane);
}

template <int V> constexpr int crc_lds_words() { return V == 3 ? kCrcV3Words : kCrcTableWords; }

extern __shared__ __attribute__((aligned(16))) uint32_t crc_lds[];

__device__ __forceinline__ void load_tables(uint32_t *L, const uint32_t *g, int words) {
  const uint4 *src = reinterpret_cast<const uint4 *>(g);
  uint4 *dst = reinterpret_cast<uint4 *>(L);
  for (int i = threadIdx.x; i < words / 4; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

__device__ __forceinline__ uint32_t be32_at(const uint8_t *p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}

// ---- independent ranges ---------------------------------------------------
template <int V>
__global__ __launch_bounds__(crc_block<V>(), 8) void crc32c_ranges_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint32_t *__restrict__ lens, const uint32_t *__restrict__ init,
    uint32_t *__restrict__ out, uint32_t n, const uint32_t *__restrict__ gtab) {
  uint32_t *L = crc_lds;
  load_tables(L, gtab, crc_lds_words<V>());
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const lds_u32 *Lt = (const lds_u32 *)L;
  for (uint32_t i = wave; i < n; i += gridDim.x * wpb) {
    const uintptr_t s = reinterpret_cast<uintptr_t>(base) + offs[i];
    const uint32_t c0 = init ? init[i] : 0u;
    const uint32_t crc = wave_crc_v<V>(s, s + lens[i], c0, true, true, Lt, lane);
    if (lane == 0) out[i] = crc;
  }
}

// ---- one long range split into kCrcChunk chunks (raw registers) ------------
template <int V>
__global__ __launch_bounds__(crc_block<V>(), 8) void crc32c_chunks_kernel(
    const uint8_t *__restrict__ p, uint64_t len, uint32_t init, uint32_t *__restrict__ raw,
    uint32_t nchunks, const uint32_t *__restrict__ gtab) {
  uint32_t *L = crc_lds;
  load_tables(L, gtab, crc_lds_words<V>());
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const lds_u32 *Lt = (const lds_u32 *)L;
  for (uint32_t i = wave; i < nchunks; i += gridDim.x * wpb) {
    const uint64_t o = uint64_t(i) * kCrcChunk;
    const uint64_t l = (len - o < kCrcChunk) ? len - o : kCrcChunk;
    const uintptr_t s = reinterpret_cast<uintptr_t>(p) + o;
    const uint32_t r = wave_crc_v<V>(s, s + l, init, i == 0, false, Lt, lane);
    if (lane == 0) raw[i] = r;
  }
}

// multiply in GF(2)[x]/P, reflected (bit 31 = x^0)
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t m = 1u << 31, p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ poly : b >> 1;
  }
  return p;
}

// register advanced by `nbytes` zero bytes
__device__ uint32_t shift_bytes(uint32_t x, uint64_t nbytes, const uint32_t *x2n, uint32_t poly) {
  uint32_t p = 1u << 31;
  int k = 3;
  for (uint64_t n = nbytes; n; n >>= 1, ++k)
    if (n & 1u) p = multmodp(x2n[k], p, poly);
  return multmodp(p, x, poly);
}

__global__ void crc32c_combine_kernel(const uint32_t *__restrict__ raw, uint32_t nchunks,
                                      uint64_t len, uint32_t *__restrict__ out,
                                      const uint32_t *__restrict__ x2n, uint32_t poly) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t x = raw[0];
  for (uint32_t i = 1; i < nchunks; ++i) {
    const uint64_t o = uint64_t(i) * kCrcChunk;
    const uint64_t l = (len - o < kCrcChunk) ? len - o : kCrcChunk;
    x = shift_bytes(x, l, x2n, poly) ^ raw[i];
  }
  *out = ~x;
}

// ---- MsgVersion 2 record batches ------------------------------------------
template <int V, int MODE>
__global__ __launch_bounds__(crc_block<V>(), 8) void crc32c_msgset_v2_kernel(
    uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint32_t *__restrict__ caps, uint32_t *__restrict__ out, uint32_t n,
    const uint32_t *__restrict__ gtab) {
  uint32_t *L = crc_lds;
  load_tables(L, gtab, crc_lds_words<V>());
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const lds_u32 *Lt = (const lds_u32 *)L;
  for (uint32_t i = wave; i < n; i += gridDim.x * wpb) {
    uint8_t *hdr = base + offs[i];
    const uint32_t length = be32_at(hdr + 8);  // RD_KAFKAP_MSGSET_V2_OF_Length
    const uint32_t cap = caps[i];
    if (length < 9u || uint64_t(length) + 12u > cap) {  // crc_len = Length-4-1-4
      if (lane == 0) out[i] = (MODE == RDK_HIP_V2_CRC_VERIFY) ? 2u : 0u;
      continue;
    }
    const uintptr_t s = reinterpret_cast<uintptr_t>(hdr) + 21u;
    const uintptr_t e = reinterpret_cast<uintptr_t>(hdr) + 12u + length;
    const uint32_t crc = wave_crc_v<V>(s, e, 0u, true, true, Lt, lane);
    if (lane == 0) {
      if (MODE == RDK_HIP_V2_CRC_VERIFY) {
        out[i] = (be32_at(hdr + 17) == crc) ? 0u : 1u;
      } else {
        out[i] = crc;
        if (MODE == RDK_HIP_V2_CRC_FINALIZE) {  // rd_kafka_buf_update_i32 (BE)
          hdr[17] = uint8_t(crc >> 24);
          hdr[18] = uint8_t(crc >> 16);
          hdr[19] = uint8_t(crc >> 8);
          hdr[20] = uint8_t(crc);
        }
      }
    }
  }
}

// ---- v4 kernels: 16 waves x 4 groups = 64 ranges per workgroup round; the
// 148 KiB table image allows one workgroup per CU
constexpr int kV4Block = 1024;
constexpr int kV4Groups = kV4Block / kV4Lanes;

__device__ __forceinline__ void load_tables_v4(uint32_t *L, const uint32_t *g) {
  const uint4 *src = reinterpret_cast<const uint4 *>(g);
  uint4 *dst = reinterpret_cast<uint4 *>(L);
  for (int i = threadIdx.x; i < kCrcV4Words / 4; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

__global__ __launch_bounds__(kV4Block, 1) void crc32c_ranges_v4_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint32_t *__restrict__ lens, const uint32_t *__restrict__ init,
    uint32_t *__restrict__ out, uint32_t n, const uint32_t *__restrict__ gtab) {
  __shared__ __attribute__((aligned(16))) uint32_t L[kCrcV4Words];  // the kernel's only LDS: at 0
  load_tables_v4(L, gtab);
  const int lane = threadIdx.x & 63;
  const uint32_t grp = blockIdx.x * kV4Groups + (threadIdx.x / kV4Lanes);
  const uint32_t stride = gridDim.x * kV4Groups;
  // every wave runs the same number of rounds (uniform trip count)
  for (uint32_t i0 = blockIdx.x * kV4Groups; i0 < n; i0 += stride) {
    const uint32_t i = i0 - blockIdx.x * kV4Groups + grp;
    const bool active = i < n;
    uintptr_t s = 0, e = 0;
    uint32_t c0 = 0;
    if (active) {
      s = reinterpret_cast<uintptr_t>(base) + offs[i];
      e = s + lens[i];
      c0 = init ? init[i] : 0u;
    }
    const uint32_t crc = ~group_crc_v4(s, e, ~c0, active, lane, (const lds_u32 *)L);
    if (active && (lane & (kV4Lanes - 1)) == 0) out[i] = crc;
  }
}

template <int MODE>
__global__ __launch_bounds__(kV4Block, 1) void crc32c_msgset_v2_v4_kernel(
    uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint32_t *__restrict__ caps, uint32_t *__restrict__ out, uint32_t n,
    const uint32_t *__restrict__ gtab) {
  __shared__ __attribute__((aligned(16))) uint32_t L[kCrcV4Words];  // the kernel's only LDS: at 0
  load_tables_v4(L, gtab);
  const int lane = threadIdx.x & 63;
  const uint32_t grp = blockIdx.x * kV4Groups + (threadIdx.x / kV4Lanes);
  const uint32_t stride = gridDim.x * kV4Groups;
  // batch metadata is software-pipelined over the rounds: the offset two rounds ahead and
  // the Length word / capacity one round ahead are loaded before this round's CRC, so no
  // round starts with a chain of dependent loads (indices clamped: always valid addresses)
  typedef __attribute__((address_space(1))) const uint8_t gbl_u8;
  auto clampi = [&](uint32_t j) { return j < n ? j : n - 1u; };
  auto len_word = [&](uint64_t o) {
    gbl_u8 *p = (gbl_u8 *)(base + o + 8);  // RD_KAFKAP_MSGSET_V2_OF_Length (big-endian)
    return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
  };
  uint32_t i = grp;
  uint64_t o_nx = offs[clampi(i)];
  uint32_t len_nx = len_word(o_nx), cap_nx = caps[clampi(i)];
  uint64_t o_nx2 = offs[clampi(i + stride)];
  for (uint32_t i0 = blockIdx.x * kV4Groups; i0 < n; i0 += stride, i += stride) {
    const bool active = i < n;
    const uint64_t o = o_nx;
    const uint32_t length = len_nx, cap = cap_nx;
    o_nx = o_nx2;
    len_nx = len_word(o_nx);
    cap_nx = caps[clampi(i + stride)];
    o_nx2 = offs[clampi(i + 2 * stride)];
    uint8_t *hdr = base + o;
    const bool bad = length < 9u || uint64_t(length) + 12u > cap;  // crc_len = Length-4-1-4
    const uintptr_t s = reinterpret_cast<uintptr_t>(hdr) + 21u;
    const uintptr_t e = reinterpret_cast<uintptr_t>(hdr) + 12u + length;
    const uint32_t crc = ~group_crc_v4(s, e, ~0u, active && !bad, lane, (const lds_u32 *)L);
    if (active && (lane & (kV4Lanes - 1)) == 0) {
      if (bad) {
        out[i] = (MODE == RDK_HIP_V2_CRC_VERIFY) ? 2u : 0u;
      } else if (MODE == RDK_HIP_V2_CRC_VERIFY) {
        out[i] = (be32_at(hdr + 17) == crc) ? 0u : 1u;
      } else {
        out[i] = crc;
        if (MODE == RDK_HIP_V2_CRC_FINALIZE) {  // rd_kafka_buf_update_i32 (BE)
          hdr[17] = uint8_t(crc >> 24);
          hdr[18] = uint8_t(crc >> 16);
          hdr[19] = uint8_t(crc >> 8);
          hdr[20] = uint8_t(crc);
        }
      }
    }
  }
}

// ---- few large batches: split each CRC range into nch chunks (more work items than
// the CUs have group slots), raw CRCs per chunk, then one combine per batch with the
// GF(2) shift of crc32c.c:144-231 (multiply by x^(8*len) mod P)
__device__ __forceinline__ void v2_range(const uint8_t *hdr, uint32_t length, uint32_t cap,
                                         bool &bad, uintptr_t &s, uintptr_t &e) {
  bad = length < 9u || uint64_t(length) + 12u > cap;  // crc_len = Length-4-1-4
  s = reinterpret_cast<uintptr_t>(hdr) + 21u;
  e = reinterpret_cast<uintptr_t>(hdr) + 12u + length;
}
__device__ __forceinline__ uint32_t split_chunk(uint32_t len, uint32_t nch) {
  return (((len + nch - 1u) / nch) + 15u) & ~15u;
}

__global__ __launch_bounds__(kV4Block, 1) void crc32c_msgset_v2_split_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint32_t *__restrict__ caps, uint32_t n, uint32_t nch, uint32_t *__restrict__ raw,
    const uint32_t *__restrict__ gtab) {
  __shared__ __attribute__((aligned(16))) uint32_t L[kCrcV4Words];  // the kernel's only LDS: at 0
  load_tables_v4(L, gtab);
  const int lane = threadIdx.x & 63;
  const uint32_t items = n * nch;
  const uint32_t stride = gridDim.x * kV4Groups;
  uint32_t w = blockIdx.x * kV4Groups + (threadIdx.x / kV4Lanes);
  for (uint32_t w0 = blockIdx.x * kV4Groups; w0 < items; w0 += stride, w += stride) {
    const bool act = w < items;
    const uint32_t i = act ? w / nch : 0u, j = act ? w % nch : 0u;
    const uint8_t *hdr = base + offs[i];
    bool bad;
    uintptr_t s, e;
    v2_range(hdr, be32_at(hdr + 8), caps[i], bad, s, e);
    const uint32_t C = bad ? 0u : split_chunk(uint32_t(e - s), nch);
    const uintptr_t cs = s + uintptr_t(j) * C;
    const uintptr_t ce = cs + C < e ? cs + C : e;
    const bool on = act && !bad && (j == 0 || cs < e);  // an empty range keeps ~init
    // chunk 0 carries crc32c()'s initial register; the others are raw (zero) registers
    const uint32_t r = group_crc_v4(cs, on ? ce : cs, j == 0 ? ~0u : 0u, on, lane,
                                    (const lds_u32 *)L);
    if (act && (lane & (kV4Lanes - 1)) == 0) raw[w] = r;
  }
}

__device__ uint32_t xpow8n(uint64_t nbytes, const uint32_t *x2n) {  // x^(8*nbytes) mod P
  uint32_t p = 1u << 31;
  int k = 3;
  for (uint64_t n = nbytes; n; n >>= 1, ++k)
    if (n & 1u) p = multmodp(x2n[k], p, kCrcPoly);
  return p;
}

template <int MODE>
__global__ void crc32c_msgset_v2_combine_kernel(uint8_t *__restrict__ base,
                                                const uint64_t *__restrict__ offs,
                                                const uint32_t *__restrict__ caps, uint32_t n,
                                                uint32_t nch, const uint32_t *__restrict__ raw,
                                                uint32_t *__restrict__ out,
                                                const uint32_t *__restrict__ x2n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t *hdr = base + offs[i];
  bool bad;
  uintptr_t s, e;
  v2_range(hdr, be32_at(hdr + 8), caps[i], bad, s, e);
  if (bad) {
    out[i] = (MODE == RDK_HIP_V2_CRC_VERIFY) ? 2u : 0u;
    return;
  }
  const uint32_t len = uint32_t(e - s), C = split_chunk(len, nch);
  const uint32_t pc = xpow8n(C, x2n);
  uint32_t r = raw[size_t(i) * nch];
  for (uint32_t j = 1; j < nch && uint64_t(j) * C < len; ++j) {
    const uint32_t cl = (uint64_t(j + 1) * C <= len) ? C : len - j * C;
    r = multmodp(cl == C ? pc : xpow8n(cl, x2n), r, kCrcPoly) ^ raw[size_t(i) * nch + j];
  }
  const uint32_t crc = ~r;
  if (MODE == RDK_HIP_V2_CRC_VERIFY) {
    out[i] = (be32_at(hdr + 17) == crc) ? 0u : 1u;
  } else {
    out[i] = crc;
    if (MODE == RDK_HIP_V2_CRC_FINALIZE) {  // rd_kafka_buf_update_i32 (BE)
      hdr[17] = uint8_t(crc >> 24);
      hdr[18] = uint8_t(crc >> 16);
      hdr[19] = uint8_t(crc >> 8);
      hdr[20] = uint8_t(crc);
    }
  }
}

}  // namespace rdk

// ============================================================ host launchers
namespace rdk {

// 4 (default): batched kernels on 16-lane groups; RDK_HIP_CRC_V=3 / RDK_HIP_CRC_V1=1 select
// the earlier per-wave kernels (A/B measurements).  Single long ranges always use v3/v1.
static int crc_variant() {
  static const int v = [] {
    if (getenv("RDK_HIP_CRC_V1") && atoi(getenv("RDK_HIP_CRC_V1"))) return 1;
    const char *e = getenv("RDK_HIP_CRC_V");
    return e ? atoi(e) : 4;
  }();
  return v;
}

static unsigned crc_grid_v4(uint32_t n) {
  uint32_t blocks = (n + kV4Groups - 1) / kV4Groups;
  if (blocks > 256u) blocks = 256u;  // one resident workgroup per CU
  return blocks ? blocks : 1u;
}

template <int V> static unsigned crc_grid(uint32_t nwork) {
  const uint32_t wpb = crc_block<V>() / kWave;
  uint32_t blocks = (nwork + wpb - 1) / wpb;
  const uint32_t resident = V == 3 ? 2u * 256u : 4u * 256u;  // per-CU LDS residency x 256 CUs
  if (blocks > resident) blocks = resident;
  return blocks ? blocks : 1u;
}

template <int V> static const uint32_t *tabs(int dev, int kind = kCrcKind32C) {
  return V == 3 ? crc_tables_v3_dev(dev, kind) : crc_tables_dev(dev, kind);
}
template <int V> static size_t lds_bytes() { return size_t(crc_lds_words<V>()) * 4u; }

template <int V>
static void launch_chunks(Ctx *c, const uint8_t *d_buf, uint64_t len, uint32_t init,
                          uint32_t *d_scratch, uint32_t nchunks, hipStream_t s, int kind) {
  hipLaunchKernelGGL(crc32c_chunks_kernel<V>, dim3(crc_grid<V>(nchunks)), dim3(crc_block<V>()),
                     lds_bytes<V>(), s, d_buf, len, init, d_scratch, nchunks,
                     tabs<V>(c->device, kind));
}

// CRC32C of one device buffer (any length) -> d_scratch[nchunks] (device).
// Used by the drop-in crc32c()/rd_slice_crc32c() after the host gather + H2D.
// d_final: where the CRC itself goes (default: behind the chunk registers, d_scratch[nchunks]);
// it may be mapped host memory, which saves the caller a copy.  d_buf may be mapped host
// memory too: the chunk kernel passes over it once.
int crc_device_buffer(Ctx *c, const uint8_t *d_buf, uint64_t len, uint32_t init,
                      uint32_t *d_scratch /* >= nchunks+1 words */, hipStream_t s, int kind,
                      uint32_t *d_final) {
  const uint32_t nchunks = len ? uint32_t((len + kCrcChunk - 1) / kCrcChunk) : 1u;
  if (!d_final) d_final = d_scratch + nchunks;
  if (len == 0) {
    // crc32c(crc, buf, 0) == crc: inversions cancel (crc32c.c:102,133)
    RDK_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_final), init, 1, s));
    return 0;
  }
  if (crc_variant() != 1) launch_chunks<3>(c, d_buf, len, init, d_scratch, nchunks, s, kind);
  else launch_chunks<1>(c, d_buf, len, init, d_scratch, nchunks, s, kind);
  hipLaunchKernelGGL(crc32c_combine_kernel, dim3(1), dim3(64), 0, s, d_scratch, nchunks, len,
                     d_final, crc_x2n_dev(c->device, kind),
                     kind == kCrcKind32 ? kCrc32Poly : kCrcPoly);
  RDK_HIP_CHECK(hipGetLastError());
  return 0;
}

uint32_t crc_scratch_words(uint64_t len) {
  return (len ? uint32_t((len + kCrcChunk - 1) / kCrcChunk) : 1u) + 1u;
}

template <int V>
static void launch_ranges(Ctx *c, const void *d_base, const uint64_t *d_offs,
                          const uint32_t *d_lens, const uint32_t *d_init, uint32_t *d_out,
                          uint32_t n, hipStream_t s, int kind) {
  hipLaunchKernelGGL(crc32c_ranges_kernel<V>, dim3(crc_grid<V>(n)), dim3(crc_block<V>()),
                     lds_bytes<V>(), s, static_cast<const uint8_t *>(d_base), d_offs, d_lens,
                     d_init, d_out, n, tabs<V>(c->device, kind));
}

// n ranges of either polynomial (the kernels are polynomial-agnostic: they take the image)
static int ranges_any(const void *d_base, const uint64_t *d_offs, const uint32_t *d_lens,
                      const uint32_t *d_init, uint32_t *d_out, uint32_t n, void *stream,
                      int kind) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_base || !d_offs || !d_lens || !d_out) return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (crc_variant() == 4)
    hipLaunchKernelGGL(crc32c_ranges_v4_kernel, dim3(crc_grid_v4(n)), dim3(kV4Block), 0, s,
                       static_cast<const uint8_t *>(d_base), d_offs, d_lens, d_init, d_out, n,
                       crc_tables_v4_dev(c->device, kind));
  else if (crc_variant() == 3)
    launch_ranges<3>(c, d_base, d_offs, d_lens, d_init, d_out, n, s, kind);
  else
    launch_ranges<1>(c, d_base, d_offs, d_lens, d_init, d_out, n, s, kind);
  RDK_HIP_CHECK(hipGetLastError());
  return RDK_HIP_OK;
}

template <int V, int MODE>
static void launch_v2(Ctx *c, uint8_t *b, const uint64_t *offs, const uint32_t *caps,
                      uint32_t *out, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((crc32c_msgset_v2_kernel<V, MODE>), dim3(crc_grid<V>(n)),
                     dim3(crc_block<V>()), lds_bytes<V>(), s, b, offs, caps, out, n,
                     tabs<V>(c->device));
}

template <int MODE>
static int launch_v2_any(Ctx *c, uint8_t *b, const uint64_t *offs, const uint32_t *caps,
                         uint32_t *out, uint32_t n, hipStream_t s) {
  // fewer than 2 batches per group slot of the chip: split every range into chunks
  constexpr uint32_t kSlots = 256u * kV4Groups;
  if (crc_variant() == 4 && n <= kSlots / 2) {
    const uint32_t nch = std::min(64u, kSlots / n);
    // at most kSlots partial registers (64 KiB), private to this thread and stream
    static_assert(size_t(kSlots) * 4 <= 65536, "crc_scratch() holds 64 KiB");
    uint32_t *raw = crc_scratch(c, s);
    if (!raw) return RDK_HIP_E_NOMEM;
    const uint32_t items = n * nch;
    hipLaunchKernelGGL(crc32c_msgset_v2_split_kernel, dim3(crc_grid_v4(items)), dim3(kV4Block),
                       0, s, b, offs, caps, n, nch, raw, crc_tables_v4_dev(c->device));
    hipLaunchKernelGGL(crc32c_msgset_v2_combine_kernel<MODE>, dim3((n + 63) / 64), dim3(64), 0,
                       s, b, offs, caps, n, nch, raw, out, crc_x2n_dev(c->device));
    RDK_HIP_CHECK(hipGetLastError());
    return RDK_HIP_OK;
  } else if (crc_variant() == 4)
    hipLaunchKernelGGL(crc32c_msgset_v2_v4_kernel<MODE>, dim3(crc_grid_v4(n)), dim3(kV4Block), 0,
                       s, b, offs, caps, out, n, crc_tables_v4_dev(c->device));
  else if (crc_variant() == 3) launch_v2<3, MODE>(c, b, offs, caps, out, n, s);
  else launch_v2<1, MODE>(c, b, offs, caps, out, n, s);
  RDK_HIP_CHECK(hipGetLastError());
  return RDK_HIP_OK;
}

}  // namespace rdk

using namespace rdk;

RDK_API int rdk_hip_crc32c_ranges(const void *d_base, const uint64_t *d_offs,
                                  const uint32_t *d_lens, const uint32_t *d_init,
                                  uint32_t *d_out, uint32_t n, void *stream) {
  return ranges_any(d_base, d_offs, d_lens, d_init, d_out, n, stream, kCrcKind32C);
}

RDK_API int rdk_hip_crc32_ranges(const void *d_base, const uint64_t *d_offs,
                                 const uint32_t *d_lens, const uint32_t *d_init,
                                 uint32_t *d_out, uint32_t n, void *stream) {
  return ranges_any(d_base, d_offs, d_lens, d_init, d_out, n, stream, kCrcKind32);
}

RDK_API int rdk_hip_msgset_v2_crc(void *d_base, const uint64_t *d_batch_offs,
                                  const uint32_t *d_batch_caps, uint32_t *d_out, uint32_t n,
                                  int mode, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_base || !d_batch_offs || !d_batch_caps || !d_out)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t *b = static_cast<uint8_t *>(d_base);
  switch (mode) {
    case RDK_HIP_V2_CRC_COMPUTE:
      return launch_v2_any<RDK_HIP_V2_CRC_COMPUTE>(c, b, d_batch_offs, d_batch_caps, d_out, n, s);
    case RDK_HIP_V2_CRC_FINALIZE:
      return launch_v2_any<RDK_HIP_V2_CRC_FINALIZE>(c, b, d_batch_offs, d_batch_caps, d_out, n, s);
    case RDK_HIP_V2_CRC_VERIFY:
      return launch_v2_any<RDK_HIP_V2_CRC_VERIFY>(c, b, d_batch_offs, d_batch_caps, d_out, n, s);
    default:
      return set_error(RDK_HIP_E_INVAL, "bad mode %d", mode);
  }
}
