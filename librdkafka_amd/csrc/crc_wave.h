// crc_wave.h -- CRC32C of a byte range by ONE wavefront, for the compress epilogue.
//
// rd_kafka_msgset_writer_calc_crc_v2 (rdkafka_msgset_writer.c:1229-1246) runs over the
// finished batch after compression.  Here every compressed block's CRC is taken by the
// wave that has just written it (the bytes are still in its L2), as a RAW register
// (zero initial value, no final inversion: then the CRC is GF(2)-linear in the data,
// leading zero bytes do not matter and pieces combine by shifting, crc32c.c:144-231), and
// the frame assembler combines header, blocks and end mark into the batch's CRC.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "crc32c_tables.h"
#include "lz4_device.h"

namespace rdk {

typedef __attribute__((address_space(3))) uint32_t crcw_lds_u32;

// multiply in GF(2)[x]/P, reflected (bit 31 = x^0)
__device__ __forceinline__ uint32_t crcw_mul(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
#pragma unroll 4
  for (int i = 0; i < 32; ++i) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

// x^(8*nbytes) mod P from the x^(2^k) table (k = 0..63)
__device__ __forceinline__ uint32_t crcw_xpow8n(uint32_t nbytes, const uint32_t *__restrict__ x2n) {
  uint32_t p = 1u << 31;
  int k = 3;
  for (uint32_t n = nbytes; n; n >>= 1, ++k)
    if (n & 1u) p = crcw_mul(x2n[k], p);
  return p;
}

// the raw register advanced over nbytes zero bytes
__device__ __forceinline__ uint32_t crcw_shift(uint32_t r, uint32_t nbytes,
                                               const uint32_t *__restrict__ x2n) {
  return nbytes ? crcw_mul(crcw_xpow8n(nbytes, x2n), r) : r;
}

// 256 dwords of the byte table T0 (raw CRC of one byte) into LDS, by one wave
__device__ __forceinline__ void crcw_load_t0(crcw_lds_u32 *t0, const uint32_t *__restrict__ tabs,
                                             int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) t0[lane + 64 * j] = tabs[lane + 64 * j];
  asm volatile("" ::: "memory");
}

// Raw CRC32C register (zero in, no inversion) of the `len` bytes at `addr`, whole wave;
// the result is wave-uniform.  Lane l takes piece l of P = ceil(len/64) bytes counted from
// the start (q full pieces, one of `rem` bytes, the rest empty), byte by byte through T0.
// The bytes come as aligned dwords through a range-checked resource (reads past the end
// return 0), 16 per step on unconditional loads, the next step's issued before this step's
// table chain -- a load under a lane predicate would be waited for at once, one memory
// round trip per byte.  The full pieces' registers combine in a shift-and-xor scan; the
// short piece follows behind a shift by its length.
__device__ __forceinline__ uint32_t wave_crc_raw(uintptr_t addr, uint32_t len,
                                                 const crcw_lds_u32 *t0,
                                                 const uint32_t *__restrict__ x2n, int lane) {
  if (!len) return 0u;
  const uint32_t P = (len + 63u) / 64u;
  const uint32_t q = len / P, rem = len - q * P;  // 1 <= q <= 64
  const uint32_t start = uint32_t(lane) * P;
  const uint32_t mine = start >= len ? 0u : (len - start < P ? len - start : P);
  const uint32_t sa = uint32_t(addr & 3u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void *>(addr - sa), 0, int((sa + len + 3u) & ~3u), 0x00020000);
  typedef uint32_t crcw_u4 __attribute__((ext_vector_type(4)));
  const uint32_t v0 = start + sa, sh = v0 & 3u;
  uint32_t r = 0;
  crcw_u4 na = __builtin_amdgcn_raw_buffer_load_b128(rs, v0 & ~3u, 0, 0);
  uint32_t nb = __builtin_amdgcn_raw_buffer_load_b32(rs, (v0 & ~3u) + 16u, 0, 0);
  for (uint32_t k = 0; k < P; k += 16u) {
    const crcw_u4 a = na;
    const uint32_t e = nb;
    na = __builtin_amdgcn_raw_buffer_load_b128(rs, ((v0 + k) & ~3u) + 16u, 0, 0);
    nb = __builtin_amdgcn_raw_buffer_load_b32(rs, ((v0 + k) & ~3u) + 32u, 0, 0);
    const uint32_t w[4] = {__builtin_amdgcn_alignbyte(a.y, a.x, sh), __builtin_amdgcn_alignbyte(a.z, a.y, sh),
                           __builtin_amdgcn_alignbyte(a.w, a.z, sh), __builtin_amdgcn_alignbyte(e, a.w, sh)};
#pragma unroll
    for (uint32_t j = 0; j < 16u; ++j) {
      const uint32_t byte = (w[j >> 2] >> (8u * (j & 3u))) & 0xFFu;
      const uint32_t nr = t0[(r ^ byte) & 0xFFu] ^ (r >> 8);
      r = k + j < mine ? nr : r;
    }
  }
  // S(L) = sum over l <= L of r_l * X^(L-l), X = x^(8P): the full pieces, at lane q-1
  uint32_t X = uint32_t(__builtin_amdgcn_readfirstlane(int(crcw_xpow8n(P, x2n))));  // x^(8P)
  const uint32_t r_short = uint32_t(__builtin_amdgcn_readlane(int(r), int(q & 63u)));  // (rem == 0: unused)
  if (uint32_t(lane) >= q) r = 0;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = uint32_t(__shfl_up(int(r), d));
    const uint32_t m = crcw_mul(X, t);
    if (lane >= d) r ^= m;
    X = crcw_mul(X, X);
  }
  const uint32_t full = uint32_t(__builtin_amdgcn_readlane(int(r), int(q - 1u)));
  return rem ? crcw_shift(full, rem, x2n) ^ r_short : full;
}

}  // namespace rdk
