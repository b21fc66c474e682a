// crc_wave.h -- CRC32C of a byte range by ONE wavefront, for the compress epilogue.
//
// rd_kafka_msgset_writer_calc_crc_v2 (rdkafka_msgset_writer.c:1229-1246) runs over the
// finished batch after compression.  Here the CRC is taken by the wave that has just written
// the bytes (they are still in its L2): of the whole batch when it is a single block, else of
// every compressed block as a RAW register (zero initial value, no final inversion: then the
// CRC is GF(2)-linear in the data, leading zero bytes do not matter and pieces combine by
// shifting, crc32c.c:144-231), which the frame assembler combines with header and end mark
// into the batch's CRC.
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

// The same with the power looked up (x2n is the device table, whose two byte-power tables
// follow the 64 squarings, crc32c_tables.h): two loads and two multiplications for any count
// below 4 MiB, where the loop above multiplies once per set bit of the count.
__device__ __forceinline__ uint32_t crcw_shift_lut(uint32_t r, uint32_t nbytes,
                                                   const uint32_t *__restrict__ x2n) {
  static_assert(kXLoN == 1024, "the split below is at bit 10");
  if (nbytes >= uint32_t(kXLoN) * uint32_t(kXHiN)) return crcw_shift(r, nbytes, x2n);
  const uint32_t lo = x2n[kXLo + (nbytes & uint32_t(kXLoN - 1))], hi = x2n[kXHi + (nbytes >> 10)];
  return crcw_mul(crcw_mul(lo, hi), r);
}

// ---- the range itself, by dwords: four byte tables (T[k][b] = raw CRC of byte b followed by
// k zero bytes, k = 0..3: the first 1024 words of the slicing image) in LDS, one lookup each
// per dword (crc32c.c:301-336 is the same recurrence, eight bytes at a time).

// 1024 dwords of T[0..3] into LDS, by one wave
__device__ __forceinline__ void crcw_load_t4(crcw_lds_u32 *t4, const uint32_t *__restrict__ tabs,
                                             int lane) {
#pragma unroll
  for (int j = 0; j < 16; ++j) t4[lane + 64 * j] = tabs[lane + 64 * j];
  asm volatile("" ::: "memory");
}

// CRC32C register (no final inversion) over the `len` bytes at `addr`, whole wave; `ones`:
// the register starts as all ones (crc32c()'s initial value), else as zero (a raw register,
// which combines by shifting).  The result is wave-uniform.
//
// The bytes up to the last multiple of 16 are laid out RIGHT-aligned over 64 pieces of
// P = 2^e bytes, one per lane: zero bytes in front of the data leave a zero register alone,
// so the pad in front costs nothing, every piece ends a multiple of P from the end, the
// pieces combine in a shift-and-xor scan whose operators x^(8P*2^j) are entries of the x2n
// table (no multiplication to find them), and no short last piece needs a shift of its own.
// The pad is a multiple of 16, so no 16-byte fetch straddles the data's first byte (a vector
// load that starts below a resource reads as zero as a whole).  An all-ones start is the
// same as inverting the first four data bytes.  The last len % 16 bytes, one per lane, go
// through the byte table behind the combined register.
__device__ __forceinline__ uint32_t wave_crc_range(uintptr_t addr, uint32_t len, bool ones,
                                                   const crcw_lds_u32 *t4,
                                                   const uint32_t *__restrict__ x2n, int lane) {
  const uint32_t len16 = len & ~15u;
  uint32_t r = ones ? ~0u : 0u;
  if (len16) {
    const uint32_t need = (len16 + 63u) / 64u;
    const uint32_t e = need <= 16u ? 4u : 32u - uint32_t(__builtin_clz(need - 1u));  // P = 2^e >= 16
    const uint32_t P = 1u << e;
    const uint32_t pad = 64u * P - len16;
    const int start = int(uint32_t(lane) << e) - int(pad);  // of this lane's piece; a multiple of 16
    const uint32_t sa = uint32_t(addr & 3u);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(addr - sa), 0, int((sa + len16 + 3u) & ~3u), 0x00020000);
    // the dword that holds data bytes 0..3: lane pad >> e, dword (pad % P) / 4 of its piece
    const uint32_t dseed = (ones && uint32_t(lane) == (pad >> e)) ? (pad & (P - 1u)) >> 2 : ~0u;
    typedef uint32_t crcw_u4 __attribute__((ext_vector_type(4)));
    // (offsets below the data wrap to far beyond the resource and read as zero; the dword
    // behind such a vector may be the resource's first and is not used: `in`)
    const uint32_t v0 = uint32_t(start);
    uint32_t reg = 0;
    crcw_u4 na = __builtin_amdgcn_raw_buffer_load_b128(rs, v0, 0, 0);
    uint32_t nb = __builtin_amdgcn_raw_buffer_load_b32(rs, v0 + 16u, 0, 0);
    for (uint32_t k = 0; k < P; k += 16u) {
      const crcw_u4 a = na;
      const uint32_t ee = nb;
      na = __builtin_amdgcn_raw_buffer_load_b128(rs, v0 + k + 16u, 0, 0);
      nb = __builtin_amdgcn_raw_buffer_load_b32(rs, v0 + k + 32u, 0, 0);
      const bool in = start + int(k) >= 0;
      const uint32_t w[4] = {__builtin_amdgcn_alignbyte(a.y, a.x, sa), __builtin_amdgcn_alignbyte(a.z, a.y, sa),
                             __builtin_amdgcn_alignbyte(a.w, a.z, sa), __builtin_amdgcn_alignbyte(ee, a.w, sa)};
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) {
        uint32_t x = in ? w[j] : 0u;
        if ((k >> 2) + j == dseed) x = ~x;
        x ^= reg;
        reg = t4[768u + (x & 0xFFu)] ^ t4[512u + ((x >> 8) & 0xFFu)] ^ t4[256u + ((x >> 16) & 0xFFu)] ^
              t4[x >> 24];
      }
    }
    // S(L) = sum over l <= L of reg_l * X^(L-l), X = x^(8P); the whole range at lane 63
#pragma unroll 1
    for (uint32_t j = 0; j < 6u; ++j) {
      const int d = 1 << j;
      const uint32_t t = uint32_t(__shfl_up(int(reg), d));
      const uint32_t m = crcw_mul(t, x2n[3u + e + j]);  // (the operator is wave-uniform: its powers run on the scalar unit)
      if (lane >= d) reg ^= m;
    }
    r = uint32_t(__builtin_amdgcn_readlane(int(reg), 63));
  }
  const uint32_t tail = len - len16;  // < 16
  if (tail) {
    const uint32_t tb = ldb(addr + len16 + (uint32_t(lane) < tail ? uint32_t(lane) : tail - 1u));
    for (uint32_t i = 0; i < tail; ++i)
      r = t4[(r ^ uint32_t(__builtin_amdgcn_readlane(int(tb), int(i)))) & 0xFFu] ^ (r >> 8);
  }
  return r;
}

}  // namespace rdk
