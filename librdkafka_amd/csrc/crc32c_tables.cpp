// crc32c_tables.cpp -- see crc32c_tables.h.
#include "crc32c_tables.h"

#include <cstring>

namespace rdk {

uint32_t crc_gf2_times(const uint32_t mat[32], uint32_t vec) {
  uint32_t s = 0;
  for (int i = 0; vec; ++i, vec >>= 1)
    if (vec & 1u) s ^= mat[i];
  return s;
}

static void gf2_compose(uint32_t dst[32], const uint32_t a[32], const uint32_t b[32]) {
  // dst = a o b (apply b, then a)
  uint32_t r[32];
  for (int i = 0; i < 32; ++i) r[i] = crc_gf2_times(a, b[i]);
  std::memcpy(dst, r, sizeof r);
}

// Operator appending `nbytes` zero bytes to a raw (un-inverted) CRC register.
// Column i = image of register bit i.  One zero BIT maps bit 0 -> poly and
// bit i -> bit i-1 (reflected shift), as in crc32c_zeros_op (crc32c.c:173).
void crc_zeros_operator(uint32_t op[32], size_t nbytes, uint32_t poly) {
  uint32_t p[32];
  p[0] = poly;
  for (int i = 1; i < 32; ++i) p[i] = 1u << (i - 1);
  for (int k = 0; k < 3; ++k) gf2_compose(p, p, p);  // 1 bit -> 8 bits
  for (int i = 0; i < 32; ++i) op[i] = 1u << i;        // identity
  while (nbytes) {
    if (nbytes & 1u) gf2_compose(op, p, op);
    nbytes >>= 1;
    if (nbytes) gf2_compose(p, p, p);
  }
}

void crc_build_tables(uint32_t *out, uint32_t poly) {
  // byte-wise table, then slicing extension (crc32c.c:69-92 generalised to 16)
  uint32_t *T = out;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t r = b;
    for (int i = 0; i < 8; ++i) r = (r >> 1) ^ ((r & 1u) ? poly : 0u);
    T[b] = r;
  }
  for (int k = 1; k < kCrcSliceTables; ++k)
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t r = T[(k - 1) * 256 + b];
      T[k * 256 + b] = T[r & 0xffu] ^ (r >> 8);
    }
  // shift operators for 32..1024 bytes, split per state byte
  for (int level = 1; level <= 6; ++level) {
    uint32_t op[32];
    crc_zeros_operator(op, size_t(16) << level, poly);
    uint32_t *S = out + crc_shift_table(level) * 256;
    for (int j = 0; j < 4; ++j)
      for (uint32_t b = 0; b < 256; ++b) S[j * 256 + b] = crc_gf2_times(op, b << (8 * j));
  }
}

void crc_build_tables_v3(uint32_t *out, uint32_t poly) {
  std::memset(out, 0, size_t(kCrcV3Bytes));
  uint32_t op[32];
  for (int map = 0; map < 2; ++map) {
    crc_zeros_operator(op, map == 0 ? size_t(kLaneStride - 12) : size_t(4), poly);
    for (int j = 0; j < 4; ++j)      // rotation y_j = rotr(x, 8j)
      for (int h = 0; h < 2; ++h)    // group at bits 7+4h .. 10+4h of y_j
        for (uint32_t e = 0; e < 16; ++e) {
          const uint32_t y = e << (7 + 4 * h);
          const uint32_t x = (j == 0) ? y : ((y << (8 * j)) | (y >> (32 - 8 * j)));
          const uint32_t v = crc_gf2_times(op, x);
          const int t = map * 4 + j;
          for (int c = 0; c < 32; ++c) {
            const int byte = h == 0 ? kV3S7 + t * 2048 + int(e) * 128 + c * 4
                                    : kV3S11 + t * 128 + int(e) * 2048 + c * 4;
            out[byte / 4] = v;
          }
        }
  }
  for (int m = 0; m < 6; ++m) {  // merge tree: advance by 16 << m bytes
    crc_zeros_operator(op, size_t(16) << m, poly);
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b)
        out[v3_byte_table(m * 4 + q) / 4 + int(b)] = crc_gf2_times(op, b << (8 * q));
  }
  for (uint32_t b = 0; b < 256; ++b) {  // T0 (crc32c.c:69-78)
    uint32_t r = b;
    for (int i = 0; i < 8; ++i) r = (r >> 1) ^ ((r & 1u) ? poly : 0u);
    out[v3_byte_table(kV3T0) / 4 + int(b)] = r;
  }
}

void crc_build_tables_v4(uint32_t *out, uint32_t poly) {
  std::memset(out, 0, size_t(kCrcV4Bytes));
  uint32_t op[32];
  crc_zeros_operator(op, size_t(kV4Step), poly);
  for (int q = 0; q < 4; ++q)
    for (uint32_t b = 0; b < 256; ++b) {
      const uint32_t v = crc_gf2_times(op, b << (8 * q));
      for (int c = 0; c < 32; ++c)
        out[((q >> 1) * 0x10000 + int(b) * 256 + (q & 1) * 128 + c * 4) / 4] = v;
    }
  for (int l = 0; l < kV4Lanes; ++l) {  // Fin: group lane l's last dword stream ends
    crc_zeros_operator(op, size_t(kV4Row - 16 * l - 12), poly);  // kV4Row-16l-12 bytes early
    for (int i = 0; i < 8; ++i)
      for (uint32_t n = 0; n < 16; ++n) {
        const uint32_t v = crc_gf2_times(op, n << (4 * i));
        for (int c = l; c < 32; c += kV4Lanes) out[(kV4Fin + i * 2048 + int(n) * 128 + c * 4) / 4] = v;
      }
  }
  crc_zeros_operator(op, 4, poly);
  for (int q = 0; q < 4; ++q)
    for (uint32_t b = 0; b < 256; ++b)
      out[(kV4Z4 + q * 1024) / 4 + int(b)] = crc_gf2_times(op, b << (8 * q));
  crc_zeros_operator(op, size_t(kV4Row), poly);
  for (int q = 0; q < 4; ++q)
    for (uint32_t b = 0; b < 256; ++b)
      out[(kV4Z256 + q * 1024) / 4 + int(b)] = crc_gf2_times(op, b << (8 * q));
}

// x2n[k] = x^(2^k) mod P in reflected form (bit 31 = x^0), for the
// multiply-mod-P shift used when combining ranges of arbitrary length.
uint32_t crc_multmodp(uint32_t a, uint32_t b, uint32_t poly) {
  if (!a) return 0;  // the loop below ends at a's lowest set bit
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ poly : b >> 1;
  }
  return p;
}

void crc_build_x2n(uint32_t *out, uint32_t poly) {
  uint32_t p = 1u << 30;  // x^1
  out[0] = p;
  for (int k = 1; k < 64; ++k) out[k] = p = crc_multmodp(p, p, poly);
}

void crc_build_x2n_dev(uint32_t *out, uint32_t poly) {
  crc_build_x2n(out, poly);
  uint32_t p = 1u << 31;  // x^0
  for (int i = 0; i < kXLoN; ++i, p = crc_multmodp(p, out[3], poly)) out[kXLo + i] = p;        // * x^8
  p = 1u << 31;
  for (int i = 0; i < kXHiN; ++i, p = crc_multmodp(p, out[13], poly)) out[kXHi + i] = p;       // * x^(8 * 1024)
}

// x^(8 * nbytes) mod P from the x2n table (bit k of the bit count selects x2n[k])
uint32_t crc_x_pow_bytes(const uint32_t x2n[64], uint64_t nbytes, uint32_t poly) {
  uint32_t p = 1u << 31;  // x^0
  for (int k = 3; nbytes; nbytes >>= 1, ++k)
    if (nbytes & 1u) p = crc_multmodp(x2n[k], p, poly);
  return p;
}

}  // namespace rdk
