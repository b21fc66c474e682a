// crc32c_tables.h -- host-side GF(2) algebra for CRC32C (reflected poly
// 0x82f63b78, src/crc32c.c:63) and the LDS table image used by the kernels.
//
// The reference builds a [8][256] slicing table (crc32c.c:69-92) and two
// [4][256] "zeros operator" tables for 8 KiB / 256 B shifts (crc32c.c:173-252).
// The MI355X kernels need: 16 slicing tables (one 16-byte vector per lane),
// and shift-by-{32,64,...,1024}-bytes operators for the lane-interleaved
// layout and the 64-lane merge tree.  All are generated here from one GF(2)
// "append n zero bytes" operator.
#pragma once

#include <cstddef>
#include <cstdint>

namespace rdk {

constexpr uint32_t kCrcPoly = 0x82f63b78u;

// LDS image layout (40 tables x 256 u32 = 40 KiB):
//   tables 0..15   : T[k][b] = raw CRC of byte b followed by k zero bytes
//   tables 16..39  : shift operators, 4 tables each (one per state byte) for
//                    32, 64, 128, 256, 512, 1024 bytes.  shift-by-16 is T[15-j].
constexpr int kCrcSliceTables = 16;
constexpr int kCrcShiftBase = 16;
constexpr int kCrcNumTables = 40;
constexpr int kCrcTableWords = kCrcNumTables * 256;
// index of the first of the 4 tables for shift-by-(16 << level), level 1..6
constexpr int crc_shift_table(int level) { return kCrcShiftBase + 4 * (level - 1); }

void crc_build_tables(uint32_t *out /* kCrcTableWords */);
void crc_build_x2n(uint32_t *out /* 64 */);

// Host GF(2) helpers (also used by unit tests through the engine API).
uint32_t crc_gf2_times(const uint32_t mat[32], uint32_t vec);
void crc_zeros_operator(uint32_t op[32], size_t nbytes);

}  // namespace rdk
