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

// ---- v2 image (default): bank-conflict-free nibble tables -----------------
// A byte lookup T[b] = N_lo[b & 15] ^ N_hi[b >> 4] (the tables are linear over
// GF(2)).  Each 16-entry nibble table is stored 32 times, entry e of copy c at
// dword e*32 + c, and lane l reads copy l%32: every lane of a 32-lane
// ds_read_b32 group hits its own bank, so a lookup costs 2 LDS cycles instead
// of the ~6.3 measured for random byte-table reads (profiles/).
constexpr int kNibCopies = 32;
constexpr int kNibTable = 16 * kNibCopies;           // dwords per nibble table
constexpr int kNibSlice = 0;                          // 16 tables: T_k (k=0..7) lo/hi -> 2k+hi
constexpr int kNibShift = 16 * kNibTable;             // 8 tables: shift-1008 of register nibble j
constexpr int kV2ByteT0 = 24 * kNibTable;             // byte table T0 (tail / short ranges)
constexpr int kV2Tree = kV2ByteT0 + 256;              // shift 16<<m, m=0..5: 4 byte tables each
constexpr int kCrcV2Words = kV2Tree + 6 * 4 * 256;    // 18688 dwords = 73 KiB
constexpr int kLaneStride = 1024;                     // bytes between a lane's vectors
void crc_build_tables_v2(uint32_t *out /* kCrcV2Words */);
void crc_build_x2n(uint32_t *out /* 64 */);

// Host GF(2) helpers (also used by unit tests through the engine API).
uint32_t crc_gf2_times(const uint32_t mat[32], uint32_t vec);
void crc_zeros_operator(uint32_t op[32], size_t nbytes);

}  // namespace rdk
