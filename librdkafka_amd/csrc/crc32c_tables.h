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
// CRC-32 (IEEE 802.3, zlib crc32()): MsgVersion 0/1 messages (rdcrc32.h:93-131 with
// WITH_ZLIB).  Same reflected register, init and final inversion, other polynomial: every
// image below is built for either polynomial and the kernels take the image they are given.
constexpr uint32_t kCrc32Poly = 0xedb88320u;

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

void crc_build_tables(uint32_t *out /* kCrcTableWords */, uint32_t poly = kCrcPoly);

// ---- v3 image (default): rotated-nibble tables, conflict-free and 1-VALU addresses
// A 32->32 GF(2)-linear map F (the CRC register advanced over n zero bytes) is
// evaluated as the xor of 8 lookups, one per 4-bit group of its input x.  The
// groups are bits [7..10] and [11..14] of y_j = rotr(x, 8j), j = 0..3, so each
// lookup address is a single v_and_or_b32: (y_j & 0x780 | lc4) for "S7" tables
// (16 entries x 32 copies, entry stride 128 B) or (y_j & 0x7800 | lc4) for
// "S11" tables (entry stride 2 KiB; 16 of them interleave in one 32 KiB region,
// table slot at bits 7..10 comes from the ds_read immediate offset).  lc4 =
// 4*(lane%32): each 32-lane ds_read_b32 group hits 32 distinct banks.
// Two maps are stored: M_1012 (map 0: the 1008-byte lane gap + one word) and
// M_4 (map 1: one 4-byte word), which is all a lane's Horner update needs:
//   u = M_1012(u) ^ w.x; u = M_4(u) ^ w.y; u = M_4(u) ^ w.z; u = M_4(u) ^ w.w.
// The unused slots 8..15 of the S11 region (1 KiB contiguous per entry row)
// hold 16 of the 25 byte tables (6x4 merge-tree operators + T0).
constexpr int kV3S11 = 0;                       // bytes; slot t at +128*t, entry e at +2048*e
constexpr int kV3S7 = 32768;                    // bytes; table t at +2048*t, entry e at +128*e
constexpr int kV3ByteHi = 49152;                // byte tables 16..24
constexpr int kV3NumByteTables = 25;            // tree (m*4+q, m=0..5), T0 = 24
constexpr int kV3T0 = 24;
constexpr int kCrcV3Bytes = kV3ByteHi + 9 * 1024;  // 58368 B = 57 KiB
constexpr int kCrcV3Words = kCrcV3Bytes / 4;
constexpr int kLaneStride = 1024;               // bytes between a lane's vectors
// byte offset of byte table i (256 dwords, contiguous)
constexpr int v3_byte_table(int i) { return i < 16 ? i * 2048 + 1024 : kV3ByteHi + (i - 16) * 1024; }
void crc_build_tables_v3(uint32_t *out /* kCrcV3Words */, uint32_t poly = kCrcPoly);
void crc_build_x2n(uint32_t *out /* 64 */, uint32_t poly = kCrcPoly);
// The device copy of the x2n table carries two more tables behind its 64 words, so that a
// kernel finds x^(8n) for a byte count n < 4 MiB with two loads and one multiplication
// instead of one multiplication per set bit of n:
//   [kXLo + i]  = x^(8 * i),         i < kXLoN
//   [kXHi + i]  = x^(8 * kXLoN * i), i < kXHiN
constexpr int kXLo = 64, kXLoN = 1024, kXHi = kXLo + kXLoN, kXHiN = 4096;
constexpr int kX2nDevWords = kXHi + kXHiN;
void crc_build_x2n_dev(uint32_t *out /* kX2nDevWords */, uint32_t poly = kCrcPoly);

// ---- v4 image (batched ranges / MsgVersion 2 kernels): 16-lane groups, byte tables
// A 16-lane group CRCs one range.  Per step the group reads kV4Vecs x 256 contiguous bytes:
// lane l owns the 16-byte vectors at V + kV4Step*k + 256v + 16l (v < kV4Vecs) and runs
// 4*kV4Vecs Horner streams, one per dword slot, all with the same map Z_kV4Step ("advance
// kV4Step zero bytes"): R = Z(R) ^ w.  Z is 4 byte tables (one per input byte q),
// 32-fold replicated (copy c = lane % 32 -> bank c, conflict-free), in two 64 KiB halves
// h = q >> 1 with the two tables t = q & 1 of a half interleaved per entry:
//   address = h*0x10000 + b*256 + t*128 + 4c
// so that ONE v_perm_b32 builds an address from the register byte b and a per-lane
// constant holding 4c, 4c|0x80 and 0x01 (kernel: v4_sel).  End of a range: each vector's
// four streams combine through Z_4, the vectors through Z_256 (both unreplicated byte
// tables; T0 = Z_4's table 3), then lane l's register is advanced by Z_{244-16l} -- "Fin",
// nibble tables whose copy c holds the map of group lane c % 16 -- and the 16 lanes
// xor-reduce inside their DPP row.
#ifndef RDK_V4_LANES
#define RDK_V4_LANES 16
#endif
constexpr int kV4Lanes = RDK_V4_LANES;          // lanes per group (one range): 16 or 32
constexpr int kV4Row = 16 * kV4Lanes;           // bytes of one group vector row
#ifndef RDK_V4_VECS
#define RDK_V4_VECS 2
#endif
constexpr int kV4Vecs = RDK_V4_VECS;            // 16-byte vectors per lane per step
constexpr int kV4Step = kV4Row * kV4Vecs;       // bytes between a lane's steps
constexpr int kV4Main = 0;
constexpr int kV4Fin = 0x20000;                 // nibble i at +2048*i, entry n at +128*n
constexpr int kV4Z4 = 0x24000;                  // byte table q at +1024*q
constexpr int kV4T0 = kV4Z4 + 3 * 1024;
constexpr int kV4Z256 = 0x25000;                // Z_kV4Row: byte table q at +1024*q
constexpr int kCrcV4Bytes = kV4Z256 + 4 * 1024; // 155648 B = 152 KiB (one workgroup per CU)
constexpr int kCrcV4Words = kCrcV4Bytes / 4;
void crc_build_tables_v4(uint32_t *out /* kCrcV4Words */, uint32_t poly = kCrcPoly);

// Host GF(2) helpers (also used by unit tests through the engine API).
uint32_t crc_gf2_times(const uint32_t mat[32], uint32_t vec);
void crc_zeros_operator(uint32_t op[32], size_t nbytes, uint32_t poly = kCrcPoly);
// a * b mod P, reflected form (bit 31 = x^0); x^(8 * nbytes) mod P from a crc_build_x2n
// table.  With them crc(init, A || B) == crc(0, B) ^ crc(init, A) * x^(8|B|): partial CRCs
// of the pieces of a buffer combine on the host.
uint32_t crc_multmodp(uint32_t a, uint32_t b, uint32_t poly = kCrcPoly);
uint32_t crc_x_pow_bytes(const uint32_t x2n[64], uint64_t nbytes, uint32_t poly = kCrcPoly);

}  // namespace rdk
