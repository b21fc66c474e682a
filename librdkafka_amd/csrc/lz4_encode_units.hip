// lz4_encode_units.hip -- throughput-mode LZ4F block compression, one 1024-thread
// workgroup per 64 KiB block with the block's source and its hash table in LDS.
//
// Same frame format, prefs and raw-block fallback as rd_kafka_lz4_compress
// (src/rdkafka_lz4.c:329-442: {blockIndependent, level 0}, 64 KiB blocks, no checksums;
// LZ4F_makeBlock lz4frame.c:739-761).  The match search is the engine's own, built for a
// compute unit instead of following LZ4_compress_generic (lz4.c:789-1177) step by step;
// frames decode with the reference decoder to the input and are not byte-identical to the
// reference's.  The result is defined by a sequential model, tests/sim/lz4_units_sim.cpp,
// which this kernel reproduces byte for byte:
//
//   * LDS holds the whole block (64 KiB, at the byte alignment it has in memory), a
//     2^13-entry hash table (the reference's byU16 table size, lz4.c:633), a double buffer
//     of candidates and a staging area for the output: nothing but the block's own bytes
//     is read from memory, once, and the output leaves in aligned 16-byte stores.
//   * Wave 0, the FINDER, runs over the block in position order, 64 positions per step:
//     LZ4_hash4 (lz4.c:631) of every position, the table's entry as the position's
//     candidate, then the position is entered (dense insertion).  It works one TICK
//     (12 units of 960 positions) ahead of the parsers and leaves one u16 candidate per
//     position in LDS.  It has its SIMD to itself.
//   * Twelve PARSER waves (on the other three SIMDs) take one unit of a tick each.  Per
//     64 positions: every lane verifies its candidate (MINMATCH) and measures the match from two 16-byte LDS
//     reads on each side (up to 28 bytes forward, 4 back for the catch-up of lz4.c:957,
//     longer matches by the whole wave); the greedy walk over the verified lanes is scalar
//     (one s_ff1 + v_readlane per sequence); the chosen lanes append (position, length,
//     candidate, catch-up) to the unit's queue, which lives in the candidate rows the unit
//     has already consumed.  A unit is parsed as if the block began at its first
//     position; a match may run past its end.
//   * After a barrier the units of the tick are stitched in order (every wave computes the
//     same short chain): the end of the last match so far may lie inside a unit, whose
//     sequences that it covers are dropped, and one that it covers in part keeps the rest
//     of its match; the first sequence kept takes over the literals left behind.  The
//     queued sequences are turned into LZ4 sequence fields 64 at a time (one per lane).
//     A second barrier and a prefix sum over the units' sizes later every parser writes
//     its unit's sequences (token, literals, offset, length bytes: lz4.c:961-1073) at
//     their final offsets into the staging area, and after a third barrier the whole
//     workgroup copies the tick's bytes out.
//   * The CRC32C of the finished batch is taken by the batched CRC kernels over the
//     assembled frames (they run at memory speed and the frames are a third of the
//     input); this kernel leaves no per-block registers.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "lz4_device.h"
#include "lz4_engine.h"
#include "lz4_wave.h"

namespace rdk {

void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s, const FuseCrc *fuse);

namespace {

#ifndef RDK_UNITS_WINDOWS
#define RDK_UNITS_WINDOWS 15
#endif
constexpr int kUnitWindows = RDK_UNITS_WINDOWS;  // 64-position windows per unit
constexpr int kUnitLen = kUnitWindows * 64;      // 960 positions
// 16 waves: a workgroup's waves w, w+4, w+8, w+12 share a SIMD.  Wave 0 is the finder and
// has its SIMD to itself (waves 4, 8 and 12 only keep the barriers); the other twelve parse.
constexpr int kWorkers = 12;                     // parser waves
constexpr int kTickLen = kWorkers * kUnitLen;    // positions per tick
constexpr int kThreads = 1024;
constexpr uint32_t kHashLogU = 13;
constexpr int kRegLen = 28;                      // match bytes a lane measures by itself
constexpr int kMaxItemsU = 64;                   // block slots per frame per pass
constexpr uint32_t kSlotU = kLz4Block + 4;       // worst-case bytes per block in a frame

// LDS map (bytes).  The source image starts kPad + (src & 15) bytes in: position -4 and
// the read-ahead past the block's end (28 bytes per lane, 256 per long-match step, the
// finder's eight steps) stay inside it.
constexpr int kPad = 32;
constexpr int kSrcBytes = 66688;
constexpr int kTabOff = 0;                       // (first: its addresses need no base)
#ifdef RDK_UNITS_TABLE_U16
constexpr int kTabBytes = 2 << kHashLogU;        // u16 entries, plain stores
#else
constexpr int kTabBytes = 4 << kHashLogU;        // u32 entries, entered with ds_max_u32
#endif
constexpr int kRingOff = kTabOff + kTabBytes;
constexpr int kRingBytes = (kTickLen + 8 * 64) * 2;  // a tick of u16 candidates + run-ahead rows
constexpr int kSrcOff = kRingOff + 2 * kRingBytes;
constexpr int kStageOff = kSrcOff + kSrcBytes;
constexpr int kStageBytes = ((160 * 1024 - 512 - kStageOff) / 16) * 16;  // what is left
constexpr int kRecOff = kStageOff + kStageBytes;
constexpr int kLdsBytes = kRecOff + 512;         // unit records (16 x 16 B) + sizes (16 x 4 B)
static_assert(kLdsBytes <= 160 * 1024, "one workgroup per CU");
static_assert(kStageBytes >= 4096, "room to stage a tick's output");
static_assert(kUnitLen / kLz4MinMatch * 8 <= kUnitLen * 2, "a unit's queue fits its candidate rows");
// a unit's queue (8 bytes per sequence, a sequence per 4 positions at most) fits the
// candidate rows of the windows it came from (2 bytes per position)
static_assert(8 * (64 / kLz4MinMatch) <= 2 * 64, "queue entries fit the consumed rows");

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32_a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) u32x2 lds_v2;
typedef __attribute__((address_space(3))) u32x4 lds_v4;
typedef __attribute__((address_space(3))) const u32x4_a1 lds_cv4u;
typedef __attribute__((address_space(3))) const u32_a1 lds_cu32u;
typedef __attribute__((address_space(3))) int lds_i32;
typedef __attribute__((address_space(1))) u32x4 g_v4;

// -DRDK_UNITS_PROF: cycle stamps around the phases of a block, summed per role (finder /
// parser) into a device array that rdk_hip_units_prof_dump() prints (timing builds only).
#ifdef RDK_UNITS_PROF
__device__ unsigned long long g_units_prof[2][12];
#define RDK_UP_DECL uint64_t up_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; uint64_t upt_ = __builtin_amdgcn_s_memtime()
#define RDK_UP(k) do { const uint64_t now_ = __builtin_amdgcn_s_memtime(); up_[k] += now_ - upt_; upt_ = now_; } while (0)
#define RDK_UP_FLUSH(role) do { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 12; ++k_) atomicAdd(&g_units_prof[role][k_], (unsigned long long)up_[k_]); } while (0)
#else
#define RDK_UP_DECL do { } while (0)
#define RDK_UP(k) do { } while (0)
#define RDK_UP_FLUSH(role) do { } while (0)
#endif

struct Blk {            // wave-uniform
  lds_u8 *L;            // LDS base
  lds_u8 *S;            // LDS address of position 0
  int n, mfl, mlim, olimit;
  uintptr_t dst;        // the block's payload in its slot
  rsrc_t w;             // byte stores into the payload; parked lanes write nothing
};

__device__ __forceinline__ uint32_t hash13(uint32_t seq) {  // LZ4_hash4, lz4.c:631
  return (seq * 2654435761u) >> (32 - kHashLogU);
}

// equal bytes a[i] == c[i] for i in [0, limit), 256 per wave step, from LDS
__device__ __forceinline__ int lds_count_fwd(const lds_u8 *a, const lds_u8 *c, int limit, int lane) {
  int cnt = 0;
  while (cnt < limit) {
    const int o = cnt + 4 * lane;
    const uint32_t x = *(lds_cu32u *)(a + o) ^ *(lds_cu32u *)(c + o);
    const int eqb = x ? int(__builtin_ctz(x) >> 3) : 4;
    const uint64_t full = ballot(eqb == 4);
    if (full == ~0ull) {
      cnt += 256;
      continue;
    }
    const int fl = __builtin_ctzll(~full);
    cnt += 4 * fl + __builtin_amdgcn_readlane(eqb, fl);
    break;
  }
  return cnt < limit ? cnt : limit;
}

// `len` bytes from LDS to memory, 64 per step
__device__ __forceinline__ void lds_copy_out(uintptr_t d, const lds_u8 *s, uint32_t len, int lane) {
  for (uint32_t base = 0; base < len; base += 256u) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = s[base + uint32_t(lane) + 64u * j];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + uint32_t(lane) + 64u * j;
      if (i < len) stb(d + i, v[j]);
    }
  }
}

// `len` bytes inside LDS, 64 per step (source and destination do not overlap)
__device__ __forceinline__ void lds_copy_lds(lds_u8 *d, const lds_u8 *s, uint32_t len, int lane) {
  for (uint32_t base = 0; base < len; base += 256u) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = s[base + uint32_t(lane) + 64u * j];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + uint32_t(lane) + 64u * j;
      if (i < len) d[i] = uint8_t(v[j]);
    }
  }
}

// ---- the finder: candidates of the positions [ts, te) (te - ts a multiple of 64 unless
// te is the block's end) into `ring`.  Every lane reads the table, then every lane of a
// position that may start a match enters its position: where several lanes of a step hit
// the same entry the highest position must land.  With u32 entries that is an LDS atomic
// maximum, right by arithmetic.
//
// Four steps are kept in flight: their table reads and entries are issued back to back
// (the LDS runs one wave's operations in order, so step k+1's read sees step k's entries
// without a wait in between), the bytes of the next four steps are requested before them,
// and only then the four candidate rows are formed and stored -- one exposed LDS round
// trip per four steps instead of three per step.
template <bool CHECKED>
__device__ __forceinline__ void finder_group(const Blk &b, int R, int ts, int te, lds_u16 *ring,
                                             uint32_t (&seq)[8], int lane) {
  constexpr int G = 8;
#ifdef RDK_UNITS_TABLE_U16
  lds_u16 *table = (lds_u16 *)(b.L + kTabOff);
#else
  lds_u32 *table = (lds_u32 *)(b.L + kTabOff);
#endif
  uint32_t nxt[G], c[G];
#pragma unroll
  for (int g = 0; g < G; ++g) nxt[g] = *(lds_cu32u *)(b.S + R + 64 * (G + g) + lane);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int i = R + 64 * g + lane;
    const uint32_t h = hash13(seq[g]);
    c[g] = table[h];
    // (CHECKED: a lane that may not start a match, or a step past the tick's end, changes nothing)
    const bool enter = !CHECKED || (i <= b.mfl && R + 64 * g < te);
#ifdef RDK_UNITS_TABLE_U16
    if (enter) table[h] = uint16_t(i);
#else
    __hip_atomic_fetch_max(table + h, enter ? uint32_t(i) : 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int i = R + 64 * g + lane;
    // (steps past te write into the slack behind the tick's rows: never read as candidates)
    if (CHECKED) ring[i - ts] = (i <= b.mfl && int(c[g]) < i) ? uint16_t(c[g]) : uint16_t(0xFFFFu);
    else ring[i - ts] = uint16_t(c[g]);
    seq[g] = nxt[g];
  }
}

// Eight steps are kept in flight: their table reads and entries are issued back to back
// (the LDS runs one wave's operations in order, so step k+1's read sees step k's entries
// without a wait in between), the bytes of the next eight steps are requested before them,
// and only then the eight candidate rows are formed and stored -- one exposed LDS round
// trip per eight steps.  A group whose positions all lie in [64, mfl] and inside the tick
// needs none of the per-lane checks (every table entry is an earlier position; 0 stands for
// position 0 or an empty entry, both of which the parser's byte comparison settles).
__device__ __forceinline__ void finder_tick(const Blk &b, int ts, int te, lds_u16 *ring, int lane) {
  constexpr int G = 8;
  uint32_t seq[G];
#pragma unroll
  for (int g = 0; g < G; ++g) seq[g] = *(lds_cu32u *)(b.S + ts + 64 * g + lane);
  for (int R = ts; R < te; R += 64 * G) {
    if (R > 0 && R + 64 * G <= te && R + 64 * G - 1 <= b.mfl) finder_group<false>(b, R, ts, te, ring, seq, lane);
    else finder_group<true>(b, R, ts, te, ring, seq, lane);
  }
}

// ---- a parser's unit [u0, u1): measure, walk, queue.
// One window's loads: the candidate row and, for every lane, 32 bytes around its position
// and around its candidate (positions -4 .. +28).
struct WinLoads {
  u32x4_a1 a0, a1, c0, c1;
  uint32_t c16;
};

__device__ __forceinline__ void window_loads(const Blk &b, WinLoads &W, int R, uint32_t c16, int lane) {
  const int c = c16 != 0xFFFFu ? int(c16) : 0;
  const lds_u8 *pi = b.S + R + lane, *pc = b.S + c;
  W.c16 = c16;
  W.a0 = *(lds_cv4u *)(pi - 4);
  W.a1 = *(lds_cv4u *)(pi + 12);
  W.c0 = *(lds_cv4u *)(pc - 4);
  W.c1 = *(lds_cv4u *)(pc + 12);
}

// The window at R: `p` is the parse position == anchor (the end of the last match); the
// chosen lanes append (position | length << 16, candidate | catch-up << 16) at queue[qn].
// The catch-up kept here is the count of equal bytes in front of position and candidate
// (at most 4); it is cut to the literals available when the fields are made.
__device__ __forceinline__ void parse_window(const Blk &b, lds_u8 *queue, int &qn, int &p,
                                             const WinLoads &W, int R, int lane) {
  if (p >= R + 64) return;  // a long match covers the window
  const int i = R + lane;
  const bool has = W.c16 != 0xFFFFu;
  const int c = has ? int(W.c16) : 0;
  const u32x4_a1 a0 = W.a0, a1 = W.a1, c0 = W.c0, c1 = W.c1;
  const bool valid = has && i >= p && a0.y == c0.y;
  const uint64_t vm = ballot(valid);
  if (!vm) return;
  // first differing bit behind the 4 verified bytes: trailing-zero counts over dword
  // pairs (64 exactly when a pair is equal: only then the next pair counts)
  const uint64_t w0 = (uint64_t(a0.w ^ c0.w) << 32) | (a0.z ^ c0.z);
  const uint64_t w1 = (uint64_t(a1.y ^ c1.y) << 32) | (a1.x ^ c1.x);
  const uint64_t w2 = (uint64_t(a1.w ^ c1.w) << 32) | (a1.z ^ c1.z);
  const uint32_t z0 = w0 ? uint32_t(__builtin_ctzll(w0)) : 64u;
  const uint32_t z1 = w1 ? uint32_t(__builtin_ctzll(w1)) : 64u;
  const uint32_t z2 = w2 ? uint32_t(__builtin_ctzll(w2)) : 64u;
  uint32_t fd = z1 + (z1 >> 6) * z2;
  fd = (z0 + (z0 >> 6) * fd) >> 3;
  int len = 4 + int(fd < uint32_t(kRegLen - 4) ? fd : uint32_t(kRegLen - 4));
  if (len > b.mlim - i) len = b.mlim - i;

  // greedy walk: first verified position at or after the end of the last match
  int xr = p - R;
  uint64_t chosen = 0;
  for (;;) {
    const int rel = xr > 0 ? xr : 0;
    if (rel >= 64) break;
    const uint64_t m = vm & (~0ull << rel);
    if (!m) break;
    const int q = __builtin_ctzll(m);
    int Lq = __builtin_amdgcn_readlane(len, q);
    if (Lq == kRegLen && R + q + kRegLen < b.mlim) {  // long match: the whole wave goes on
      const int qi = R + q, ci = __builtin_amdgcn_readlane(c, q);
      Lq += lds_count_fwd(b.S + qi + kRegLen, b.S + ci + kRegLen, b.mlim - qi - kRegLen, lane);
      if (lane == q) len = Lq;
    }
    chosen |= 1ull << q;
    xr = q + Lq;
  }
  if (!chosen) return;
  p = R + xr;
  const uint32_t xb = a0.x ^ c0.x;
  const uint32_t bk0 = xb ? uint32_t(__builtin_clz(xb) >> 3) : 4u;  // equal bytes in front (lz4.c:957)
  const int rank = int(__builtin_amdgcn_mbcnt_hi(uint32_t(chosen >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(uint32_t(chosen), 0u)));
  if (__builtin_amdgcn_inverse_ballot_w64(chosen)) {
    const u32x2 e = {uint32_t(i) | (uint32_t(len) << 16), uint32_t(c) | (bk0 << 16)};
    *(lds_v2 *)(queue + 8 * (qn + rank)) = e;
  }
  qn += __builtin_popcountll(chosen);
}

// `row` is the unit's part of the tick's candidate buffer (one u16 per position).  The loads
// run ahead of the parse: a window's candidate row is read two windows early, its bytes one
// window early (two register sets, used in turn), so a window's LDS round trips pass behind
// the parse of the window before it.  The queue grows into the rows already read: a window
// adds at most 16 entries of 8 bytes, the 128 bytes of its own row.
__device__ __forceinline__ int parse_unit(const Blk &b, int u0, int u1, lds_u16 *row, int lane) {
  int qn = 0, p = u0;
  lds_u8 *queue = (lds_u8 *)row;
  uint32_t ka = row[lane], kb = row[64 + lane];
  WinLoads WA, WB;
  window_loads(b, WA, u0, ka, lane);
  for (int R = u0; R < u1; R += 128) {
    ka = row[R - u0 + 128 + lane];
    window_loads(b, WB, R + 64, kb, lane);
    parse_window(b, queue, qn, p, WA, R, lane);
    if (R + 64 >= u1) break;
    kb = row[R - u0 + 192 + lane];
    window_loads(b, WA, R + 128, ka, lane);
    parse_window(b, queue, qn, p, WB, R + 64, lane);
  }
  return qn;
}

// ---- the unit's queue turned into LZ4 sequence fields, 64 entries a pass, and stitched
// against the end of the last match kept so far (`ain`): drops and trims as the model does,
// gives the first sequence kept the literals from ain on.  The entries are rewritten in
// place as (literal start | literal length << 16, offset | (match length - 4) << 16), offset
// 0 = dropped.  Returns the bytes the unit's sequences take.
__device__ __forceinline__ uint32_t stitch_unit(const Blk &b, lds_u8 *queue, int nseq, int u0, int ain,
                                                int lane) {
  uint32_t total = 0;
  bool firstdone = false;
  int prev_last = u0;  // end of the match in front of the pass's first entry
  for (int base = 0; base < nseq; base += 64) {
    const bool valid = base + lane < nseq;
    const u32x2 e = *(lds_v2 *)(queue + 8 * (base + lane));
    const int q = int(e.x & 0xFFFFu), len = int(e.x >> 16);
    const int c = int(e.y & 0xFFFFu), bk0 = int(e.y >> 16);
    const int end = valid ? q + len : 0;
    // the anchor: the end of the entry in front (wave_shr:1; lane 0 takes the pass's carry)
    int anchor = __builtin_amdgcn_update_dpp(prev_last, end, 0x138, 0xf, 0xf, false);
    if (lane == 0) anchor = prev_last;
    prev_last = __builtin_amdgcn_readlane(end, 63);
    const int bk = min(bk0, min(q - anchor, c));  // literals only, inside the block
    int ms = q - bk;
    const int me = end;
    bool keep = valid && me > ain;
    if (ms < ain) {
      keep = keep && me - ain >= kLz4MinMatch && ain <= b.mfl;
      ms = ain;
    }
    uint32_t lstart = uint32_t(anchor);
    const uint64_t km = ballot(keep);
    if (!firstdone && km) {
      if (lane == __builtin_ctzll(km)) lstart = uint32_t(ain);
      firstdone = true;
    }
    const uint32_t lit = uint32_t(ms) - lstart, mc = uint32_t(me - ms) - 4u;
    const uint32_t off = uint32_t(q - c);
    const u32x2 o = {keep ? (lstart | (lit << 16)) : 0u, keep ? (off | (mc << 16)) : 0u};
    *(lds_v2 *)(queue + 8 * (base + lane)) = o;
    const uint32_t sz = keep ? 3u + lit + ext_bytes(lit) + ext_bytes(mc) : 0u;
    uint32_t t;
    (void)wave_excl_scan(sz, t);
    total += t;
  }
  return total;
}

// the end of a unit's last match and where it starts (catch-up included): what the chain
// over the units needs
__device__ __forceinline__ void unit_last_match(lds_u8 *queue, int nseq, int u0, int &ms, int &me) {
  const u32x2 e = *(lds_v2 *)(queue + 8 * (nseq - 1));
  const u32x2 f = *(lds_v2 *)(queue + 8 * (nseq > 1 ? nseq - 2 : 0));
  const int q = int(uni(e.x) & 0xFFFFu), len = int(uni(e.x) >> 16);
  const int c = int(uni(e.y) & 0xFFFFu), bk0 = int(uni(e.y) >> 16);
  const int anchor = nseq > 1 ? int(uni(f.x) & 0xFFFFu) + int(uni(f.x) >> 16) : u0;
  ms = q - min(bk0, min(q - anchor, c));
  me = q + len;
}

// ---- a unit's sequences written at offset `at` of the image at `out` (the staging area,
// byte stores in LDS)
__device__ __forceinline__ void emit_unit_lds(const Blk &b, const lds_u8 *queue, int nseq, lds_u8 *out,
                                              uint32_t at, int lane) {
  constexpr uint32_t kShortLit = 16;
  for (int base = 0; base < nseq; base += 64) {
    const u32x2 e = *(lds_v2 *)(queue + 8 * (base + lane));
    const uint32_t off = base + lane < nseq ? e.y & 0xFFFFu : 0u, mc = e.y >> 16;
    const bool ch = off != 0u;
    const uint32_t lstart = e.x & 0xFFFFu, lit = ch ? e.x >> 16 : 0u;
    const uint32_t lext = ext_bytes(lit), mext = ext_bytes(mc);
    const uint32_t sz = ch ? 3u + lit + lext + mext : 0u;
    uint32_t tot;
    const uint32_t o = wave_excl_scan(sz, tot);
    lds_u8 *tp = out + at + o;           // token
    lds_u8 *lp = tp + 1u + lext;         // first literal
    lds_u8 *fp = lp + lit;               // offset field
    if (ch) {
      tp[0] = uint8_t(((lit < 15u ? lit : 15u) << 4) | (mc < 15u ? mc : 15u));
      fp[0] = uint8_t(off);
      fp[1] = uint8_t(off >> 8);
      if (mc >= 15u) {  // 255-runs + remainder (one byte for mc < 270)
        uint32_t r = mc - 15u;
        lds_u8 *x = fp + 2;
        for (; r >= 255u; r -= 255u) *x++ = 255u;
        *x = uint8_t(r);
      }
      if (lit >= 15u) {
        uint32_t r = lit - 15u;
        lds_u8 *x = tp + 1;
        for (; r >= 255u; r -= 255u) *x++ = 255u;
        *x = uint8_t(r);
      }
    }
    const bool need_win = ch && lit != 0u && lit <= kShortLit;
    if (ballot(need_win)) {  // up to 16 literals: one 16-byte LDS read per lane
      const u32x4_a1 v = *(lds_cv4u *)(b.S + (need_win ? lstart : 0u));
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (uint32_t k = 0; k < kShortLit; ++k)
        if (need_win && k < lit) lp[k] = uint8_t(vv[k >> 2] >> (8u * (k & 3u)));
    }
    uint64_t longm = ballot(ch && lit > kShortLit);  // long runs: the whole wave, one at a time
    while (longm) {
      const int l = __builtin_ctzll(longm);
      longm &= longm - 1;
      const uint32_t o_l = uint32_t(__builtin_amdgcn_readlane(int(o), l));
      const uint32_t lext_l = uint32_t(__builtin_amdgcn_readlane(int(lext), l));
      lds_copy_lds(out + at + o_l + 1u + lext_l,
                   b.S + uint32_t(__builtin_amdgcn_readlane(int(lstart), l)),
                   uint32_t(__builtin_amdgcn_readlane(int(lit), l)), lane);
    }
    at += tot;
  }
}

// the same straight into memory (a tick whose output does not fit the staging area: long
// literal runs in front of its first match)
__device__ __forceinline__ void emit_unit_mem(const Blk &b, const lds_u8 *queue, int nseq, uint32_t at,
                                              int lane) {
  constexpr uint32_t kShortLit = 16;
  for (int base = 0; base < nseq; base += 64) {
    const u32x2 e = *(lds_v2 *)(queue + 8 * (base + lane));
    const uint32_t off = base + lane < nseq ? e.y & 0xFFFFu : 0u, mc = e.y >> 16;
    const bool ch = off != 0u;
    const uint32_t lstart = e.x & 0xFFFFu, lit = ch ? e.x >> 16 : 0u;
    const uint32_t lext = ext_bytes(lit);
    const uint32_t sz = ch ? 3u + lit + lext + ext_bytes(mc) : 0u;
    uint32_t tot;
    const uint32_t o = wave_excl_scan(sz, tot);
    const uint32_t tp = at + o, lp = tp + 1u + lext, fp = lp + lit;
    __builtin_amdgcn_raw_buffer_store_b8(
        uint8_t(((lit < 15u ? lit : 15u) << 4) | (mc < 15u ? mc : 15u)), b.w, ch ? tp : kNoLoad, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off), b.w, ch ? fp : kNoLoad, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off >> 8), b.w, ch ? fp + 1u : kNoLoad, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(mc - 15u), b.w,
                                         (ch && mc >= 15u && mc < 270u) ? fp + 2u : kNoLoad, 0, 0);
    if (ballot(ch && lit >= 15u)) {
      if (ch && lit >= 15u) put_len(b.dst + tp + 1u, lit);
    }
    if (ballot(ch && mc >= 270u)) {
      if (ch && mc >= 270u) put_len(b.dst + fp + 2u, mc);
    }
    const bool need_win = ch && lit != 0u && lit <= kShortLit;
    if (ballot(need_win)) {
      const u32x4_a1 v = *(lds_cv4u *)(b.S + (need_win ? lstart : 0u));
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (uint32_t k = 0; k < kShortLit; ++k)
        __builtin_amdgcn_raw_buffer_store_b8(uint8_t(vv[k >> 2] >> (8u * (k & 3u))), b.w,
                                             (need_win && k < lit) ? lp + k : kNoLoad, 0, 0);
    }
    uint64_t longm = ballot(ch && lit > kShortLit);
    while (longm) {
      const int l = __builtin_ctzll(longm);
      longm &= longm - 1;
      lds_copy_out(b.dst + uint32_t(__builtin_amdgcn_readlane(int(lp), l)),
                   b.S + uint32_t(__builtin_amdgcn_readlane(int(lstart), l)),
                   uint32_t(__builtin_amdgcn_readlane(int(lit), l)), lane);
    }
    at += tot;
  }
}

// ---- `len` staged bytes to memory at g, by the whole workgroup: the aligned 16-byte
// chunks inside [g, g+len) with one store per thread (read from LDS at whatever alignment
// that gives), the ragged head and tail byte by byte
__device__ __forceinline__ void stage_copy_out(const lds_u8 *stage, uintptr_t g, uint32_t len, int tid) {
  const uintptr_t a0 = (g + 15u) & ~uintptr_t(15);  // first aligned address at or after g
  const uint32_t head = uint32_t(a0 - g) < len ? uint32_t(a0 - g) : len;
  const uint32_t nchunk = (len - head) >> 4;
  for (uint32_t k = uint32_t(tid); k < nchunk; k += uint32_t(kThreads)) {
    const u32x4_a1 v = *(lds_cv4u *)(stage + head + 16u * k);
    const u32x4 w = {v.x, v.y, v.z, v.w};
    *(g_v4 *)(a0 + 16u * k) = w;
  }
  const uint32_t tail0 = head + 16u * nchunk;  // bytes [tail0, len) are the ragged tail
  if (uint32_t(tid) < head) stb(g + uint32_t(tid), stage[tid]);
  if (tid >= 64 && uint32_t(tid - 64) < len - tail0)
    stb(g + tail0 + uint32_t(tid - 64), stage[tail0 + uint32_t(tid - 64)]);
}

// One block of n (>= 13) bytes at src into the payload at dst (capacity n-1).  Every wave
// of the workgroup returns the same compressed size, or 0 when the block does not fit
// (stored raw).
__device__ int units_block(lds_u8 *L, uintptr_t src, int n, uintptr_t dst) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = int(uni(uint32_t(tid >> 6)));
  const bool parser = (wave & 3) != 0;                 // waves 0, 4, 8, 12 do not parse
  const int worker = (wave >> 2) * 3 + (wave & 3) - 1;  // 0..11 for the parsers
  Blk b;
  b.L = L;
  const uint32_t sa = uint32_t(src & 15u);
  b.S = L + kSrcOff + kPad + sa;
  b.n = n;
  b.mfl = n - kLz4MFLimit;        // last position a match may start (lz4.c:907)
  b.mlim = n - kLz4LastLiterals;  // matchlimit (lz4.c:822)
  b.olimit = n - 1;               // LZ4F_makeBlock dstCapacity
  b.dst = dst;
  b.w = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(dst), 0, n, 0x00020000);

  RDK_UP_DECL;
  __syncthreads();  // the previous block's readers are done with the LDS
  RDK_UP(0);
  {  // the block's bytes, as the aligned 16-byte chunks that hold them; table zeroed
    const uintptr_t lo = src - sa;
    const rsrc_t r = block_rsrc(lo, (src + uint32_t(n) + 15u) & ~uintptr_t(15));
    const int nchunks = int((sa + uint32_t(n) + 15u) >> 4);
    u32x4 v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int j = tid + kThreads * k;
      v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, j < nchunks ? uint32_t(j) * 16u : kNoLoad, 0, 0);
    }
    const u32x4 z = {0u, 0u, 0u, 0u};
    static_assert(kTabBytes % (16 * kThreads) == 0, "whole 16-byte stores per thread clear the table");
#pragma unroll
    for (int k = 0; k < kTabBytes / (16 * kThreads); ++k)
      *(lds_v4 *)(L + kTabOff + 16 * (tid + kThreads * k)) = z;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int j = tid + kThreads * k;
      if (j < nchunks) *(lds_v4 *)(L + kSrcOff + kPad + 16 * j) = v[k];
    }
  }
  __syncthreads();
  RDK_UP(1);

  const int nunits = (n + kUnitLen - 1) / kUnitLen;
  const int nticks = (nunits + kWorkers - 1) / kWorkers;
  lds_u16 *ring0 = (lds_u16 *)(L + kRingOff), *ring1 = (lds_u16 *)(L + kRingOff + kRingBytes);
  lds_u8 *stage = L + kStageOff;
  lds_i32 *recs = (lds_i32 *)(L + kRecOff);          // [16][4]: ms, me, nseq of a unit's last match
  lds_i32 *sizes = (lds_i32 *)(L + kRecOff + 256);   // [16]

  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);
    finder_tick(b, 0, n < kTickLen ? n : kTickLen, ring0, lane);
    __builtin_amdgcn_s_setprio(0);
  }
  RDK_UP(2);
  __syncthreads();
  RDK_UP(3);

  int carry = 0;       // end of the last match kept so far == start of the literals not yet written
  uint32_t obase = 0;  // payload bytes written so far
  bool fits = true;
  for (int t = 0; t < nticks; ++t) {
    const int ts = t * kTickLen;
    lds_u16 *ring = (t & 1) ? ring1 : ring0;
    const int u = t * kWorkers + (parser ? worker : 0);
    const int u0 = u * kUnitLen, u1 = u0 + kUnitLen < n ? u0 + kUnitLen : n;
    lds_u16 *row = ring + (parser ? worker * kUnitLen : 0);
    lds_u8 *queue = (lds_u8 *)row;
    int nseq = 0;
    if (wave == 0) {
      if (t + 1 < nticks) {
        const int ns = ts + kTickLen, ne = ns + kTickLen < n ? ns + kTickLen : n;
        __builtin_amdgcn_s_setprio(3);
        finder_tick(b, ns, ne, (t & 1) ? ring0 : ring1, lane);
        __builtin_amdgcn_s_setprio(0);
      }
    } else if (parser) {
      int ms = 0, me = 0;
      if (u < nunits) {
        nseq = parse_unit(b, u0, u1, row, lane);
        if (nseq) unit_last_match(queue, nseq, u0, ms, me);
      }
      if (lane == 0) {
        recs[4 * worker + 0] = ms;
        recs[4 * worker + 1] = me;
        recs[4 * worker + 2] = nseq;
      }
    }
    RDK_UP(4);
    __syncthreads();
    RDK_UP(5);
    // ---- the chain over the tick's units, the same in every wave
    int ain = carry;
    {
      const int j4 = 4 * (lane < kWorkers ? lane : 0);
      const int vms = recs[j4], vme = recs[j4 + 1], vnq = recs[j4 + 2];
      int a = carry;
#pragma unroll
      for (int j = 0; j < kWorkers; ++j) {
        const int ms = __builtin_amdgcn_readlane(vms, j), me = __builtin_amdgcn_readlane(vme, j);
        const int nq = __builtin_amdgcn_readlane(vnq, j);
        if (parser && j == worker) ain = a;
        const bool keep = nq > 0 && me > a && (ms >= a || (me - a >= kLz4MinMatch && a <= b.mfl));
        a = keep ? me : a;
      }
      carry = a;
    }
    uint32_t mine = 0;
    if (nseq) mine = stitch_unit(b, queue, nseq, u0, ain, lane);
    if (parser && lane == 0) sizes[worker] = int(mine);
    RDK_UP(6);
    __syncthreads();
    RDK_UP(7);
    const uint32_t sz = lane < kWorkers ? uint32_t(sizes[lane]) : 0u;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan(sz, tot);
    const uint32_t at = uint32_t(__builtin_amdgcn_readlane(int(ex), parser ? worker : 0));
    // keep room for the shortest possible last-literals token (lz4.c:1146)
    if (int(obase + tot) + 1 > b.olimit) fits = false;
    if (!fits) break;  // the same in every wave: stored raw
    const bool staged = tot <= uint32_t(kStageBytes);
    if (nseq) {
      if (staged) emit_unit_lds(b, queue, nseq, stage, at, lane);
      else emit_unit_mem(b, queue, nseq, obase + at, lane);
    }
    RDK_UP(8);
    __syncthreads();  // the tick's bytes are staged; its queues are free for the finder
    RDK_UP(9);
    if (staged) stage_copy_out(stage, dst + obase, tot, tid);
    obase += tot;
    RDK_UP(10);
  }
  // last literals (lz4.c:1141-1166)
  const uint32_t last = uint32_t(n - carry);
  const uint32_t total = obase + 1u + ext_bytes(last) + last;
  const bool ok = fits && int(total) <= b.olimit;
  if (ok && wave == 0) {
    if (lane == 0) {
      uintptr_t p0 = dst + obase;
      stb(p0++, (last < 15u ? last : 15u) << 4);
      if (last >= 15u) put_len(p0, last);
    }
    lds_copy_out(dst + obase + 1u + ext_bytes(last), b.S + carry, last, lane);
  }
  RDK_UP(11);
  if (parser || wave == 0) RDK_UP_FLUSH(parser ? 1 : 0);
  return ok ? int(total) : 0;
}

__global__ __launch_bounds__(kThreads) void lz4_units_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_mem[kLdsBytes];  // the kernel's only LDS
  lds_u8 *L = (lds_u8 *)lds_mem;
  const uint64_t items = uint64_t(n) * kMaxItemsU;
  for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
    // slot-major items: all frames' block 0, then all block 1, ...: the blocks that exist
    // come first and are dense in blockIdx
    const uint32_t f = uint32_t(it % n), kk = uint32_t(it / n);
    const uint32_t len = uni(in_lens[f]);
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    for (uint32_t k = kk; k < nb; k += kMaxItemsU) {
      const uint32_t bn = (len - k * kLz4Block) < kLz4Block ? (len - k * kLz4Block) : kLz4Block;
      const uintptr_t src = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kLz4Block;
      const uintptr_t slot = reinterpret_cast<uintptr_t>(out) + out_offs[f] + 7u + uint64_t(k) * kSlotU;
      int csize = 0;
      if (bn >= uint32_t(kLz4MFLimit + 1)) csize = units_block(L, src, int(bn), slot + 4u);
      const uint32_t w = csize ? uint32_t(csize) : (bn | 0x80000000u);  // LZ4F_makeBlock
      if (threadIdx.x == 0) {
        stb(slot, w & 0xFFu); stb(slot + 1, (w >> 8) & 0xFFu);
        stb(slot + 2, (w >> 16) & 0xFFu); stb(slot + 3, w >> 24);
      }
    }
  }
}

}  // namespace

#ifdef RDK_UNITS_PROF
extern "C" __attribute__((visibility("default"))) void rdk_hip_units_prof_dump(void) {
  unsigned long long h[2][12];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_units_prof), sizeof h) != hipSuccess) return;
  static const char *names[12] = {"wait-prev", "load", "finder0", "wait-finder0", "role-work", "wait-B1",
                                  "chain+stitch", "wait-B2", "prefix+emit", "wait-B3", "copy-out", "final"};
  for (int r = 0; r < 2; ++r) {
    unsigned long long tot = 0;
    for (int k = 0; k < 12; ++k) tot += h[r][k];
    fprintf(stderr, "units prof %s:", r ? "parsers" : "finder");
    for (int k = 0; k < 12; ++k) fprintf(stderr, " %s %.1f%%", names[k], tot ? 100.0 * double(h[r][k]) / double(tot) : 0.0);
    fprintf(stderr, " | total Mcycles %.1f\n", double(tot) / 1e6);
  }
}
#endif

// Blocks of n frames into their worst-case slots (size word + payload), then frame
// assembly.  `fuse` (finalize mode) carries no block registers here: the assembler writes
// the header with a zero CRC and the caller runs the CRC pass over the finished batches.
int lz4f_compress_units_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                               const uint32_t *d_in_lens, uint8_t *d_out,
                               const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                               hipStream_t s, const FuseCrc *fuse) {
  if (!n) return 0;
  const uint64_t items = uint64_t(n) * kMaxItemsU;
  const unsigned grid = unsigned(items < 256u ? items : 256u);  // one workgroup per CU
  hipLaunchKernelGGL(lz4_units_blocks_kernel, dim3(grid), dim3(kThreads), 0, s, d_in, d_in_offs,
                     d_in_lens, d_out, d_out_offs, n);
  lz4f_assemble_launch(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, s, fuse);
  RDK_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace rdk
