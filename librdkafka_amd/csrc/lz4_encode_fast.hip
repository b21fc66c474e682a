// lz4_encode_fast.hip -- throughput-mode LZ4F compression on gfx950.
//
// Same frame format and block independence as rd_kafka_lz4_compress
// (src/rdkafka_lz4.c:329-442: prefs {blockIndependent, level}, 64 KiB blocks,
// no checksums, LZ4F_makeBlock's raw fallback lz4frame.c:739-761), but the
// match search is restructured for a wavefront instead of emulating the
// sequential LZ4_compress_generic loop (lz4.c:789-1177) step by step:
//
//   * positions are processed in rounds of 64 probes (one per lane).  Every position
//     <= n-12 is hashed with LZ4_hash4 (lz4.c:631) into a 2^12-entry u16 table in LDS that
//     holds the LATEST earlier position per hash (dense insertion, the reference inserts
//     only the positions it probes);
//   * a lane's candidate is the table entry as of the start of its round; the lane verifies
//     MINMATCH bytes, measures up to 28 match bytes and up to 4 catch-up bytes (lz4.c:957)
//     from two 36-byte register windows (its own position's, loaded three rounds ahead, and
//     the candidate's, gathered one round ahead), so a round costs two gathers, not a chain
//     of dependent loads per sequence;
//   * the greedy parse (first verified position at or after the end of the previous match)
//     is a scalar walk of one readlane per sequence over successors that every lane has
//     worked out for itself; only matches longer than 28 bytes go back to memory (64 bytes
//     per wave step);
//   * a block whose first 2 KiB match well is probed at every second position from there on
//     (every position is still entered into the table); data that has stopped matching
//     altogether is probed at every eighth position until a match turns up;
//   * sequences are queued in LDS and emitted 64 at a time: a wave prefix sum places every
//     sequence, each lane writes its token, length bytes, literals and offset (LZ4 block
//     format, lz4.c:961-1073).
//
// The output is a valid LZ4 frame that the reference decoder
// (rd_kafka_lz4_decompress, rdkafka_lz4.c:167) decodes to the input; it is NOT
// byte-identical to the reference's frame (use the exact engine in
// lz4_encode.hip for that).  The compression ratio is pinned against the
// reference's by tests/test_gpu_lz4.py (north_star: within 5 %).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "crc_wave.h"
#include "lz4_finish_wave.h"
#include "lz4_device.h"
#include "lz4_engine.h"
#include "lz4_wave.h"

namespace rdk {

void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s, const FuseCrc *fuse);

namespace {

constexpr int kFastMaxItems = 64;              // block slots per frame per pass
constexpr uint32_t kFastSlot = kLz4Block + 4;  // worst-case bytes per block in a frame
constexpr uint32_t kFastHashLog = 12;
#ifndef RDK_FAST_PAIRS
#define RDK_FAST_PAIRS 3
#endif
#ifndef RDK_FAST_MAXDIST
#define RDK_FAST_MAXDIST 65535
#endif
constexpr int kFastMaxDist = RDK_FAST_MAXDIST;  // candidates farther back are not looked at
constexpr int kFastPairs = RDK_FAST_PAIRS;     // dword pairs behind the 4 verified bytes
constexpr int kFastLen = 4 + 8 * kFastPairs;   // match bytes measured from registers
constexpr int kWinDwords = 3 + 2 * kFastPairs; // 4 catch-up bytes, the position's dword pair, the pairs
static_assert(kFastPairs == 2 || kFastPairs == 3, "window loads are written for 7 or 9 dwords");

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef __attribute__((address_space(1))) const u32x4a g_cu32x4a;
typedef __attribute__((address_space(1))) const u32x2a g_cu32x2a;

__device__ __forceinline__ uint32_t hash4(uint32_t seq) {  // LZ4_hash4, lz4.c:631
  return (seq * 2654435761u) >> (32 - kFastHashLog);
}

constexpr uint32_t kShortLit = 16;  // literal runs copied by their own lane
#ifndef RDK_FAST_SPARSE
#define RDK_FAST_SPARSE 1  // 0: data that stops matching stays at one probe per position (A/B runs)
#endif
constexpr int kSparse = 8;      // stride of the rounds over data that has stopped matching
constexpr int kColdRounds = 16;  // dense rounds without a verified match before they start (1 KiB)

struct BlockCtx {
  uintptr_t src, dst;
  rsrc_t r;            // the block's dwords
  rsrc_t w;            // the block's output slot (byte stores; parked lanes write nothing)
  uint32_t sa;         // src & 3: byte offset of position 0 inside the resource
  int n, mfl, mlim, olimit;
  int p;               // parse position == anchor (end of the last match)
  int op;              // output bytes written
  int qn;              // sequences queued in LDS (flush_sequences)
  int rend;            // positions at or past it belong to the next phase: not entered yet
  int nseq, mbytes;    // sequences so far; match bytes so far, a partial sum per lane (the stride decision)
  bool full;           // the block does not fit in olimit bytes: nothing more is written
  int cold;            // rounds in a row without a single verified match (dense rounds)
  bool sparse;         // the rounds in progress are the sparse ones
  bool trig;           // this run of rounds was told to end (rend pulled in): the mode changes
  int back;            // where the dense rounds resume after the sparse ones
};

// Per round the lane's own 36-byte window (Win, loaded three rounds ahead),
// and its candidate with the candidate's window (Cand, gathered one round
// ahead).
struct Win {
  uint32_t d[kWinDwords];
};
struct Cand {
  uint32_t t[kWinDwords];
  int c;       // the table's entry for the lane's position
  uint64_t m;  // lanes whose candidate was gathered (t holds zeros in the others)
};

// The block's LDS: the hash table, one spare entry that parked lanes read and write (an
// unconditional LDS access needs no EXEC change, and the code around it stays one basic
// block that the scheduler can arrange), and the queue of finished sequences.
constexpr uint32_t kTableEntries = 1u << kFastHashLog;
typedef uint32_t u32x2q __attribute__((ext_vector_type(2)));  // a queued sequence
struct __attribute__((aligned(16))) FastLds {
  uint16_t table[kTableEntries + 8];
  u32x2q queue[64];
};
typedef __attribute__((address_space(3))) u32x2q lds_u2;

// kWinDwords dwords at block offset a-4 (a 4-aligned).  Nine dwords: load9.  Seven dwords:
// two loads, 16 bytes from a-4 and 12 from a+12.  A load that starts below the resource
// reads as zero as a whole, so a window at a == 0 (the block's first dword) is not usable:
// win_usable() keeps those positions out of the match search, as position and as candidate
// (they are still hashed and entered; an entry that points at one is rejected).
__device__ __forceinline__ void load_win(rsrc_t r, uint32_t a, uint32_t *d) {
  if constexpr (kWinDwords == 9) {
    load9(r, a, d);
  } else {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u3 __attribute__((ext_vector_type(3)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, a - 4u, 0, 0);
    const u3 w = __builtin_amdgcn_raw_buffer_load_b96(r, a + 12u, 0, 0);
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    d[4] = w.x; d[5] = w.y; d[6] = w.z;
  }
}
__device__ __forceinline__ bool win_usable(uint32_t a) { return kWinDwords == 9 || a != 0u; }

// S = stride of the probed positions: lane l of the round at R stands at R + S * l.  With
// S == 2 every position is still hashed and entered, but only the even ones are looked up,
// gathered and measured; a match that starts on an odd position is found one byte later
// and grown back by the catch-up.
template <int S>
__device__ __forceinline__ void round_load(const BlockCtx &b, Win &x, int R, int lane) {
  const int i = R + S * lane;
  load_win(b.r, i <= b.mfl ? ((uint32_t(i) + b.sa) & ~3u) : kNoLoad, x.d);
}

// Lookup, first half: hash + table for the round at R (window x.d arrived).  All 64 lanes
// store their position in one ds_write_b16; where several hit the same entry the highest
// lane -- the latest position -- is the one that lands (measured on gfx950; a fixed order
// either way, so the output is deterministic).  Returns the entry read; the caller uses it
// only after other work (round_gather), so the LDS round trip is not waited for.
template <int S>
__device__ __forceinline__ int round_lookup(const BlockCtx &b, const Win &x, int R, lds_u16 *table,
                                            int lane) {
  const int i = R + S * lane;
  const bool act = i <= b.mfl && i < b.rend;
  const uint32_t shi = (uint32_t(i) + b.sa) & 3u;
  const uint32_t h = act ? hash4(__builtin_amdgcn_alignbyte(x.d[2], x.d[1], shi)) : kTableEntries;
  const int c = int(table[h]);
  table[h] = uint16_t(i);
  if (S == 2) {  // the odd position behind it: entered, never looked up
    const bool act1 = i + 1 <= b.mfl && i + 1 < b.rend;
    const bool wrap = shi == 3u;  // its four bytes start in the next dword
    const uint32_t lo = wrap ? x.d[2] : x.d[1], hi = wrap ? x.d[3] : x.d[2];
    const uint32_t h1 = act1 ? hash4(__builtin_amdgcn_alignbyte(hi, lo, (shi + 1u) & 3u)) : kTableEntries;
    table[h1] = uint16_t(i + 1);
  }
  return c;
}

// Lookup, second half: issue the candidate gather for the lanes the parse may still need
// (i >= p).
template <int S>
__device__ __forceinline__ void round_gather(const BlockCtx &b, Cand &y, int c, int R, int lane) {
  const int i = R + S * lane;
  const uint32_t ai = (uint32_t(i) + b.sa) & ~3u, ac = (uint32_t(c) + b.sa) & ~3u;
  const bool ok = i <= b.mfl && i < b.rend && i >= b.p && c < i && i - c <= kFastMaxDist &&
                  win_usable(ai) && win_usable(ac);
  y.c = c;
  y.m = ballot(ok);
  load_win(b.r, ok ? ac : kNoLoad, y.t);
}

// Write out the queued sequences (entry q < qn: literal start | literal length << 16,
// offset | matchlength-4 << 16): every lane writes its own token, literals, offset and length
// bytes at a wave-prefix-sum position.  A block that does not fit in olimit bytes sets b.full
// and writes nothing from then on (the caller stores it raw).
//
// The call ends with every load and store of its own retired.  It runs once in several rounds
// behind a branch; without that wait the compiler has to assume, where the branch joins the
// round again, that the call's loads may still be pending on registers the round reuses, and
// drains the round's own loads (the windows and candidates fetched ahead) in every round.
__device__ __forceinline__ void flush_sequences(BlockCtx &b, lds_u2 *queue, int lane) {
  const bool ch = lane < b.qn;
  asm volatile("" ::: "memory");  // (the entries were stored by other lanes)
  const u32x2q e = queue[lane];
  const uint32_t lstart = e.x & 0xFFFFu, lit = ch ? e.x >> 16 : 0u;
  const uint32_t off = e.y & 0xFFFFu, mc = e.y >> 16;
  const uint32_t lext = ext_bytes(lit);
  const uint32_t sz = ch ? 3u + lit + lext + ext_bytes(mc) : 0u;
  uint32_t tot;
  const uint32_t o = wave_excl_scan(sz, tot);
  // keep room for the shortest possible last-literals token (lz4.c:1146)
  // (wave-uniform, and said to be: the rounds' control flow must stay on the scalar unit)
  if (__builtin_amdgcn_readfirstlane(int(b.full || b.op + int(tot) + 1 > b.olimit))) {
    b.full = true;
    b.qn = 0;
    return;
  }
  const uint32_t tp = uint32_t(b.op) + o;  // token position in the block output
  const uint32_t lp = tp + 1u + lext;      // first literal
  const uint32_t fp = lp + lit;            // offset field
  __builtin_amdgcn_raw_buffer_store_b8(
      uint8_t(((lit < 15u ? lit : 15u) << 4) | (mc < 15u ? mc : 15u)), b.w, ch ? tp : kNoLoad, 0, 0);
  // offset (LE16) and a single match-length byte (15 <= mc < 270)
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off), b.w, ch ? fp : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off >> 8), b.w, ch ? fp + 1u : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(mc - 15u), b.w,
                                       (ch && mc >= 15u && mc < 270u) ? fp + 2u : kNoLoad, 0, 0);
  // rare shapes, each behind a wave-uniform test
  if (ballot(ch && lit >= 15u)) {  // literal length bytes: 255-runs + remainder
    if (ch && lit >= 15u) put_len(b.dst + tp + 1u, lit);
  }
  if (ballot(ch && mc >= 270u)) {
    if (ch && mc >= 270u) put_len(b.dst + fp + 2u, mc);
  }
  const bool need_win = ch && lit != 0u && lit <= kShortLit;
  if (ballot(need_win)) {  // up to 16 literals: one 20-byte window per lane
    uint32_t w[5];
    load5(b.r, need_win ? ((lstart + b.sa) & ~3u) : kNoLoad, w);
    const uint32_t sh = (lstart + b.sa) & 3u;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
#pragma unroll
    for (uint32_t k = 0; k < kShortLit; ++k)
      __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v[k >> 2] >> (8u * (k & 3u))), b.w,
                                           (need_win && k < lit) ? lp + k : kNoLoad, 0, 0);
  }
  // long literal runs: the whole wave copies them one at a time
  uint64_t longm = ballot(ch && lit > kShortLit);
  while (longm) {
    const int j = __builtin_ctzll(longm);
    longm &= longm - 1;
    const uint32_t jl = __builtin_amdgcn_readlane(lit, j);
    const uint32_t jp = __builtin_amdgcn_readlane(lp, j);
    const uint32_t js = __builtin_amdgcn_readlane(lstart, j);
    wave_copy_bytes(b.dst + jp, b.src + js, jl, lane);
  }
  b.op += int(tot);
  b.qn = 0;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
}

// What round_measure hands to round_walk.
struct Meas {
  uint64_t vm;  // lanes with a verified match (MINMATCH bytes equal at a gathered candidate)
  int len;      // match bytes measured from the register windows, clamped to the block
  uint32_t shi, shc;
};

// Measure the round's matches (windows arrived): vector work only.
template <int S>
__device__ __forceinline__ Meas round_measure(const BlockCtx &b, const Win &x, const Cand &y, int R,
                                              int lane) {
  const int i = R + S * lane;
  Meas m;
  m.shi = (uint32_t(i) + b.sa) & 3u;
  m.shc = (uint32_t(y.c) + b.sa) & 3u;
  const uint32_t shi = m.shi, shc = m.shc;
  // (positions before the parse position need no exclusion here: the walk starts at it and
  // only moves forward.  One compare per lane mask: a predicate combined from several goes
  // through a 0/1 register and a second compare)
  m.vm = ballot(__builtin_amdgcn_alignbyte(x.d[2], x.d[1], shi) ==
                __builtin_amdgcn_alignbyte(y.t[2], y.t[1], shc)) & y.m;
  // first differing bit behind the 4 verified bytes: trailing-zero counts over dword pairs
  // (64 exactly when a pair is equal: only then the next pair counts)
  uint32_t cz[kFastPairs];
#pragma unroll
  for (int k = 0; k < kFastPairs; ++k) {
    const uint32_t z0 = __builtin_amdgcn_alignbyte(x.d[2 * k + 3], x.d[2 * k + 2], shi) ^
                        __builtin_amdgcn_alignbyte(y.t[2 * k + 3], y.t[2 * k + 2], shc);
    const uint32_t z1 = __builtin_amdgcn_alignbyte(x.d[2 * k + 4], x.d[2 * k + 3], shi) ^
                        __builtin_amdgcn_alignbyte(y.t[2 * k + 4], y.t[2 * k + 3], shc);
    const uint64_t w = (uint64_t(z1) << 32) | z0;
    cz[k] = w ? uint32_t(__builtin_ctzll(w)) : 64u;
  }
  uint32_t fd = cz[kFastPairs - 1];
#pragma unroll
  for (int k = kFastPairs - 2; k >= 0; --k) fd = cz[k] + __umul24(cz[k] >> 6, fd);  // (a full-rate multiply)
  fd >>= 3;
  m.len = 4 + int(fd < uint32_t(kFastLen - 4) ? fd : uint32_t(kFastLen - 4));
  if (m.len > b.mlim - i) m.len = b.mlim - i;
  return m;
}

// Walk the greedy parse over the measured round (scalar: one readlane per sequence), then
// queue the chosen sequences: every chosen lane stores its sequence's fields at its rank in
// the LDS queue; flush_sequences writes them out 64 at a time.
template <int S>
__device__ __forceinline__ void round_walk(BlockCtx &b, const Win &x, const Cand &y, const Meas &m,
                                           int R, lds_u2 *queue, int lane) {
  const int i = R + S * lane;
  const int rel_lane = S * lane;  // this lane's position relative to R
  // (the parse position is wave-uniform; saying so keeps the walk below on the scalar unit
  // in every instantiation -- left to the compiler's analysis, the stride-2 one ran it as a
  // divergent vector loop, 2.5 times the vector instructions per round)
  const int p0 = __builtin_amdgcn_readfirstlane(b.p);
  const uint64_t vm = m.vm;
  int len = m.len;
  if constexpr (S == kSparse) {
    // A sparse round takes no match: the first one it sees ends the sparse rounds, and the
    // dense rounds resume at the start of the round BEFORE this one -- a match seen here has
    // its candidate from an earlier round at the latest, so the data may have begun to match
    // anywhere in the round before -- and parse from there position by position.  (The
    // positions the sparse rounds have entered find themselves in the table then and go
    // without a candidate: one in eight.)
    const int f0 = ((p0 - R > 0 ? p0 - R : 0) + S - 1) / S;
    if (f0 < 64 && (vm >> f0)) {
      b.rend = min(b.rend, R + 64 * S);
      b.back = max(R - 64 * S, b.back);  // (b.back: where these sparse rounds began)
      b.trig = true;
    }
    return;
  }

  // Greedy walk: first verified position at or after the end of the last match.  Every lane
  // works out its own successor (the first verified lane at or past the end of its match), so
  // the scalar walk is one readlane per sequence; only a match that fills the register
  // window is continued from memory, and its successor found from its final length.
  const int fl = (rel_lane + len + S - 1) / S;  // first lane at or past this lane's match end
  const uint64_t longm = vm & ballot(len == kFastLen) & ballot(i + kFastLen < b.mlim);
  // a lane's successor, as the walk reads it: its lane number, + 64 when that lane holds a
  // long match (the walk stops there to measure it), 128 when there is none in this round
  const auto encode = [&](uint64_t ahead, int first) {  // ahead = vm >> first
    const int t = first + int(__builtin_ctzll(ahead));
    return ahead ? t + int(((longm >> (t & 63)) & 1ull) << 6) : 128;
  };
  const int succ = encode(uint32_t(fl) < 64u ? vm >> fl : 0ull, fl);
  const int xin = p0 - R;
  uint64_t chosen = 0;
  const int fl0 = ((xin > 0 ? xin : 0) + S - 1) / S;
  int q = __builtin_amdgcn_readfirstlane(encode(fl0 < 64 ? vm >> fl0 : 0ull, fl0));
  for (;;) {
    while (q < 64) {
      chosen |= 1ull << q;
      q = __builtin_amdgcn_readlane(succ, q);
    }
    if (q >= 128) break;
    q -= 64;  // long match: continue from memory
    chosen |= 1ull << q;
    const int qi = R + S * q;
    const int off = qi - __builtin_amdgcn_readlane(y.c, q);
    const int L = __builtin_amdgcn_readfirstlane(
        kFastLen + wave_count_fwd(b.src + uint32_t(qi + kFastLen),
                                  b.src + uint32_t(qi - off + kFastLen),
                                  b.mlim - qi - kFastLen, lane));
    if (lane == q) len = L;
    const int f2 = (S * q + L + S - 1) / S;
    q = __builtin_amdgcn_readfirstlane(encode(f2 < 64 ? vm >> f2 : 0ull, f2));
  }
  // Data without matches (already compressed, encrypted) is not worth 64 probes per 64
  // positions: after kColdRounds rounds in a row without one verified match the block goes
  // on at every kSparse-th position -- what the reference's growing search step does
  // (lz4.c:886).  The change takes effect by pulling the end of this run of rounds in to the
  // end of the NEXT round, whose positions the lookup ahead has already entered: the loop
  // then drains by itself.  (Only the position-by-position rounds count: a block that has
  // earned the stride of two matches well, and its rounds keep their loop bound in a
  // register.)
  if (!chosen) {
    if constexpr (S == 1 && RDK_FAST_SPARSE) {
      if (!vm && xin < 64 * S && ++b.cold == kColdRounds) {
        b.rend = min(b.rend, R + 2 * 64 * S);
        b.trig = true;
      }
    }
    return;
  }
  if constexpr (S == 1) b.cold = 0;
  const int lastq = 63 - int(__builtin_clzll(chosen));
  b.p = R + S * lastq + __builtin_amdgcn_readlane(len, lastq);

  const bool ch = __builtin_amdgcn_inverse_ballot_w64(chosen);
  const int cnt = __builtin_popcountll(chosen);
  if constexpr (S == 1) {  // what the stride decision reads (per-lane partial sums)
    b.nseq += cnt;
    b.mbytes += ch ? len : 0;
  }
  // this sequence's anchor (relative): the end of the previous chosen match -- match ends
  // grow with the lane, so that is the running maximum over the lanes below -- or, for the
  // round's first sequence, the end of the last round's last match
  const int pm = wave_excl_max(ch ? rel_lane + len : 0);
  const int prev = pm > 0 ? pm : xin;
  const uint32_t xb = __builtin_amdgcn_alignbyte(x.d[1], x.d[0], m.shi) ^
                      __builtin_amdgcn_alignbyte(y.t[1], y.t[0], m.shc);
  int bk = xb ? int(__builtin_clz(xb) >> 3) : 4;  // catch-up bytes (lz4.c:957)
  bk = min(bk, min(rel_lane - prev, y.c));        // literals only, inside the block
  const uint32_t lit = uint32_t(rel_lane - bk - prev);
  const uint32_t mc = uint32_t(len + bk) - 4u;
  const uint32_t off = uint32_t(i - y.c);
  const uint32_t lstart = uint32_t(R + prev);  // absolute literal start
  b.qn = __builtin_amdgcn_readfirstlane(b.qn);  // (wave-uniform: keeps the count in a scalar register)
  if (b.qn + cnt > 64) flush_sequences(b, queue, lane);
  const int rank = int(__builtin_amdgcn_mbcnt_hi(uint32_t(chosen >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(uint32_t(chosen), 0u)));
  if (ch) queue[b.qn + rank] = u32x2q{lstart | (lit << 16), off | (mc << 16)};
  b.qn += cnt;
}

// One pipelined step: the table lookup of the next round and the window of the round three
// ahead are issued first; round R is measured while the LDS answers; then the next round's
// candidate gather goes out, and round R is walked and queued.  Every load is issued
// unconditionally (parked lanes read nothing), so the compiler's waits stay exact, and the
// stores of a flush never sit between a load and its first use (vmcnt counts loads and
// stores together).
template <int S>
__device__ __forceinline__ void round_step(BlockCtx &b, const Win &cur, Win &next, Win &far,
                                           const Cand &ccur, Cand &cnext, int R, FastLds *lds,
                                           int lane) {
  const int c = round_lookup<S>(b, next, R + 64 * S, (lds_u16 *)lds->table, lane);
  round_load<S>(b, far, R + 192 * S, lane);
  const Meas m = round_measure<S>(b, cur, ccur, R, lane);
  __builtin_amdgcn_sched_barrier(0);  // (the scheduler would pull the gather, and its wait for the LDS, up front)
  round_gather<S>(b, cnext, c, R + 64 * S, lane);
  round_walk<S>(b, cur, ccur, m, R, (lds_u2 *)lds->queue, lane);
}

// The rounds of [r0, b.rend) at stride S (r0 a multiple of 64 * S; positions past mfl are
// parked).  The pipeline is primed at r0 and drains at the end: positions at or past b.rend
// are loaded ahead but not entered into the table.  A block that turns out not to fit
// (b.full) is parsed to its end all the same, writing nothing: such a block has few matches,
// hence few sequences, and is rarely found out before its last flush anyway, while an exit
// from inside a round joins the round's path and costs every round a wait for all the loads
// in flight (the compiler cannot tell at the join which of them the exit left pending).
template <int S>
__device__ __forceinline__ void fast_rounds(BlockCtx &b, FastLds *lds, int r0, int lane) {
  constexpr int kSpan = 64 * S;
  // the last position that starts a round's work (b.rend may be pulled in by a round, see
  // round_walk; wave-uniform, and said to be, so that the loop's control stays scalar)
  const int last_fixed = min(b.mfl, b.rend - 1);
  const auto last_pos = [&] {
    if constexpr (S == 2) return last_fixed;
    else return min(b.mfl, __builtin_amdgcn_readfirstlane(b.rend) - 1);
  };
  if (r0 > last_pos()) return;
  Win W0, W1, W2, W3;
  Cand C0, C1;
  round_load<S>(b, W0, r0, lane);
  round_load<S>(b, W1, r0 + kSpan, lane);
  round_load<S>(b, W2, r0 + 2 * kSpan, lane);
  round_gather<S>(b, C0, round_lookup<S>(b, W0, r0, (lds_u16 *)lds->table, lane), r0, lane);
  for (int R = r0; R <= last_pos(); R += 4 * kSpan) {
    round_step<S>(b, W0, W1, W3, C0, C1, R, lds, lane);
    if (R + kSpan > last_pos()) break;
    round_step<S>(b, W1, W2, W0, C1, C0, R + kSpan, lds, lane);
    if (R + 2 * kSpan > last_pos()) break;
    round_step<S>(b, W2, W3, W1, C0, C1, R + 2 * kSpan, lds, lane);
    if (R + 3 * kSpan > last_pos()) break;
    round_step<S>(b, W3, W0, W2, C1, C0, R + 3 * kSpan, lds, lane);
  }
}

// The first kProbe positions of a block are probed one by one; if the matches found there
// average kStride2MinMatch bytes or more, the rest of the block is probed at every second
// position.  Long matches survive that unharmed (a match that starts on a skipped position
// is picked up one byte later and grown back), short ones do not: on text whose matches are
// 4 to 6 bytes long, probing every second position costs 8 % of the ratio, on the JSON
// records 2 %, for a third more speed -- so the block's own first matches decide.
#ifndef RDK_FAST_STRIDE2
#define RDK_FAST_STRIDE2 1
#endif
#ifndef RDK_FAST_PROBE
#define RDK_FAST_PROBE 2048
#endif
constexpr int kProbe = RDK_FAST_PROBE;  // a multiple of 128
constexpr int kStride2MinMatch = 9;

// Compress one block of n (>= 13) bytes at src into dst (capacity n-1).
// Returns the compressed size, or 0 when it does not fit (stored raw).
__device__ int fast_block(uintptr_t src, int n, uintptr_t dst, FastLds *lds, int lane) {
  BlockCtx b;
  b.src = src;
  b.dst = dst;
  const uintptr_t lo = src & ~uintptr_t(3);
  b.r = block_rsrc(lo, (src + uint32_t(n) + 3u) & ~uintptr_t(3));
  b.w = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(dst), 0, n, 0x00020000);
  b.sa = uint32_t(src & 3u);
  b.n = n;
  b.mfl = n - kLz4MFLimit;        // last position a match may start (lz4.c:907)
  b.mlim = n - kLz4LastLiterals;  // matchlimit (lz4.c:822)
  b.olimit = n - 1;               // LZ4F_makeBlock dstCapacity
  b.p = b.op = 0;
  b.qn = 0;
  b.nseq = b.mbytes = 0;
  b.full = false;

  b.sparse = b.trig = false;
  b.back = 0;
  int S = 1;                        // stride of the dense rounds
  bool decided = !RDK_FAST_STRIDE2;  // ... once the block's first kProbe positions have decided it
  for (int r0 = 0;;) {
    if (!decided && r0 >= kProbe) {
      decided = true;
      const int nseq = __builtin_amdgcn_readfirstlane(b.nseq);
      uint32_t mbytes;
      wave_excl_scan(uint32_t(b.mbytes), mbytes);
      if (nseq > 0 && int(mbytes) >= kStride2MinMatch * nseq) S = 2;
    }
    b.rend = (!decided && !b.sparse) ? kProbe : n;
    b.cold = 0;
    b.back = r0;
    if (b.sparse) fast_rounds<kSparse>(b, lds, r0, lane);
    else if (S == 2) fast_rounds<2>(b, lds, r0, lane);
    else fast_rounds<1>(b, lds, r0, lane);
    const int rend = __builtin_amdgcn_readfirstlane(b.rend);
    if (__builtin_amdgcn_readfirstlane(int(b.full)) || rend >= n || b.mfl < rend) break;
    r0 = rend;
    if (__builtin_amdgcn_readfirstlane(int(b.trig))) {
      // (out of the sparse rounds: back to the start of the round that saw a match)
      if (b.sparse) r0 = __builtin_amdgcn_readfirstlane(b.back);
      b.sparse = !b.sparse;
    }
    b.trig = false;
  }
  flush_sequences(b, (lds_u2 *)lds->queue, lane);
  if (b.full) return 0;
  // last literals (lz4.c:1141-1166)
  const uint32_t last = uint32_t(n - b.p);
  if (b.op + 1 + int(ext_bytes(last)) + int(last) > b.olimit) return 0;
  if (lane == 0) {
    uintptr_t p0 = dst + uint32_t(b.op);
    stb(p0++, (last < 15u ? last : 15u) << 4);
    if (last >= 15u) put_len(p0, last);
  }
  const int op = b.op + 1 + int(ext_bytes(last));
  wave_copy_bytes(dst + uint32_t(op), src + uint32_t(b.p), last, lane);
  return op + int(last);
}

// (four waves per SIMD: the measured optimum; the bound also keeps the register count there)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void lz4_fast_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t *__restrict__ out_lens, uint32_t n,
    FuseCrc fuse) {
  __shared__ FastLds lds;
  uint16_t *table_mem = lds.table;
  const int lane = threadIdx.x;
  // block slots per frame per pass: 64, or the largest block count of any frame when the
  // caller had it found (FuseCrc::max_nb)
  uint32_t slots = uint32_t(kFastMaxItems);
  if (fuse.max_nb) {
    const uint32_t m = uni(*fuse.max_nb);
    slots = m < 1u ? 1u : (m < slots ? m : slots);
  }
  const uint64_t items = uint64_t(n) * slots;
  for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
    // slot-major items: all frames' block 0, then all block 1, ...  The blocks that exist
    // come first and are dense in blockIdx, so they spread over every XCD, shader engine
    // and CU (a frame-major order parks the missing blocks of short frames in a periodic
    // pattern that leaves half of the shader engines idle)
    const uint32_t f = uint32_t(it % n), kk = uint32_t(it / n);
    const uint32_t len = uni(in_lens[f]);
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    for (uint32_t k = kk; k < nb; k += slots) {
      const uint32_t bn = (len - k * kLz4Block) < kLz4Block ? (len - k * kLz4Block) : kLz4Block;
      const uintptr_t src = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kLz4Block;
      const uintptr_t slot = reinterpret_cast<uintptr_t>(out) + out_offs[f] + 7u + uint64_t(k) * kFastSlot;
      int csize = 0;
      if (bn >= uint32_t(kLz4MFLimit + 1)) {
        typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) u32x4e lds_u4;
        lds_u4 *t4 = (lds_u4 *)table_mem;
        const u32x4e z = {0u, 0u, 0u, 0u};
        for (int x = lane; x < int((2u << kFastHashLog) / 16u); x += 64) t4[x] = z;
        asm volatile("" ::: "memory");
        csize = fast_block(src, int(bn), slot + 4u, &lds, lane);
      }
      const uint32_t w = csize ? uint32_t(csize) : (bn | 0x80000000u);  // LZ4F_makeBlock
      if (lane == 0) {
        stb(slot, w & 0xFFu); stb(slot + 1, (w >> 8) & 0xFFu);
        stb(slot + 2, (w >> 16) & 0xFFu); stb(slot + 3, w >> 24);
      }
      if (fuse.block_crc && k < uint32_t(kFastMaxItems)) {
        // the compress epilogue's CRC (lz4_finish_wave.h); the byte tables go into the hash
        // table's LDS, dead until the next block
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        wave_block_epilogue(uni(w), slot, src, k, nb, f, reinterpret_cast<uintptr_t>(out) + out_offs[f],
                            reinterpret_cast<uintptr_t>(in) + in_offs[f], len, out_lens, fuse,
                            (crcw_lds_u32 *)table_mem, lane);
      }
    }
  }
}

}  // namespace

int lz4f_compress_units_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                               const uint32_t *d_in_lens, uint8_t *d_out,
                               const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                               hipStream_t s, const FuseCrc *fuse);

// RDK_HIP_LZ4_FAST_ENGINE=units makes the throughput entry points (and the producer's FAST
// mode) run the workgroup-per-block engine of lz4_encode_units.hip instead of this file's
// one-wavefront-per-block engine (A/B runs; rdk_hip_lz4f_compress_units always runs it).
bool lz4f_fast_engine_is_units() {
  static const bool units = [] {
    const char *e = getenv("RDK_HIP_LZ4_FAST_ENGINE");
    return e && e[0] == 'u';
  }();
  return units;
}

int lz4f_compress_fast_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                              const uint32_t *d_in_lens, uint8_t *d_out,
                              const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                              hipStream_t s, const FuseCrc *fuse) {
  if (!n) return 0;
  if (lz4f_fast_engine_is_units())
    return lz4f_compress_units_device(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n,
                                      s, fuse);
  const uint64_t items = uint64_t(n) * kFastMaxItems;
  const unsigned grid = unsigned(items < 2560u * 8u ? items : 2560u * 8u);
  FuseCrc fz = fuse ? *fuse : FuseCrc();
  fz.single_done = fz.block_crc != nullptr;
  // (without a caller's spare word: d_out_lens is not written before the assembler runs)
  if (!fuse && n > kMaxNbFrames) fz.max_nb = d_out_lens;
  if (fz.max_nb) lz4f_max_blocks_launch(d_in_lens, n, fz.max_nb, s);
  hipLaunchKernelGGL(lz4_fast_blocks_kernel, dim3(grid), dim3(64), 0, s, d_in, d_in_offs,
                     d_in_lens, d_out, d_out_offs, d_out_lens, n, fz);
  lz4f_assemble_launch(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, s,
                       fuse ? &fz : nullptr);
  RDK_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace rdk
