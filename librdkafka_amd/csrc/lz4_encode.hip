// lz4_encode.hip -- LZ4F frame compression on gfx950.
//
// Replaces rd_kafka_lz4_compress (src/rdkafka_lz4.c:329-442) ->
// LZ4F_compressUpdate/End (lz4frame.c:823-1018) -> LZ4F_makeBlock (:739) ->
// LZ4_compress_fast_extState_fastReset (lz4.c:1211) -> LZ4_compress_generic
// (lz4.c:789-1177, byU16 table, limitedOutput, dstCapacity = srcSize-1).
//
// One wavefront (one 64-thread workgroup) per independent 64 KiB block with
// its own 8192-entry u16 hash table (16 KiB) and a 4 KiB source ring in LDS
// (8 blocks per CU).  The greedy parse is emulated EXACTLY, so frames are
// byte-identical to the reference's.  Two engines:
//
//  * window_block() (acceleration 1, i.e. compression.level 0..2): the parse runs
//    in WINDOWS of 64 consecutive positions, one per lane.  Every lane loads its
//    own 36 source bytes and its table candidate's 36 bytes once, verifies
//    MINMATCH, measures the match (up to 28 bytes, extended to 92 from the ring)
//    and the catch-up (up to 4) from registers.  The sequential loop's path over
//    those per-lane results -- which positions are probed and inserted, the first
//    verifying probe, catch-up, ip-2 insertion and the immediate re-test after a
//    match (lz4.c:1084-1134) -- is then the orbit of the entry lane under "next
//    verified lane behind this lane's match", hopped on the scalar unit over per-lane
//    results (the parallel walk); windows outside the conditions under
//    which that shortcut is exact are replayed one sequence at a time (the scalar
//    walk).  A candidate inserted earlier in the same window is found with a
//    hash-equality mask over the lanes.  Several sequences per window cost two
//    gathers, not a chain of dependent loads each; their bytes are emitted
//    together at wave-prefix-sum positions.  Searches that outlast the stride-1
//    probes (lz4.c:896-905) continue in generic_search().
//
//  * compress_block() (acceleration > 1, negative compression.level): one
//    sequence at a time, every step through memory:
//   * the match search evaluates 64 consecutive probe positions at once
//     (the skip schedule step = searchMatchNb++ >> 6 is reproduced by a lane
//     prefix-sum); each lane's candidate is the latest earlier probe with the
//     same hash (13 ballots, one per hash bit) or else the table entry; the
//     first verifying lane wins and only probes up to it update the table,
//     last-writer-per-hash, as the sequential loop would;
//   * catch-up, LZ4_count and literal copies compare / move 64 bytes per step;
//   * the limitedOutput checks of lz4.c:961-1160 are applied verbatim, so a
//     block that does not fit in srcSize-1 bytes is stored raw (bit 31) like
//     LZ4F_makeBlock does.
// Blocks are written into worst-case slots of the caller's frame buffer;
// lz4f_assemble_kernel then writes the frame header / size words / end mark
// and slides the blocks down into stream order.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "crc_wave.h"
#include "lz4_device.h"
#include "lz4_engine.h"
#include "lz4_wave.h"
#include "lz4_finish_wave.h"
#include "win_ring.h"

#ifdef RDK_WIN_PROF
#define RDK_PT(k) do { const uint64_t now_ = __builtin_amdgcn_s_memtime(); b.pt[k] += now_ - tprev_; tprev_ = now_; } while (0)
#else
#define RDK_PT(k) do { } while (0)
#endif

namespace rdk {

constexpr int kEncMaxItems = 64;           // block slots per frame per pass
constexpr uint32_t kSlot = kLz4Block + 4;  // worst-case bytes per block in a frame
constexpr uint32_t kHashLog = 13;          // LZ4_HASHLOG+1 for byU16 (lz4.c:633)

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lz4_hash(uint32_t seq) {  // LZ4_hash4, lz4.c:631
  return (seq * 2654435761u) >> (32 - kHashLog);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d);
    if (lane >= d) v += t;
  }
  return v;
}

// number of equal bytes a[i]==b[i] for i in [0, limit), 64 per step
__device__ __forceinline__ int wave_count(uintptr_t a, uintptr_t b, int limit, int lane) {
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

// catch-up: equal bytes walking backwards from a-1 / b-1, at most limit
__device__ __forceinline__ int wave_count_back(uintptr_t a, uintptr_t b, int limit, int lane) {
  int cnt = 0;
  while (cnt < limit) {
    const int l = cnt + lane;
    const bool ok = l < limit && ldb(a - 1 - l) == ldb(b - 1 - l);
    const uint64_t m = ballot(ok);
    const int run = m == ~0ull ? 64 : __builtin_ctzll(~m);
    cnt += run;
    if (run < 64) break;
  }
  return cnt;
}

__device__ __forceinline__ void wave_copy(uintptr_t d, uintptr_t s, uint32_t len, int lane) {
  for (uint32_t base = 0; base < len; base += 256u) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + lane + 64u * j;
      v[j] = ldb(s + (i < len ? i : len - 1u));  // (clamped, not predicated)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + lane + 64u * j;
      if (i < len) stb(d + i, v[j]);
    }
  }
}

// n bytes of 255 followed by one `rest` byte at d (length extension bytes)
__device__ __forceinline__ void put_run(uintptr_t d, uint32_t n255, uint32_t rest, int lane) {
  for (uint32_t i = lane; i < n255; i += 64u) stb(d + i, 255u);
  if (lane == 0) stb(d + n255, rest);
}

// LZ4_compress_generic(byU16, limitedOutput, noDict, noDictIssue), table
// already zeroed.  Returns compressed size, or 0 if it does not fit in n-1.
__device__ int compress_block(uintptr_t src, int n, uintptr_t dst, int accel, lds_u16 *table,
                              int lane) {
  const int mflimitPlusOne = n - kLz4MFLimit + 1;  // lz4.c:821
  const int matchlimit = n - kLz4LastLiterals;     // lz4.c:822
  const int olimit = n - 1;                        // LZ4F_makeBlock dstCapacity
  const uint32_t A64 = uint32_t(accel) << 6;       // searchMatchNb start
  int ip = 1, anchor = 0, op = 0, match = 0;

  // position 0 hashes to the zero entry it already holds (lz4.c:879)
  for (;;) {
    // ------------------------------------------------ find a match (lz4.c:909-957)
    {
      int fwd = ip;
      uint32_t cbase = 0;
      for (;;) {
        const uint32_t c = cbase + uint32_t(lane);
        const uint32_t s = (c == 0) ? 1u : ((A64 + c - 1u) >> 6);
        const uint32_t incl = wave_incl_scan(s, lane);
        const int P = fwd + int(incl - s);
        const int Pn = fwd + int(incl);
        const bool valid = Pn <= mflimitPlusOne;
        const uint64_t vmask = ballot(valid);
        const uint32_t seq = valid ? ld32u(src + uint32_t(P)) : 0u;
        const uint32_t h = lz4_hash(seq);
        uint64_t eq = same_value_lanes<int(kHashLog)>(h, vmask);
        const uint64_t lower = eq & ((1ull << lane) - 1ull);
        const int pred = lower ? 63 - __builtin_clzll(lower) : 0;
        const int predP = __shfl(P, pred);
        int cand = lower ? predP : int(table[h]);
        const bool m = valid && ld32u(src + uint32_t(cand)) == seq;
        const uint64_t mm = ballot(m);
        const int f = ffs64(mm);
        const int e = ffs64(~vmask);
        if (f < e) {
          const uint64_t upto = (2ull << f) - 1ull;
          const uint64_t later = eq & ~((2ull << lane) - 1ull) & upto;
          if (lane <= f && !later) table[h] = uint16_t(P);
          ip = __builtin_amdgcn_readlane(P, f);
          match = __builtin_amdgcn_readlane(cand, f);
          break;
        }
        if (e < 64) goto last_literals;  // forwardIp > mflimitPlusOne
        {
          const uint64_t later = eq & ~((2ull << lane) - 1ull);
          if (!later) table[h] = uint16_t(P);
        }
        fwd = __builtin_amdgcn_readlane(Pn, 63);
        cbase += 64u;
      }
    }
    // ------------------------------------------------ catch up (lz4.c:958-959)
    {
      const int lim = (ip - anchor) < match ? (ip - anchor) : match;
      const int back = wave_count_back(src + uint32_t(ip), src + uint32_t(match), lim, lane);
      ip -= back;
      match -= back;
    }
    uint32_t token_at, token;
    // ------------------------------------------------ literals (lz4.c:961-988)
    {
      const uint32_t litLength = uint32_t(ip - anchor);
      token_at = uint32_t(op++);
      if (op + int(litLength) + (2 + 1 + kLz4LastLiterals) + int(litLength / 255u) > olimit)
        return 0;
      if (litLength >= 15u) {
        const uint32_t len = litLength - 15u;
        put_run(dst + uint32_t(op), len / 255u, len % 255u, lane);
        op += int(len / 255u) + 1;
        token = 15u << 4;
      } else {
        token = litLength << 4;
      }
      wave_copy(dst + uint32_t(op), src + uint32_t(anchor), litLength, lane);
      op += int(litLength);
    }
    for (;;) {  // _next_match (lz4.c:990-1135)
      const uint32_t offset = uint32_t(ip - match);
      if (lane == 0) {
        stb(dst + uint32_t(op), offset & 0xFFu);
        stb(dst + uint32_t(op) + 1, offset >> 8);
      }
      op += 2;
      const int mc0 = wave_count(src + uint32_t(ip + kLz4MinMatch),
                                 src + uint32_t(match + kLz4MinMatch),
                                 matchlimit - (ip + kLz4MinMatch), lane);
      uint32_t matchCode = uint32_t(mc0);
      ip += mc0 + kLz4MinMatch;
      if (op + (1 + kLz4LastLiterals) + int((matchCode + 240u) / 255u) > olimit) return 0;
      if (matchCode >= 15u) {
        token += 15u;
        matchCode -= 15u;
        put_run(dst + uint32_t(op), matchCode / 255u, matchCode % 255u, lane);
        op += int(matchCode / 255u) + 1;
      } else {
        token += matchCode;
      }
      if (lane == 0) stb(dst + token_at, token);
      anchor = ip;
      if (ip >= mflimitPlusOne) goto last_literals;  // lz4.c:1081
      // fill table with ip-2, then test the next position (lz4.c:1084-1134)
      const uint32_t h2 = lz4_hash(ld32u(src + uint32_t(ip - 2)));
      if (lane == 0) table[h2] = uint16_t(ip - 2);
      const uint32_t seq = ld32u(src + uint32_t(ip));
      const uint32_t h = lz4_hash(seq);
      const int mi = int(uni(table[h]));
      if (lane == 0) table[h] = uint16_t(ip);
      if (ld32u(src + uint32_t(mi)) == seq) {
        token_at = uint32_t(op++);
        token = 0;
        match = mi;
        continue;
      }
      ip++;
      break;
    }
  }

last_literals : {  // lz4.c:1141-1166
  const uint32_t lastRun = uint32_t(n - anchor);
  if (op + int(lastRun) + 1 + int((lastRun + 255u - 15u) / 255u) > olimit) return 0;
  if (lastRun >= 15u) {
    if (lane == 0) stb(dst + uint32_t(op), 15u << 4);
    op++;
    const uint32_t acc = lastRun - 15u;
    put_run(dst + uint32_t(op), acc / 255u, acc % 255u, lane);
    op += int(acc / 255u) + 1;
  } else {
    if (lane == 0) stb(dst + uint32_t(op), lastRun << 4);
    op++;
  }
  wave_copy(dst + uint32_t(op), src + uint32_t(anchor), lastRun, lane);
  op += int(lastRun);
}
  return op;
}

// ===================================================================== windows
// The search loop of lz4.c:909-957 from probe index `cbase` at position `fwd`, 64 probes
// per step (strides above 1 included).  true: a probe verified, P / cand are set and the
// table holds every probe up to P; false: forwardIp passed mflimitPlusOne (last literals).
__device__ __forceinline__ bool generic_search(uintptr_t src, int mflimitPlusOne, uint32_t A64,
                                               int fwd, uint32_t cbase, lds_u16 *table,
                                               int lane, int &P_out, int &cand_out) {
  for (;;) {
    const uint32_t c = cbase + uint32_t(lane);
    const uint32_t s = (c == 0) ? 1u : ((A64 + c - 1u) >> 6);
    const uint32_t incl = wave_incl_scan(s, lane);
    const int P = fwd + int(incl - s);
    const int Pn = fwd + int(incl);
    const bool valid = Pn <= mflimitPlusOne;
    const uint64_t vmask = ballot(valid);
    // (a valid probe and every table entry have 12 block bytes behind them: the branch-free
    // 8-byte reads stay inside; a load under a lane predicate would be waited for at once)
    const uint32_t sv = ld32u_nb(src + uint32_t(valid ? P : 0));
    const uint32_t seq = valid ? sv : 0u;
    const uint32_t h = lz4_hash(seq);
    uint64_t eq = same_value_lanes<int(kHashLog)>(h, vmask);
    const uint64_t lower = eq & ((1ull << lane) - 1ull);
    const int pred = lower ? 63 - __builtin_clzll(lower) : 0;
    const int predP = __shfl(P, pred);
    const int cand = lower ? predP : int(table[h]);
    const uint32_t cv = ld32u_nb(src + uint32_t(valid ? cand : 0));
    const bool m = valid && cv == seq;
    const uint64_t mm = ballot(m);
    const int f = ffs64(mm);
    const int e = ffs64(~vmask);
    if (f < e) {
      const uint64_t upto = (2ull << f) - 1ull;
      const uint64_t later = eq & ~((2ull << lane) - 1ull) & upto;
      if (lane <= f && !later) table[h] = uint16_t(P);
      P_out = __builtin_amdgcn_readlane(P, f);
      cand_out = __builtin_amdgcn_readlane(cand, f);
      return true;
    }
    if (e < 64) return false;
    {
      const uint64_t later = eq & ~((2ull << lane) - 1ull);
      if (!later) table[h] = uint16_t(P);
    }
    fwd = __builtin_amdgcn_readlane(Pn, 63);
    cbase += 64u;
  }
}

constexpr int kRegLen = 28;   // match bytes a lane measures from its two register windows
constexpr int kMaxLen = 92;   // ... and with up to 64 more bytes from the source ring
constexpr int kRegBack = 4;   // catch-up bytes a lane measures from them
constexpr uint32_t kShortLit = 16;  // literal runs copied by their own lane

enum WinMode { W_SEARCH = 0, W_POSTMATCH = 1, W_FORCED = 2 };
enum WinStatus { W_CONTINUE = 0, W_LAST = 1, W_OVERFLOW = 2 };

struct WinBlock : SrcRing {  // + the block's source and its LDS ring (win_ring.h)
  uintptr_t dst;
  rsrc_t w;   // the block's output slot (byte stores; parked lanes write nothing)
  int n, mfl1, mlim, olimit;  // size, mflimitPlusOne, matchlimit, dstCapacity
  int ip;      // next probe (W_SEARCH) / end of the last match (W_POSTMATCH)
  int cnt;     // probes already made in the current search
  int anchor, op;
  int mode;    // how the next window starts
  uint32_t q0, q1;  // the sequence queue, one entry per lane (flush_sequences)
  int qn;           // entries queued
#ifdef RDK_WIN_PROF
  uint64_t pt[8], pn;
#endif
};

// Write out the queued sequences (lane q < qn holds one: literal start | literal length << 16,
// offset | matchlength-4 << 16): token, literal-length bytes, literals, offset and
// match-length bytes at wave-prefix-sum positions.  true: the block does not fit
// (limitedOutput).
__device__ __forceinline__ bool flush_sequences(WinBlock &b, int lane) {
  const bool ch = lane < b.qn;
  const uint32_t lstart = b.q0 & 0xFFFFu, lit = ch ? b.q0 >> 16 : 0u;
  const uint32_t off = b.q1 & 0xFFFFu, mc = b.q1 >> 16;
  const uint32_t lext = ext_bytes(lit);
  const uint32_t sz = ch ? 3u + lit + lext + ext_bytes(mc) : 0u;
  uint32_t tot;
  const uint32_t o = wave_excl_scan(sz, tot);
  const uint32_t tp = uint32_t(b.op) + o;  // token position in the block output
  const uint32_t lp = tp + 1u + lext;      // first literal
  const uint32_t fp = lp + lit;            // offset field
  // limitedOutput, lz4.c:964 (literals) and lz4.c:1044 (match length)
  const bool ov = ch && (int(tp + 1u + lit + (2u + 1u + kLz4LastLiterals) + lit / 255u) > b.olimit ||
                         int(fp + 2u + (1u + kLz4LastLiterals) + (mc + 240u) / 255u) > b.olimit);
  if (ballot(ov)) return true;
  __builtin_amdgcn_raw_buffer_store_b8(
      uint8_t(((lit < 15u ? lit : 15u) << 4) | (mc < 15u ? mc : 15u)), b.w, ch ? tp : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off), b.w, ch ? fp : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off >> 8), b.w, ch ? fp + 1u : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(mc - 15u), b.w,
                                       (ch && mc >= 15u && mc < 270u) ? fp + 2u : kNoLoad, 0, 0);
  // rare shapes, each behind a wave-uniform test
  if (ballot(ch && lit >= 15u)) {
    if (ch && lit >= 15u) put_len(b.dst + tp + 1u, lit);
  }
  if (ballot(ch && mc >= 270u)) {
    if (ch && mc >= 270u) put_len(b.dst + fp + 2u, mc);
  }
  // up to 16 literals: one 20-byte window per lane, from the ring while it still holds them
  const uint32_t la = (lstart + b.sa) & ~3u;
  const bool need_win = ch && lit != 0u && lit <= kShortLit && int(la) >= b.H - int(kRingBytes);
  if (ballot(need_win)) {
    uint32_t wv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      wv[k] = *(lds_u32 *)((lds_u8 *)b.ring + ((la + 4u * uint32_t(k)) & (kRingBytes - 1u)));
    const uint32_t sh = (lstart + b.sa) & 3u;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], sh);
#pragma unroll
    for (uint32_t k = 0; k < kShortLit; ++k)
      __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v[k >> 2] >> (8u * (k & 3u))), b.w,
                                           (need_win && k < lit) ? lp + k : kNoLoad, 0, 0);
  }
  uint64_t longm = ballot(ch && lit != 0u && !need_win);  // long runs: the whole wave copies them
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
  return false;
}

// One window of 64 positions from w0.  See the file comment; tests/sim/lz4_window_sim.cpp
// is the same walk with the lanes as arrays.
__device__ __forceinline__ int window_step(WinBlock &b, int w0, int forced_cand, lds_u16 *table,
                                           int lane) {
  const int mode = b.mode;
#ifdef RDK_WIN_PROF
  uint64_t tprev_ = __builtin_amdgcn_s_memtime();
  b.pn++;
#endif
  // ---------------------------------------------------------------- per lane
  const int i = w0 + lane;
  const bool act = i <= b.n - kLz4MFLimit;  // position + 1 <= mflimitPlusOne
  // the ring covers this window's own bytes (positions w0 .. w0+63 and 35 bytes beyond) and
  // the bytes a lane compares when it measures a match past its register window
  while (b.H < w0 + int(b.sa) + 64 + kMaxLen + 8) ring_fill(b, lane);
  uint32_t xd[9], yt[9];
  // (the window's 64 lanes read consecutive positions: all straight unless the window
  // straddles the end of the ring, one window in ~40)
  const uint32_t wb = (uint32_t(w0) + b.sa) & (kRingBytes - 1u);
  if (wb >= 4u && wb + 64u + 32u <= kRingBytes)
    ring_load9_straight(b, (uint32_t(i) + b.sa) & ~3u, xd);
  else
    ring_load9(b, (uint32_t(i) + b.sa) & ~3u, xd);
  const uint32_t shi = (uint32_t(i) + b.sa) & 3u;
  const uint32_t seq = __builtin_amdgcn_alignbyte(xd[2], xd[1], shi);
  const uint32_t h = lz4_hash(seq);
  RDK_PT(0);
  int tc = act ? int(table[h]) : 0;
  if (mode == W_FORCED && lane == 0) tc = forced_cand;
  // the candidate's 36 bytes: from the ring when it is that recent, else from memory
  const uint32_t ac = (uint32_t(tc) + b.sa) & ~3u;
  // (a candidate whose 36 bytes run over an end of the ring is fetched like a far one)
  const bool far = act && (int(ac) - 4 < b.H - int(kRingBytes) || !ring_straight(ac));
  ring_load9_straight(b, ac, yt);
  // (issued for every window -- parked lanes touch no memory -- and consumed behind the
  // hash comparison below, which then runs while the gather is in flight)
  uint32_t g[9];
  load9(b.r, far ? ac : kNoLoad, g);
  // lanes with the same hash (the candidate may be a position inserted in this window)
  const uint64_t ACT = ballot(act);
  uint64_t eq = same_value_lanes<int(kHashLog)>(h, ACT);
  if (!act) eq = 0;
  const uint64_t DUP = ballot((eq & ((1ull << lane) - 1ull)) != 0);
#pragma unroll
  for (int k = 0; k < 9; ++k) yt[k] = far ? g[k] : yt[k];
  const uint32_t shc = (uint32_t(tc) + b.sa) & 3u;
  const bool tver = act && seq == __builtin_amdgcn_alignbyte(yt[2], yt[1], shc);
  const uint64_t VT = ballot(tver);
  RDK_PT(1);
  // first differing bit behind the 4 hashed bytes: count of trailing zeros over dword pairs
  // (64 when a pair is equal), chained arithmetically -- no compare-and-select per dword
  uint32_t zz[6];
#pragma unroll
  for (int k = 1; k <= 6; ++k)
    zz[k - 1] = __builtin_amdgcn_alignbyte(xd[k + 2], xd[k + 1], shi) ^
                __builtin_amdgcn_alignbyte(yt[k + 2], yt[k + 1], shc);
  uint32_t cz[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint64_t w = (uint64_t(zz[2 * k + 1]) << 32) | zz[2 * k];
    cz[k] = w ? uint32_t(__builtin_ctzll(w)) : 64u;
  }
  // (a pair's count is 64 exactly when the pair is equal: only then the next pair counts)
  uint32_t fd = cz[1] + (cz[1] >> 6) * cz[2];
  fd = cz[0] + (cz[0] >> 6) * fd;
  fd >>= 3;
  int len = 4 + int(fd < uint32_t(kRegLen - 4) ? fd : uint32_t(kRegLen - 4));
  // a match that fills the register window is measured on from the ring, 4 bytes a step, up
  // to kMaxLen; `sat` = the length is still not final (kMaxLen reached, or a candidate older
  // than the ring) and has to be finished from memory if the parse takes this match
  bool more = tver && len == kRegLen && !far;
  if (ballot(more)) {
    const uint32_t vi = uint32_t(i) + b.sa, vc = uint32_t(tc) + b.sa;
#pragma unroll 1
    for (int j = 0; j < (kMaxLen - kRegLen) / 4; ++j) {
      if (!ballot(more)) break;
      const uint32_t pi = vi + uint32_t(len), pc = vc + uint32_t(len);
      lds_u8 *rb = (lds_u8 *)b.ring;
      const uint32_t a0 = *(lds_u32 *)(rb + (pi & (kRingBytes - 4u)));
      const uint32_t a1 = *(lds_u32 *)(rb + ((pi + 4u) & (kRingBytes - 4u)));
      const uint32_t c0 = *(lds_u32 *)(rb + (pc & (kRingBytes - 4u)));
      const uint32_t c1 = *(lds_u32 *)(rb + ((pc + 4u) & (kRingBytes - 4u)));
      const uint32_t z = __builtin_amdgcn_alignbyte(a1, a0, pi & 3u) ^
                         __builtin_amdgcn_alignbyte(c1, c0, pc & 3u);
      if (more) {
        len += z ? int(__builtin_ctz(z) >> 3) : 4;
        if (z) more = false;
      }
    }
  }
  RDK_PT(2);
  if (len > b.mlim - i) len = b.mlim - i;  // LZ4_count stops at matchlimit
  const bool sat = tver && i + len < b.mlim && (len == kMaxLen || (far && len == kRegLen));
  const uint32_t back = __builtin_amdgcn_alignbyte(xd[1], xd[0], shi);  // bytes i-4 .. i-1
  const uint32_t xb = back ^ __builtin_amdgcn_alignbyte(yt[1], yt[0], shc);
  int bkr = xb ? int(__builtin_clz(xb) >> 3) : kRegBack;
  if (bkr > tc) bkr = tc;  // nothing in front of the block
  const int NA = ~ACT ? __builtin_ctzll(~ACT) : 64;  // first lane that may not be probed

  // one readlane per sequence fetches the lane's candidate, match length and catch-up
  const uint32_t pk = uint32_t(tc) | (uint32_t(len) << 16) | (uint32_t(bkr) << 24) |
                      (sat ? 1u << 27 : 0u);
  const uint64_t VD = VT | DUP;  // lanes >= NA have neither bit

  // ------------------------------------------------------------- scalar walk
  // One loop iteration per sequence: the pending match (lz4.c:958-1081), then ip-2
  // insertion and the re-test of ip (lz4.c:1084-1134), then the search for the next match
  // (lz4.c:909-957).  The scalar unit is shared by the CU's waves, so the common path is
  // kept to a few dozen scalar instructions; lanes whose hash repeats inside the window
  // (DUP) take the slow lookup.
  const int anchor_in = b.anchor;
  uint64_t INS = 0, chosen = 0;
  int L_cand = 0, L_len = 0, L_bk = 0;  // per lane: the sequence whose match starts here
  int anchor = b.anchor, cnt = b.cnt;
  int q = 0, x = 0, cand = 0, ipn = 0;
  bool inwin = false, ver = false;
  int st = W_CONTINUE;
  b.mode = W_SEARCH;

  // candidate of lane lx given the inserts so far: the latest inserted lane of this window
  // with the same hash, else the table entry read when the window started
#define RDK_WIN_LOOKUP(lx)                                                                  \
  do {                                                                                      \
    const uint64_t eqx = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(eq >> 32), (lx)))) << 32) | \
                         uint32_t(__builtin_amdgcn_readlane(int(eq), (lx)));                \
    const uint64_t m_ = eqx & INS & bits_below(lx);                                         \
    if (m_) {                                                                               \
      const int j_ = 63 - __builtin_clzll(m_);                                              \
      cand = w0 + j_;                                                                       \
      inwin = true;                                                                         \
      ver = __builtin_amdgcn_readlane(int(seq), j_) == __builtin_amdgcn_readlane(int(seq), (lx)); \
    } else {                                                                                \
      inwin = false;                                                                        \
      ver = (VT >> (lx)) & 1ull;                                                            \
    }                                                                                       \
  } while (0)

  // ------------------------------------------------------------ parallel walk
  // Matches hop from one verified lane to the next: f(m) = first verified lane at or after
  // m + len[m]; the chosen lanes are the orbit of f from the entry (a match is at least 4
  // long, so at most 16 fit in a window).  This assumes
  // every candidate is the table's (no lane of this window supplies one); that and the rare
  // shapes (length or catch-up not final, strides above 1, end of block) are checked
  // afterwards, and the scalar walk below redoes the window when a check fails.
  bool fast_done = false;
  int seq_prev = 0;  // per lane: the anchor of a sequence that starts here
  if (NA == 64 && mode != W_FORCED) {
    const int e = mode == W_POSTMATCH ? 2 : 0;
    const int tl = lane + len;
    const uint64_t fm = tl >= 64 ? 0ull : VT & (~0ull << tl);
    const int J0 = fm ? __builtin_ctzll(fm) : 64;
    // the orbit of the entry lane under J0, hop by hop on the scalar unit: one v_readlane
    // and a handful of scalar instructions per match, a dependent chain far shorter than
    // the cross-lane shuffles of a pointer-doubling scheme
    const uint64_t em = VT & ~bits_below(e);
    uint64_t ch = 0;
    for (int pos = em ? __builtin_ctzll(em) : 64; pos < 64; pos = __builtin_amdgcn_readlane(J0, pos))
      ch |= 1ull << pos;
    // per lane: the end of the previous chosen match (0: none).  Chosen matches do not
    // overlap, so their ends grow with the lane: a running maximum, shifted by one lane.
    // The tests below are one vector compare each; their lane masks are combined on the
    // scalar unit (a ballot of a combined predicate goes through a 0/1 register).
    const bool isch = __builtin_amdgcn_inverse_ballot_w64(ch);
    const int mend = i + len;
    const int pend = wave_excl_max(isch ? mend : 0);
    // (a match never ends at position 0, and pend == i + 2 puts the re-test inside the
    // window exactly for lanes below 62)
    const uint64_t Mv = ballot(pend <= i) & (~0ull << e);  // not inside a chosen match
    uint64_t Tm = ballot(pend == i) & ~uint64_t(w0 == 0);
    uint64_t Rm = ballot(pend == i + 2) & bits_below(62);
    if (mode == W_POSTMATCH) {
      Tm |= 4ull;
      Rm |= 1ull;
    }
    const uint64_t ins = Mv | Rm;
    const int prev = pend > anchor_in ? pend : anchor_in;  // (a chosen end lies behind the anchor)
    const int blim = i - prev < tc ? i - prev : tc;  // lz4.c:958: ip>anchor, match>lowLimit
    const int fbk = bkr < blim ? bkr : blim;
    const uint64_t Blong = ballot(bkr == kRegBack) & ballot(blim > kRegBack);
    const uint64_t Bsat = ballot(sat), Bend = ballot(mend >= b.mfl1);
    const uint64_t Bdup = ballot((eq & ins & ((1ull << lane) - 1ull)) != 0);
    const uint64_t badm = (ch & (Blong | Bsat | Bend)) | (Mv & Bdup);
    const int x1 = ch ? __builtin_ctzll(ch) : 63;
#ifdef RDK_WIN_PROF
    if (ch & Blong) b.pt[7] += 1;
    if (ch & Bsat) b.pt[7] += 1ull << 16;
    if (Mv & Bdup) b.pt[7] += 1ull << 32;
    if (mode == W_SEARCH && b.cnt + x1 > 64) b.pt[7] += 1ull << 48;
#endif
    if (!badm && !(mode == W_SEARCH && b.cnt + x1 > 64)) {
      fast_done = true;
      seq_prev = prev;
      INS = ins;
      chosen = ch;
      L_cand = tc;
      L_len = len;
      L_bk = fbk;
      if (ch) {
        const int cl = 63 - __builtin_clzll(ch);
        const int end = cl + __builtin_amdgcn_readlane(len, cl);  // lane after the last match
        anchor = w0 + end;
        if (end >= 64) {
          b.ip = w0 + end;
          b.mode = W_POSTMATCH;
        } else {
          b.ip = w0 + 64;
          b.cnt = 63 - (63 - __builtin_clzll(Tm));  // probes after the last re-tested lane
        }
      } else {
        b.ip = w0 + 64;
        b.cnt = Tm ? 63 - (63 - __builtin_clzll(Tm)) : b.cnt + 64;
      }
    }
  }

  RDK_PT(3);
  if (!fast_done) {
  bool have = false;  // a verified match at lane x is pending
  bool post = false;  // a match just ended at ipn
  if (mode == W_POSTMATCH) {
    ipn = w0 + 2;
    post = true;
  } else if (mode == W_FORCED) {
    x = 0;  // lane 0's candidate was set to forced_cand above
    have = true;
  }
  for (;;) {
    if (have) {
      have = false;
      const int P = w0 + x;
      const uint32_t pkx = uint32_t(__builtin_amdgcn_readlane(int(pk), x));
      if (!inwin) cand = int(pkx & 0xFFFFu);
      const int blim = P - anchor < cand ? P - anchor : cand;  // lz4.c:958: ip>anchor, match>lowLimit
      int fl, bk;
      if (inwin) {
        fl = win_count_fwd(b, P + 4, cand + 4, b.mlim - (P + 4), lane);
        bk = wave_count_back(b.src + uint32_t(P), b.src + uint32_t(cand), blim, lane);
      } else {
        const int lx = int((pkx >> 16) & 0xFFu), bx = int((pkx >> 24) & 7u);
        fl = lx - 4;
        if (pkx & (1u << 27))  // length not final: finish it from the ring / memory
          fl += win_count_fwd(b, P + lx, cand + lx, b.mlim - P - lx, lane);
        bk = bx < blim ? bx : blim;
        if (bx == kRegBack && blim > kRegBack)
          bk = kRegBack + wave_count_back(b.src + uint32_t(P - kRegBack),
                                          b.src + uint32_t(cand - kRegBack), blim - kRegBack, lane);
      }
      if (lane == x) {
        L_cand = cand;
        L_len = 4 + fl;
        L_bk = bk;
      }
      chosen |= 1ull << x;
      ipn = P + 4 + fl;
      anchor = ipn;
      if (ipn >= b.mfl1) {  // lz4.c:1081
        st = W_LAST;
        break;
      }
      post = true;
    }
    if (post) {
      post = false;
      const int r = ipn - 2 - w0;
      if (r >= 62) {  // the re-test position lies beyond this window
        b.ip = ipn;
        b.mode = W_POSTMATCH;
        break;
      }
      x = r + 2;
      INS |= 5ull << r;  // LZ4_putPosition(ip-2), lz4.c:1084, and the re-tested ip itself
      if ((DUP >> x) & 1ull) {
        RDK_WIN_LOOKUP(x);
      } else {
        inwin = false;
        ver = (VT >> x) & 1ull;
      }
      if (ver) {  // immediate match: no literals, no catch-up (anchor == position)
        have = true;
        continue;
      }
      q = x + 1;
      cnt = 0;
    }
    // search from lane q, whose probe index is cnt; lanes from xlim on have strides above 1
    const int xlim = q + 65 - cnt;
    uint64_t cm = q < 64 ? VD & (~0ull << q) : 0ull;
    if (xlim < 64) cm &= bits_below(xlim);
    if (!cm) {  // no candidate left in this window
      int stop = NA;  // <= 64
      int why = NA < 64 ? 1 : 0;  // 1: last literals, 0: window end
      if (xlim <= stop) {         // 2: strides above 1 from here on
        stop = xlim;
        why = 2;
      }
      INS |= bits_range(q, stop);
      if (why == 1) {
        st = W_LAST;
      } else {
        b.ip = w0 + stop;
        b.cnt = cnt + (stop - q);
      }
      break;
    }
    x = __builtin_ctzll(cm);
    INS |= (~0ull << q) & ~(~1ull << x);  // lanes q..x are probed and inserted
    cnt += x + 1 - q;
    q = x + 1;
    if ((DUP >> x) & 1ull) {
      RDK_WIN_LOOKUP(x);
      have = ver;
    } else {  // x has no earlier lane with its hash: its table candidate verified (VT)
      inwin = false;
      have = true;
    }
  }
  }  // !fast_done
#undef RDK_WIN_LOOKUP

  RDK_PT(4);
  // ------------------------------------------------------------ table update
  // every inserted lane; the latest position per hash wins
  if (st != W_LAST) {
    const bool ins = __builtin_amdgcn_inverse_ballot_w64(INS);
    const uint64_t later = eq & INS & ~bits_below(lane + 1);
    if (ins && !later) table[h] = uint16_t(i);
    asm volatile("" ::: "memory");
  }
  RDK_PT(5);
  // ---------------------------------------------------------------- sequences
  // A window holds a handful of sequences, far fewer than lanes: they are queued, one per
  // lane of the queue registers, and written out 64 at a time (flush_sequences).
  {
    const bool ch = __builtin_amdgcn_inverse_ballot_w64(chosen);
    int prev = seq_prev;  // this sequence's anchor (the parallel walk has it already)
    if (!fast_done) {
      const uint64_t lowc = chosen & ((1ull << lane) - 1ull);
      const int pl = lowc ? 63 - __builtin_clzll(lowc) : lane;
      const int pend = __shfl(i + L_len, pl);  // end of the previous chosen match
      prev = lowc ? pend : anchor_in;
    }
    const uint32_t lit = uint32_t(i - L_bk - prev);
    const uint32_t mc = uint32_t(L_len + L_bk - 4);
    const uint32_t off = uint32_t(i - L_cand);
    const int cnt = __builtin_popcountll(chosen);
    if (cnt) {
      if (b.qn + cnt > 64 && flush_sequences(b, lane)) return W_OVERFLOW;
      // chosen lane -> queue lane qn + its rank among the chosen lanes: a forward permute
      // (scatter); the other lanes send to a lane outside the accepted range
      const int rank = int(__builtin_amdgcn_mbcnt_hi(uint32_t(chosen >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(uint32_t(chosen), 0u)));
      const int tgt = ch ? b.qn + rank : ((b.qn + cnt) & 63);
      const uint32_t r0 = uint32_t(__builtin_amdgcn_ds_permute(tgt << 2, int(uint32_t(prev) | (lit << 16))));
      const uint32_t r1 = uint32_t(__builtin_amdgcn_ds_permute(tgt << 2, int(off | (mc << 16))));
      const bool acc = lane >= b.qn && lane < b.qn + cnt;
      b.q0 = acc ? r0 : b.q0;
      b.q1 = acc ? r1 : b.q1;
      b.qn += cnt;
    }
  }
  b.anchor = anchor;
  RDK_PT(6);
  return st;
}

// LZ4_compress_generic(byU16, limitedOutput, acceleration 1) in windows; table already
// zeroed.  Returns the compressed size, or 0 when it does not fit in n-1 bytes.
__device__ int window_block(uintptr_t src, int n, uintptr_t dst, lds_u16 *table, lds_u32 *ring,
                            int lane) {
  WinBlock b;
  ring_init(b, src, uint32_t(n), ring, lane);
  b.dst = dst;
  b.w = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(dst), 0, n, 0x00020000);
  b.n = n;
  b.mfl1 = n - kLz4MFLimit + 1;
  b.mlim = n - kLz4LastLiterals;
  b.olimit = n - 1;  // LZ4F_makeBlock dstCapacity
  b.ip = 1;          // position 0 goes into the zero entry it already holds (lz4.c:879)
  b.cnt = 0;
  b.anchor = 0;
  b.op = 0;
  b.mode = W_SEARCH;
  b.q0 = b.q1 = 0;
  b.qn = 0;
#ifdef RDK_WIN_PROF
  for (int k = 0; k < 8; ++k) b.pt[k] = 0;
  b.pn = 0;
  const uint64_t tstart_ = __builtin_amdgcn_s_memtime();
#endif
  int forced = 0;
  for (;;) {
    int w0;
    if (b.mode == W_SEARCH && b.cnt > 64) {  // strides above 1: the search continues probe by probe
      int P, cand;
      if (!generic_search(src, b.mfl1, 1u << 6, b.ip, uint32_t(b.cnt), table, lane, P, cand)) break;
      asm volatile("" ::: "memory");
      b.mode = W_FORCED;
      forced = cand;
      w0 = P;
    } else {
      w0 = b.mode == W_POSTMATCH ? b.ip - 2 : b.ip;
    }
    const int st = window_step(b, w0, forced, table, lane);
    if (st == W_OVERFLOW) return 0;
    if (st == W_LAST) break;
  }
  if (flush_sequences(b, lane)) return 0;
#ifdef RDK_WIN_PROF
  if (lane == 0 && (blockIdx.x % 509) == 0)
    printf("WINPROF blk %u windows %llu total %llu | own %llu cand %llu ext %llu walk %llu scalar %llu table %llu emit %llu\n", blockIdx.x,
           (unsigned long long)b.pn, (unsigned long long)(__builtin_amdgcn_s_memtime() - tstart_), (unsigned long long)b.pt[0],
           (unsigned long long)b.pt[1], (unsigned long long)b.pt[2], (unsigned long long)b.pt[3], (unsigned long long)b.pt[4],
           (unsigned long long)b.pt[5], (unsigned long long)b.pt[6]);
  if (lane == 0 && (blockIdx.x % 509) == 0)
    printf("WINWHY blk %u longback %llu sat %llu inwin %llu stride %llu\n", blockIdx.x, (unsigned long long)(b.pt[7] & 0xFFFF),
           (unsigned long long)((b.pt[7] >> 16) & 0xFFFF), (unsigned long long)((b.pt[7] >> 32) & 0xFFFF),
           (unsigned long long)(b.pt[7] >> 48));
#endif
  // last literals (lz4.c:1141-1166)
  const uint32_t last = uint32_t(n - b.anchor);
  if (b.op + int(last) + 1 + int((last + 255u - 15u) / 255u) > b.olimit) return 0;
  if (lane == 0) {
    uintptr_t p0 = dst + uint32_t(b.op);
    stb(p0++, (last < 15u ? last : 15u) << 4);
    if (last >= 15u) put_len(p0, last);
  }
  const int op = b.op + 1 + int(ext_bytes(last));
  wave_copy_bytes(dst + uint32_t(op), src + uint32_t(b.anchor), last, lane);
  return op + int(last);
}

// One wavefront per block.  Block k of frame f goes to the worst-case slot
// at out_offs[f] + 7 + k*kSlot as [LE32 size word][payload]; a block stored
// raw gets only its size word (payload is taken from the input later).
// max over frames of ceil(len / 64 KiB), one workgroup
__global__ __launch_bounds__(1024) void lz4f_max_blocks_kernel(const uint32_t *__restrict__ in_lens,
                                                              uint32_t n, uint32_t *__restrict__ out) {
  __shared__ uint32_t part[16];
  uint32_t m = 0;
  for (uint32_t f = threadIdx.x; f < n; f += 1024u) {
    const uint32_t nb = (in_lens[f] + kLz4Block - 1) / kLz4Block;
    m = nb > m ? nb : m;
  }
  for (int d = 32; d; d >>= 1) {
    const uint32_t o = uint32_t(__shfl_xor(int(m), d));
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63u) == 0u) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) m = part[w] > m ? part[w] : m;
    *out = m;
  }
}

void lz4f_max_blocks_launch(const uint32_t *d_in_lens, uint32_t n, uint32_t *d_max_nb, void *stream) {
  hipLaunchKernelGGL(lz4f_max_blocks_kernel, dim3(1), dim3(1024), 0, static_cast<hipStream_t>(stream),
                     d_in_lens, n, d_max_nb);
}

template <bool WINDOWS>
__global__ __launch_bounds__(64) void lz4_compress_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t *__restrict__ out_lens, uint32_t n, int accel,
    FuseCrc fuse) {
  // the source ring (windowed engine) sits in front of the hash table
  constexpr uint32_t kRingLds = WINDOWS ? kRingBytes : 0u;
  __shared__ __attribute__((aligned(16))) uint8_t lds_mem[kRingLds + (2u << kHashLog)];
  uint16_t *table_mem = reinterpret_cast<uint16_t *>(lds_mem + kRingLds);
  lds_u16 *table = (lds_u16 *)table_mem;
  const int lane = threadIdx.x;
  // block slots per frame per pass: 64, or the largest block count of any frame when the
  // caller had it found (FuseCrc::max_nb)
  uint32_t slots = uint32_t(kEncMaxItems);
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
      const uintptr_t slot = reinterpret_cast<uintptr_t>(out) + out_offs[f] + 7u + uint64_t(k) * kSlot;
      int csize = 0;
      if (bn >= uint32_t(kLz4MFLimit + 1)) {  // LZ4_minLength: shorter blocks never fit
        // LZ4_prepareTable: a fresh zeroed byU16 table per block (lz4.c:739-785)
        typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) u32x4e lds_u4;
        lds_u4 *t4 = (lds_u4 *)table_mem;
        const u32x4e z = {0u, 0u, 0u, 0u};
        for (int i = lane; i < int((2u << kHashLog) / 16u); i += 64) t4[i] = z;
        asm volatile("" ::: "memory");
        csize = WINDOWS ? window_block(src, int(bn), slot + 4u, table, (lds_u32 *)lds_mem, lane)
                        : compress_block(src, int(bn), slot + 4u, accel, table, lane);
      }
      const uint32_t w = csize ? uint32_t(csize) : (bn | 0x80000000u);  // LZ4F_makeBlock
      if (lane == 0) {
        stb(slot, w & 0xFFu); stb(slot + 1, (w >> 8) & 0xFFu);
        stb(slot + 2, (w >> 16) & 0xFFu); stb(slot + 3, w >> 24);
      }
      if (fuse.block_crc && k < uint32_t(kEncMaxItems)) {
        // the compress epilogue's CRC (lz4_finish_wave.h); the byte tables go into the front
        // of the block's LDS, which is dead once the block is compressed
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the block's own stores are done
        wave_block_epilogue(uni(w), slot, src, k, nb, f, reinterpret_cast<uintptr_t>(out) + out_offs[f],
                            reinterpret_cast<uintptr_t>(in) + in_offs[f], len, out_lens, fuse,
                            (crcw_lds_u32 *)lds_mem, lane);
      }
    }
  }
}

// One workgroup per frame: header (lz4frame.c:671-701), size words, blocks
// slid down from their slots (raw blocks copied from the input), end mark.
// FIN: the frame sits 61 bytes into a MsgVersion 2 batch slot and the workgroup also
// finishes the batch (see FuseCrc): codec choice, header, CRC32C from the block registers.
// kAsmThreads: threads per workgroup.  1024 (16 KiB per read-then-write step of the slide)
// when there are few frames; 256 when there are thousands, which are then short: a frame's
// fixed work is a chain of dependent steps that keeps one workgroup busy for microseconds
// whatever its size, so what counts is how many frames are in flight per CU.
template <bool FIN, uint32_t kAsmThreads>
__global__ __launch_bounds__(kAsmThreads) void lz4f_assemble_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *out, const uint64_t *__restrict__ out_offs,
    uint32_t *__restrict__ out_lens, uint32_t n, FuseCrc fuse) {
  constexpr uint32_t kHdr = 61;  // RD_KAFKAP_MSGSET_V2_SIZE (rdkafka_proto.h:540)
  __shared__ uint32_t t0_mem[FIN ? 1024 : 1];  // the four byte tables; the first is T0
  __shared__ uint32_t s_w[64];
  __shared__ uint32_t s_sz[FIN ? 64 : 1];
  __shared__ uint32_t s_term[FIN ? 65 : 1];
  const int t = threadIdx.x;
  if (FIN) {
    for (uint32_t i = uint32_t(t); i < 1024u; i += kAsmThreads) t0_mem[i] = fuse.t0[i];
    __syncthreads();
  }
  crcw_lds_u32 *t0 = (crcw_lds_u32 *)t0_mem;
  for (uint32_t f = blockIdx.x; f < n; f += gridDim.x) {
    const uint32_t len = in_lens[f];
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    if (FIN && fuse.single_done && nb == 1u) continue;  // finished by the block kernel's wave
    const uintptr_t ob = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    const uintptr_t ib = reinterpret_cast<uintptr_t>(in) + in_offs[f];
    if (t == 0) {  // magic, FLG 0x60 (v01, independent), BD 0x40 (64 KB), HC 0x82
      stb(ob + 0, 0x04); stb(ob + 1, 0x22); stb(ob + 2, 0x4D); stb(ob + 3, 0x18);
      stb(ob + 4, 0x60); stb(ob + 5, 0x40); stb(ob + 6, 0x82);
    }
    uint64_t pos = 7;
    for (uint32_t k0 = 0; k0 < nb; k0 += 64u) {
      // the size words of the next 64 slots, one per thread, before any of those blocks
      // moves (a block's new place ends below the next slot, so it overwrites no size word
      // that is still to be read -- and none of a later group)
      const uint32_t kn = nb - k0 < 64u ? nb - k0 : 64u;
      __syncthreads();
      if (uint32_t(t) < kn) {
        const uintptr_t slot = ob + 7u + uint64_t(k0 + uint32_t(t)) * kSlot;
        s_w[t] = ldb(slot) | (ldb(slot + 1) << 8) | (ldb(slot + 2) << 16) | (ldb(slot + 3) << 24);
      }
      __syncthreads();
      for (uint32_t k = k0; k < k0 + kn; ++k) {
        const uintptr_t slot = ob + 7u + uint64_t(k) * kSlot;
        // (the same word in every thread: saying so keeps the addresses below in scalar registers)
        const uint32_t w = uint32_t(__builtin_amdgcn_readfirstlane(int(s_w[k - k0])));
        const bool raw = w & 0x80000000u;
        const uint32_t sz = w & 0x7FFFFFFFu;
        const uintptr_t from = raw ? ib + uint64_t(k) * kLz4Block : slot + 4u;
        const uintptr_t to = ob + pos + 4u;
        // (no barrier between blocks: block k + 1 is read from its own slot, which block k's
        // new place does not reach, and written behind the barrier of its own move)
        if (from != to) asm_slide<kAsmThreads>(to, from, sz, t);
        if (t == 0) {
          stb(ob + pos, w & 0xFFu); stb(ob + pos + 1, (w >> 8) & 0xFFu);
          stb(ob + pos + 2, (w >> 16) & 0xFFu); stb(ob + pos + 3, w >> 24);
          if (FIN && k < 64u) s_sz[k] = sz;
        }
        pos += 4u + sz;
      }
    }
    __syncthreads();
    const uint32_t flen = uint32_t(pos + 4u);
    if (t == 0) {
      stb(ob + pos, 0); stb(ob + pos + 1, 0); stb(ob + pos + 2, 0); stb(ob + pos + 3, 0);
      out_lens[f] = flen;
    }
    if (FIN) {
      // ---- rd_kafka_msgset_writer_compress's verdict (rdkafka_msgset_writer.c:1179-1187)
      // and finalize_MessageSet_v2_header (:1251-1295)
      const uintptr_t bo = ob - kHdr;                     // the batch slot
      const uintptr_t hdr = ib - kHdr;                    // the header the writer left
      const bool compressed = flen <= len;
      const uint32_t payload = compressed ? flen : len;
      __syncthreads();                                    // the frame is complete
      if (!compressed) asm_slide<kAsmThreads>(ob, ib, len, t);  // keep the records plain
      if (uint32_t(t) < kHdr) {
        uint32_t v = ldb(hdr + uint32_t(t));
        const uint32_t length = kHdr + payload - 12u;
        if (t >= 8 && t < 12) v = (length >> (8u * (3u - (uint32_t(t) - 8u)))) & 0xFFu;
        if (t == 22 && compressed) v |= 3u;               // Attributes |= RD_KAFKA_COMPRESSION_LZ4
        if (t >= 17 && t < 21) v = 0;
        stb(bo + uint32_t(t), v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      // ---- calc_crc_v2 (:1229-1246) over [21, 61 + payload) without re-reading the frame:
      // header bytes and LZ4F header through the byte table, then one term per block
      uint32_t crc;
      if (!fuse.block_crc) {
        // no block registers (the unit engine): the caller runs the batched CRC32C pass
        // over the finished batches behind this kernel
        crc = 0;
      } else if (compressed && nb <= 64u) {
        if (uint32_t(t) < nb) {
          uint32_t after = 4u;                            // the end mark
          for (uint32_t j = uint32_t(t) + 1u; j < nb; ++j) after += 4u + s_sz[j];
          s_term[t] = crcw_shift_lut(fuse.block_crc[size_t(f) * 64u + uint32_t(t)], after, fuse.x2n);
        } else if (t >= 64 && t < 128) {
          // the second wavefront: header bytes [21, 68) one per lane in a register, then the
          // byte-table chain over them (no memory access inside the chain)
          const uint32_t k = 21u + uint32_t(t - 64);
          const uint32_t hb = ldb(bo + (k < kHdr + 7u ? k : 21u));
          uint32_t r = ~0u;                               // crc32c()'s initial register
#pragma unroll
          for (int j = 0; j < int(kHdr + 7u - 21u); ++j)
            r = t0[(r ^ uint32_t(__builtin_amdgcn_readlane(int(hb), j))) & 0xFFu] ^ (r >> 8);
          if (t == 64) s_term[64] = crcw_shift_lut(r, flen - 7u, fuse.x2n);
        }
        __syncthreads();
        uint32_t r = s_term[64];
        for (uint32_t k = 0; k < nb; ++k) r ^= s_term[k];
        crc = ~r;
      } else {
        // plain records, or more blocks than registers were kept for: the workgroup's waves
        // run over the finished bytes, a slice each, and the slices combine by shifting
        constexpr uint32_t kWaves = kAsmThreads / 64u;
        const uint32_t total = kHdr - 21u + payload;
        const uint32_t wv = uint32_t(t) >> 6, ln = uint32_t(t) & 63u;
        const uint32_t per = ((total + kWaves - 1u) / kWaves + 15u) & ~15u;
        const uint32_t s0 = wv * per;
        const uint32_t sl = s0 >= total ? 0u : (total - s0 < per ? total - s0 : per);
        const uint32_t r = wave_crc_range(bo + 21u + s0, sl, wv == 0u, t0, fuse.x2n, int(ln));
        if (ln == 0u) s_term[wv] = sl || wv == 0u ? crcw_shift_lut(r, total - s0 - sl, fuse.x2n) : 0u;
        __syncthreads();
        uint32_t x = 0;
        for (uint32_t k = 0; k < kWaves; ++k) x ^= s_term[k];
        crc = ~x;
      }
      if (t == 0) {
        stb(bo + 17, crc >> 24); stb(bo + 18, (crc >> 16) & 0xFFu);
        stb(bo + 19, (crc >> 8) & 0xFFu); stb(bo + 20, crc & 0xFFu);
        fuse.batch_lens[f] = kHdr + payload;
        fuse.crcs[f] = crc;
      }
    }
    __syncthreads();
  }
}

size_t lz4f_compress_bound(size_t len) {
  const size_t nb = (len + kLz4Block - 1) / kLz4Block;
  return 7u + nb * size_t(kSlot) + 4u;
}

void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s, const FuseCrc *fuse = nullptr);

int lz4f_compress_device(Ctx *c, const uint8_t *d_in, const uint64_t *d_in_offs,
                         const uint32_t *d_in_lens, uint8_t *d_out, const uint64_t *d_out_offs,
                         uint32_t *d_out_lens, uint32_t n, int accel, hipStream_t s,
                         const FuseCrc *fuse) {
  (void)c;
  if (!n) return 0;
  FuseCrc fz = fuse ? *fuse : FuseCrc();
  fz.single_done = fz.block_crc != nullptr;
  // (without a caller's spare word: d_out_lens is not written before the assembler runs)
  if (!fuse && n > kMaxNbFrames) fz.max_nb = d_out_lens;
  if (fz.max_nb) lz4f_max_blocks_launch(d_in_lens, n, fz.max_nb, s);
  uint64_t items = uint64_t(n) * kEncMaxItems;
  const unsigned grid = unsigned(items < 2560u * 8u ? items : 2560u * 8u);
  // RDK_HIP_LZ4_EXACT_SEQ=1 keeps the sequence-at-a-time engine for acceleration 1 too
  // (A/B measurements of the same frames)
  static const bool seq_only = getenv("RDK_HIP_LZ4_EXACT_SEQ") && atoi(getenv("RDK_HIP_LZ4_EXACT_SEQ"));
  if (accel == 1 && !seq_only)
    hipLaunchKernelGGL(lz4_compress_blocks_kernel<true>, dim3(grid), dim3(64), 0, s, d_in,
                       d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, accel, fz);
  else
    hipLaunchKernelGGL(lz4_compress_blocks_kernel<false>, dim3(grid), dim3(64), 0, s, d_in,
                       d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, accel, fz);
  lz4f_assemble_launch(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, s,
                       fuse ? &fz : nullptr);
  RDK_HIP_CHECK(hipGetLastError());
  return 0;
}

void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s, const FuseCrc *fuse) {
  const FuseCrc fz = fuse ? *fuse : FuseCrc();
  if (n > 2048u) {  // thousands of frames: many small workgroups in flight
    const dim3 grid(n < 32768u ? n : 32768u), block(256);
    if (fuse)
      hipLaunchKernelGGL((lz4f_assemble_kernel<true, 256>), grid, block, 0, s, d_in, d_in_offs, d_in_lens,
                         d_out, d_out_offs, d_out_lens, n, fz);
    else
      hipLaunchKernelGGL((lz4f_assemble_kernel<false, 256>), grid, block, 0, s, d_in, d_in_offs, d_in_lens,
                         d_out, d_out_offs, d_out_lens, n, fz);
  } else {
    const dim3 grid(n), block(1024);
    if (fuse)
      hipLaunchKernelGGL((lz4f_assemble_kernel<true, 1024>), grid, block, 0, s, d_in, d_in_offs, d_in_lens,
                         d_out, d_out_offs, d_out_lens, n, fz);
    else
      hipLaunchKernelGGL((lz4f_assemble_kernel<false, 1024>), grid, block, 0, s, d_in, d_in_offs, d_in_lens,
                         d_out, d_out_offs, d_out_lens, n, fz);
  }
}

int lz4f_compress_fast_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                              const uint32_t *d_in_lens, uint8_t *d_out,
                              const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                              hipStream_t s, const FuseCrc *fuse);
int lz4hc_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, int level, hipStream_t s);
int lz4f_compress_units_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                               const uint32_t *d_in_lens, uint8_t *d_out,
                               const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                               hipStream_t s, const FuseCrc *fuse);

}  // namespace rdk

using namespace rdk;


RDK_API size_t rdk_hip_lz4f_compress_bound(size_t len) { return lz4f_compress_bound(len); }

RDK_API int rdk_hip_lz4f_compress(const void *d_in, const uint64_t *d_in_offs,
                                  const uint32_t *d_in_lens, void *d_out,
                                  const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                                  int level, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_lens)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (level >= 3)  // LZ4F_selectCompression (lz4frame.c:797-805): LZ4HC (hash chain 3..9, optimal 10+)
    return lz4hc_compress_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                 static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n, level, s);
  const int accel = level < 0 ? -level + 1 : 1;  // LZ4F_compressBlock, lz4frame.c:766
  return lz4f_compress_device(c, static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                              static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n, accel, s,
                              nullptr);
}

RDK_API int rdk_hip_lz4f_compress_fast(const void *d_in, const uint64_t *d_in_offs,
                                       const uint32_t *d_in_lens, void *d_out,
                                       const uint64_t *d_out_offs, uint32_t *d_out_lens,
                                       uint32_t n, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_lens)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  return lz4f_compress_fast_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                   static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n,
                                   static_cast<hipStream_t>(stream), nullptr);
}

RDK_API int rdk_hip_lz4f_compress_units(const void *d_in, const uint64_t *d_in_offs,
                                        const uint32_t *d_in_lens, void *d_out,
                                        const uint64_t *d_out_offs, uint32_t *d_out_lens,
                                        uint32_t n, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_lens)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  return lz4f_compress_units_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                    static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n,
                                    static_cast<hipStream_t>(stream), nullptr);
}
