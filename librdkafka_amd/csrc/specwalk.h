// specwalk.h -- speculative parallel walk of a length-prefixed record chain (shared by the
// MsgVersion 0/1 message walk, legacy.hip, and the MsgVersion 2 record index, records.hip).
//
// A MessageSet / record batch is a chain: record p is [p, next(p)) and the next one starts
// where it ends, so finding the records is inherently sequential; one wave walking it one
// LDS round trip per record runs at ~0.1 B/clk/CU.  Here a whole 512-thread workgroup
// works on one chain, a 130 KiB LDS window at a time, and discovers it SPECULATIVELY in
// parallel:
//
//   A. every thread owns a 260-byte segment of the window and scans it (format-specific,
//      Fmt::scan) for the first position that looks like a record start; thread 0's
//      segment starts at the window base, which is a true record start;
//   B. from its guess each thread walks the chain to the first position past its segment
//      (its "exit"), classifying every record exactly as the reference reader does
//      (Fmt::classify);
//   C. thread l links to thread m when its exit lies in m's segment AND equals m's guess.
//      Links only go forward, so binary lifting (10 levels of pointer doubling in LDS)
//      tells every thread, in O(log) steps, whether it lies on the path from thread 0 --
//      i.e. whether its guess is a true record start.  The heuristic only decides speed,
//      never results: a wrong or missing guess ends the verified path there, and the next
//      window starts at the last verified exit (thread 0 is always exact, so every window
//      advances);
//   D. a block prefix sum over the verified threads' record counts numbers the rows and
//      every verified thread emits its own records (Emit) from LDS, while the next
//      window's loads are in flight.
// A record larger than the window is handled by Big (format-specific).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rdk {
namespace spec {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint8_t lds_b;
typedef __attribute__((address_space(3))) uint32_t lds_w;

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
// bytes scanned per thread: 65 dwords, so the 64 lanes of a wave, which scan in lockstep
// from the same offset of their segments, hit 64 different LDS banks (a 256-byte stride
// put them all in one bank)
constexpr uint32_t kSeg = 260;
constexpr uint32_t kWin = kThreads * kSeg;  // LDS window (130 KiB)
constexpr int kLev = 10;                    // 2^10 >= kThreads hops
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kV = int((kWin + kThreads * 16 - 1) / (kThreads * 16));  // 16-byte loads / thread

// classification of the record at p
enum : uint32_t { kOk = 0, kDone = 1, kPartial = 2, kErr = 3, kCut = 4 };  // kCut: not whole in the window

struct Shared {
  __attribute__((aligned(16))) uint8_t win[kWin + 64];
  uint16_t J[kLev][kThreads];
  uint32_t cand[kThreads];
  uint32_t wsum[kWaves];
  uint32_t term[2];  // exit and class of the path's last thread
  uint32_t err;      // first failing row found while emitting
};

struct Win {
  const lds_b *w;           // window byte q (chain offset) is w[q - base]
  uint32_t base, end, len;  // staged [base, end) of the chain's [0, len)
  __device__ __forceinline__ uint32_t b(uint32_t q) const { return w[q - base]; }
  // big-endian u32 at any q: two aligned LDS dwords and one v_alignbyte
  __device__ __forceinline__ uint32_t be32(uint32_t q) const {
    const uint32_t i = uint32_t(reinterpret_cast<uintptr_t>(w + (q - base)));
    const lds_w *a = reinterpret_cast<const lds_w *>(w + (q - base) - (i & 3u));
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(a[1], a[0], i & 3u));
  }
  // 16-byte aligned window start and the LDS index offset (index of q = q + off)
  __device__ __forceinline__ const lds_b *w0() const {
    return w - (uint32_t(reinterpret_cast<uintptr_t>(w)) & 15u);
  }
  __device__ __forceinline__ uint32_t off() const {
    return (uint32_t(reinterpret_cast<uintptr_t>(w)) & 15u) - base;
  }
};

// per byte: 0x80 where the byte is zero / nonzero / even
__device__ __forceinline__ uint32_t zb(uint32_t x) {
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t nzb(uint32_t x) {
  return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t evb(uint32_t x) { return (~x << 7) & 0x80808080u; }

// First q in [s0, lim) with pre() marking it and full(q) true, or kNone.  pre(D, k) gives
// the 0x80-per-byte survivor mask of candidates i+4k..i+4k+3 from the sliding run of
// aligned LDS dwords D[j] = bytes i+4j..i+4j+3 (j < 10).  Sixteen candidates per step,
// four new dwords per step loaded a step ahead.  Rounds: every lane first advances (no
// dependent loads) to its next surviving candidate, then all lanes run the full test
// together, so the wave pays one full test per round rather than one per step in which
// any lane has a survivor.
template <class Pre, class Full>
__device__ __forceinline__ uint32_t scan(const Win &W, uint32_t s0, uint32_t lim, Pre pre,
                                         Full full) {
  const lds_b *w0 = W.w0();
  const uint32_t off = W.off();
  auto W32 = [&](uint32_t i) { return *reinterpret_cast<const lds_w *>(w0 + i); };
  uint32_t i = (s0 + off) & ~3u;
  const uint32_t ie = lim + off;
  uint32_t D[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) D[k] = W32(i + 4u * k);
  uint64_t mlo = 0, mhi = 0;  // survivors of candidates mi..mi+7 / mi+8..mi+15
  uint32_t mi = i;
  for (;;) {
    while (!(mlo | mhi) && i < ie) {
      uint32_t N[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) N[k] = W32(i + 40u + 4u * k);  // next step's D[6..9]
      uint32_t g[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = pre(D, k);
      mlo = g[0] | (uint64_t(g[1]) << 32);
      mhi = g[2] | (uint64_t(g[3]) << 32);
      mi = i;
      i += 16u;
#pragma unroll
      for (int k = 0; k < 6; ++k) D[k] = D[k + 4];
#pragma unroll
      for (int k = 0; k < 4; ++k) D[6 + k] = N[k];
    }
    if (!(mlo | mhi)) break;
    uint32_t bit;
    if (mlo) {
      bit = uint32_t(__builtin_ctzll(mlo));
      mlo &= mlo - 1u;
    } else {
      bit = 64u + uint32_t(__builtin_ctzll(mhi));
      mhi &= mhi - 1u;
    }
    const uint32_t q = mi + 4u * (bit >> 5) + ((bit & 31u) >> 3) - off;
    if (q >= s0 && q < lim && full(q)) return q;
  }
  return kNone;
}

#ifdef RDK_LG_PROF  // phase timing (A/B builds only): s_memtime cycles summed over blocks
static __device__ unsigned long long g_lg_prof[8];  // per translation unit
#define SPEC_T(i)                                                        \
  do {                                                                   \
    __syncthreads();                                                     \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();          \
    if (t == 0) atomicAdd(&::rdk::spec::g_lg_prof[i], _n - prof_t);      \
    prof_t = _n;                                                         \
  } while (0)
#else
#define SPEC_T(i) do { } while (0)
#endif

// The driver.  Returns the record count, or -(1+k) for the first failing record k.
//   Fmt::scan(W, s0, lim)        -> guess in [s0, lim) or kNone
//   Fmt::classify(W, p, next)    -> kOk (record [p, next) whole in the window), kDone (p is
//                                   the end), kPartial (stops, not an error), kErr, kWin
//   emit(W, c, k, rb)            -> emits the k records from c as rows rb.. (only rows
//                                   below cap); returns the first failing row or kNone
//   big(W, base, row, next)      -> the record at base, larger than the window, as row
//                                   `row`; false = it fails
template <class Fmt, class Emit, class Big>
__device__ int32_t walk(const uint8_t *chain, uint32_t len, uint32_t cap, Shared &S,
                        const Fmt &fmt, Emit emit, Big big) {
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  uint32_t pos = 0, nrow = 0;
  int32_t res = 0;
  bool run = true;
  u32x4 pv[kV];
  bool pref = false;
  auto issue = [&](uint32_t b0) {  // the window at b0 into pv (bytes past the chain read 0)
    const uintptr_t ga = reinterpret_cast<uintptr_t>(chain + b0);
    const uintptr_t al = ga & ~uintptr_t(15);
    const uint32_t sh0 = uint32_t(ga - al), av = len - b0;
    const uint32_t wl0 = av < kWin - sh0 ? av : kWin - sh0;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(al), 0,
                                                        int((sh0 + wl0 + 3u) & ~3u), 0x00020000);
#pragma unroll
    for (int it = 0; it < kV; ++it)
      pv[it] = __builtin_amdgcn_raw_buffer_load_b128(rs, (t + kThreads * it) * 16u, 0, 0);
  };
#ifdef RDK_LG_PROF
  unsigned long long prof_t = __builtin_amdgcn_s_memtime();
#endif
  while (run) {
    // ---- stage [base, end): 16-byte buffer loads from the aligned address below base
    // (issued during the previous window's emit phase when that window could tell where
    // this one starts), stored once the previous window's readers are done
    const uint32_t base = pos;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(chain + base)) & 15u;
    const uint32_t avail = len - base;
    const uint32_t wl = avail < kWin - sh ? avail : kWin - sh;
    if (!pref) issue(base);
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kV; ++it)
      if ((t + kThreads * it) * 16u < kWin)
        *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(
            (lds_b *)S.win + (t + kThreads * it) * 16u) = pv[it];
    if (t == 0) S.err = kNone;
    Win W;
    W.w = (const lds_b *)S.win + sh;
    W.base = base;
    W.end = base + wl;
    W.len = len;
    __syncthreads();
    SPEC_T(0);
    // ---- A: guess the first record start in this thread's segment
    const uint32_t s0 = base + t * kSeg, s1 = s0 + kSeg;
    uint32_t c = kNone;
    if (t == 0) {
      c = base;
    } else if (s0 < W.end) {
      c = fmt.scan(W, s0, s1 < W.end ? s1 : W.end);
    }
    S.cand[t] = c;
    SPEC_T(1);
    // ---- B: walk from the guess to the first position past the segment
    uint32_t x = c, k = 0, cls = kOk;
    if (c != kNone) {
      while (x < s1) {
        uint32_t nx = 0;
        cls = fmt.classify(W, x, nx);
        if (cls != kOk) break;
        x = nx;
        ++k;
      }
    }
    __syncthreads();
    SPEC_T(2);
    // ---- C: link to the thread whose guess is our exit; binary lifting from thread 0
    uint32_t nxt = t;
    if (c != kNone && cls == kOk && x < W.end) {
      const uint32_t m = (x - base) / kSeg;
      if (m < uint32_t(kThreads) && S.cand[m] == x) nxt = m;
    }
    S.J[0][t] = uint16_t(nxt);
    for (int lv = 1; lv < kLev; ++lv) {
      __syncthreads();
      S.J[lv][t] = S.J[lv - 1][S.J[lv - 1][t]];
    }
    __syncthreads();
    uint32_t cur = 0;
    for (int lv = kLev - 1; lv >= 0; --lv) {
      const uint32_t y = S.J[lv][cur];
      if (y <= t) cur = y;
    }
    const bool on = c != kNone && cur == t;
    if (on && S.J[kLev - 1][0] == t) {  // the path's last thread
      S.term[0] = x;
      S.term[1] = cls;
    }
    SPEC_T(3);
    // ---- D: number the rows (block exclusive scan of the verified counts), emit
    const uint32_t mine = on ? k : 0u;
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d);
      if (lane >= uint32_t(d)) inc += y;
    }
    if (lane == 63u) S.wsum[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < uint32_t(kWaves); ++w) {
      const uint32_t y = S.wsum[w];
      before += w < wv ? y : 0u;
      total += y;
    }
    const uint32_t rb = nrow + before + inc - mine;
    const uint32_t tx = S.term[0], tc = S.term[1];
    // the next window's start is known now: overlap its loads with the emit phase
    pref = nrow + total <= cap && tc != kDone && tc != kPartial && tc != kErr && tx != base &&
           tx < len;
    if (pref) issue(tx);
    if (on && k) {
      const uint32_t e = emit(W, c, k, rb);
      if (e != kNone) atomicMin(&S.err, e);
    }
    __syncthreads();
    SPEC_T(4);
#ifdef RDK_LG_PROF
    if (t == 0) atomicAdd(&g_lg_prof[6], 1ull);
    if (t == 0) atomicAdd(&g_lg_prof[7], (unsigned long long)(tx - base));
#endif
    const uint32_t err = S.err;
    nrow += total;
    if (err != kNone) {
      res = -(1 + int32_t(err));
      run = false;
    } else if (nrow > cap) {
      res = -(1 + int32_t(cap));
      run = false;
    } else if (tc == kDone || tc == kPartial) {
      res = int32_t(nrow);
      run = false;
    } else if (tc == kErr) {
      res = -(1 + int32_t(nrow));
      run = false;
    } else if (tx != base) {
      pos = tx;  // the verified path's exit: the next window starts there
    } else {
      // the record at base is larger than the window
      uint32_t nx = base;
      const bool ok = nrow < cap && big(W, base, nrow, nx);
      if (!ok) {
        res = -(1 + int32_t(nrow));
        run = false;
      } else {
        nrow += 1;
        pos = nx;
      }
    }
    if (run && pos >= len) {  // (the walk reports kDone at len; kept for safety)
      res = int32_t(nrow);
      run = false;
    }
  }
  return res;
}

}  // namespace spec
}  // namespace rdk
