// legacy.hip -- MsgVersion 0/1 MessageSets: the per-message CRC-32.
//
// Reference (bluelichen19/librdkafka v1.3.0):
//   writer  rd_kafka_msgset_writer_write_msg_v0_1  src/rdkafka_msgset_writer.c:583-645
//           (Offset, MessageSize, Crc = CRC-32 over MagicByte..Value, :613-641)
//   reader  rd_kafka_msgset_reader_msg_v0_1        src/rdkafka_msgset_reader.c:538-640
//           (header reads :566-587, MessageSize < hdrsize :590-597, partial :599-600,
//           check.crcs :602-628 through rd_slice_crc32, rdbuf.c:1093-1104)
//   CRC-32  rdcrc32.h:93-131 with WITH_ZLIB: zlib crc32(), reflected 0xedb88320
//
// A MessageSet is a chain: message p is [p, p + 12 + MessageSize) and the next one starts
// where it ends, so finding the messages is inherently sequential.  Walking it one message
// per LDS round trip on one wave per set runs at ~0.1 B/clk/CU (the MsgVersion 2 record
// index shows that ceiling).  Here a whole 512-thread workgroup works on one set, a 130 KiB
// LDS window at a time, and the chain is discovered SPECULATIVELY in parallel:
//
//   A. every thread owns a 260-byte segment of the window and scans it for the first
//      position that looks like a message header (MagicByte 0/1, sane Attributes, a
//      MessageSize that its Key and Value length fields fill exactly, and the message after
//      it also looking like one, with a larger Offset);
//      thread 0's segment starts at the window base, which is a true message start;
//   B. from its guess each thread walks the chain to the first position past its segment
//      (its "exit"), classifying every message exactly as the reader does;
//   C. thread l links to thread m when its exit lies in m's segment AND equals m's guess.
//      The links only go forward, so binary lifting (10 levels of pointer doubling in LDS)
//      gives every thread, in O(log) steps, whether it lies on the path from thread 0 --
//      i.e. whether its guess is a true message start.  The heuristic only decides speed,
//      never results: a wrong or missing guess ends the verified path there, and the next
//      window starts at the last verified exit (thread 0 is always exact, so every window
//      advances);
//   D. a block prefix sum over the verified threads' message counts numbers the rows; each
//      verified thread computes the CRC-32 of its own messages from LDS (slicing-by-8).
// A message larger than the window is computed by the whole workgroup from global memory
// (per-thread chunks combined with x^(8n) mod P shifts).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "common.h"

namespace rdk {
namespace {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint8_t lds_b;
typedef __attribute__((address_space(3))) uint32_t lds_w;
typedef __attribute__((address_space(3))) uint16_t lds_h;

constexpr int kLgThreads = 512;                    // threads per set
constexpr int kLgWaves = kLgThreads / 64;
// bytes scanned per thread: 65 dwords, so the 64 lanes of a wave, which scan in lockstep
// from the same offset of their segments, hit 64 different LDS banks (a 256-byte stride
// put them all in one bank)
constexpr uint32_t kLgSeg = 260;
constexpr uint32_t kLgWin = kLgThreads * kLgSeg;   // LDS window (130 KiB)
constexpr int kLgLev = 10;                         // 2^10 >= kLgThreads hops
constexpr uint32_t kNone = 0xffffffffu;

// classification of the message at p (rdkafka_msgset_reader.c:566-600)
enum : uint32_t { kOk = 0, kDone = 1, kPartial = 2, kErr = 3, kWin = 4 };

struct Win {
  const lds_b *w;  // window byte q (set offset) is w[q - base]
  uint32_t base, end, len;  // staged [base, end) of the set's [0, len)
  uint32_t q_idx0;          // LDS address of window byte base (w)
  __device__ __forceinline__ uint32_t b(uint32_t q) const { return w[q - base]; }
  // big-endian u32 at any q: two aligned LDS dwords and one v_alignbyte
  __device__ __forceinline__ uint32_t be32(uint32_t q) const {
    const uint32_t i = uint32_t(reinterpret_cast<uintptr_t>(w + (q - base)));
    const lds_w *a = reinterpret_cast<const lds_w *>(w + (q - base) - (i & 3u));
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(a[1], a[0], i & 3u));
  }
  // MessageSize at p when the message at p is whole in the window, else the class
  __device__ __forceinline__ uint32_t classify(uint32_t p, uint32_t &S) const {
    if (p == len) return kDone;
    const uint32_t R = len - p;
    if (R < 16u) return kPartial;                     // Offset, MessageSize, Crc :566-570
    if (p + 16u > end) return kWin;
    const int32_t s = int32_t(be32(p + 8u));
    if (s < 4) return kErr;                           // see DESIGN: the reference asserts
    if (uint32_t(s) - 4u > R - 16u) return kPartial;  // narrow_copy / check_len :571-573
    if (R < 18u) return kPartial;                     // MagicByte, Attributes :575-576
    if (p + 18u > end) return kWin;
    uint32_t hdr = 6u;
    if (b(p + 16u) == 1u) {                           // MsgVersion 1: Timestamp :578-580
      if (R < 26u) return kPartial;
      hdr = 14u;
    }
    if (uint32_t(s) < hdr) return kErr;               // MessageSize < hdrsize :590-597
    if (p + 12u + uint32_t(s) > end) return kWin;     // not whole in the window
    S = uint32_t(s);
    return kOk;
  }
  // first q in [s0, lim) passing plausible(), or kNone.  Sixteen candidates i..i+15 per
  // step, tested bytewise (SWAR) on a sliding run of aligned LDS dwords D[k] = bytes
  // i+4k..i+4k+3: bytes q, q+1 (Offset's top bytes: offsets < 2^48), q+8 (MessageSize's
  // top byte: < 16 MiB), q+16 (MagicByte <= 1) and q+17 (Attributes < 8).  Four new dwords
  // per step, loaded a step ahead.  Rounds: every lane first advances (no dependent
  // loads) to its next surviving candidate, then all lanes run the full test together, so
  // the wave pays one full test per round rather than one per step in which any lane has
  // a survivor.
  __device__ __forceinline__ uint32_t scan(uint32_t s0, uint32_t lim) const {
    const lds_b *w0 = w - (q_idx0 & 15u);  // 16-byte aligned window start
    const uint32_t off = (q_idx0 & 15u) - base;  // LDS index of q = q + off
    auto W32 = [&](uint32_t i) { return *reinterpret_cast<const lds_w *>(w0 + i); };
    auto zb = [](uint32_t x) { return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u; };
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
        for (int k = 0; k < 4; ++k)
          g[k] = zb(D[k]) & zb(__builtin_amdgcn_alignbyte(D[k + 1], D[k], 1u)) & zb(D[k + 2]) &
                 zb(D[k + 4] & 0xfefefefeu) &
                 zb(__builtin_amdgcn_alignbyte(D[k + 5], D[k + 4], 1u) & 0xf8f8f8f8u);
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
      if (q >= s0 && q < lim && plausible(q)) return q;
    }
    return kNone;
  }
  // heuristic message-start test (phase A): never decides a result.  Branch-free in two
  // rounds of independent LDS loads (the candidate's fields, then the ones their values
  // point at), so a test costs two LDS round trips.
  __device__ __forceinline__ bool plausible(uint32_t q) const {
    if (q + 34u > end) return false;
    // round 1: Offset, MessageSize, MagicByte/Attributes, KeyLength (v0 at +18, v1 at +26)
    const uint32_t o1h = be32(q), o1l = be32(q + 4u), S = be32(q + 8u), h = be32(q + 16u);
    const uint32_t k0 = be32(q + 18u), k1 = be32(q + 26u);
    const uint32_t m = h >> 24, a = (h >> 16) & 0xffu, hdr = m ? 14u : 6u;
    bool ok = m <= 1u && !(a & 0xf0u) && (a & 7u) <= 4u && S >= hdr + 8u &&
              S <= len - q - 12u;
    const int32_t kl = int32_t(m ? k1 : k0);
    ok = ok && kl >= -1 && (kl <= 0 || uint32_t(kl) <= S - hdr - 8u);
    const uint32_t kb = kl > 0 ? uint32_t(kl) : 0u;
    const uint32_t r = q + 12u + S;
    const bool at_end = r == len;
    ok = ok && (at_end || r + 28u <= end);  // the next header must be staged too
    // round 2: ValueLength, the next message's Offset, MessageSize, MagicByte
    const uint32_t va = ok ? q + 16u + hdr + kb : q, ra = ok && !at_end ? r : q;
    const int32_t vl = int32_t(be32(va));
    const uint32_t o2h = be32(ra), o2l = be32(ra + 4u), S2 = be32(ra + 8u), m2 = b(ra + 16u);
    // Key and Value length fields fill the message exactly (:630-637)
    ok = ok && vl >= -1 && hdr + 8u + kb + (vl > 0 ? uint32_t(vl) : 0u) == S;
    if (at_end) return ok;
    const uint64_t o1 = (uint64_t(o1h) << 32) | o1l, o2 = (uint64_t(o2h) << 32) | o2l;
    return ok && m2 <= 1u && S2 >= (m2 ? 14u : 6u) && S2 <= len - r - 12u &&
           int64_t(o2 - o1) > 0 && o2 - o1 < (uint64_t(1) << 32);  // Offsets increase
  }
};

// slicing-by-8 CRC-32 over LDS bytes [i, e) of the window (register form, no inversions):
// one dependent LDS round trip per 8 bytes
__device__ __forceinline__ uint32_t crc_lds(const lds_b *w, uint32_t i, uint32_t e, uint32_t c,
                                            const lds_w *T) {
  const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(w + i)) & 3u;
  uint32_t h = mis ? 4u - mis : 0u;
  if (h > e - i) h = e - i;
  for (uint32_t k = 0; k < h; ++k, ++i) c = T[(c ^ w[i]) & 0xffu] ^ (c >> 8);
  for (; i + 8u <= e; i += 8u) {
    const uint32_t lo = c ^ *reinterpret_cast<const lds_w *>(w + i);
    const uint32_t hi = *reinterpret_cast<const lds_w *>(w + i + 4u);
    c = T[1792 + (lo & 0xffu)] ^ T[1536 + ((lo >> 8) & 0xffu)] ^ T[1280 + ((lo >> 16) & 0xffu)] ^
        T[1024 + (lo >> 24)] ^ T[768 + (hi & 0xffu)] ^ T[512 + ((hi >> 8) & 0xffu)] ^
        T[256 + ((hi >> 16) & 0xffu)] ^ T[hi >> 24];
  }
  if (i + 4u <= e) {
    c ^= *reinterpret_cast<const lds_w *>(w + i);
    c = T[768 + (c & 0xffu)] ^ T[512 + ((c >> 8) & 0xffu)] ^ T[256 + ((c >> 16) & 0xffu)] ^
        T[c >> 24];
    i += 4u;
  }
  for (; i < e; ++i) c = T[(c ^ w[i]) & 0xffu] ^ (c >> 8);
  return c;
}

// same over global bytes [p, e) (the big-message path)
__device__ __forceinline__ uint32_t crc_gbl(const uint8_t *p, const uint8_t *e, uint32_t c,
                                            const lds_w *T) {
  while (p < e && (reinterpret_cast<uintptr_t>(p) & 3u)) c = T[(c ^ *p++) & 0xffu] ^ (c >> 8);
  for (; p + 4 <= e; p += 4) {
    c ^= *reinterpret_cast<const uint32_t *>(p);
    c = T[768 + (c & 0xffu)] ^ T[512 + ((c >> 8) & 0xffu)] ^ T[256 + ((c >> 16) & 0xffu)] ^
        T[c >> 24];
  }
  while (p < e) c = T[(c ^ *p++) & 0xffu] ^ (c >> 8);
  return c;
}

__device__ __forceinline__ uint32_t mulp(uint32_t a, uint32_t b) {  // GF(2)[x]/P, reflected
  uint32_t m = 1u << 31, p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ 0xedb88320u : b >> 1;
  }
  return p;
}

__device__ __forceinline__ uint32_t xpow8(uint64_t nbytes, const uint32_t *x2n) {
  uint32_t p = 1u << 31;
  int k = 3;
  for (uint64_t n = nbytes; n; n >>= 1, ++k)
    if (n & 1u) p = mulp(x2n[k], p);
  return p;
}

__device__ __forceinline__ void put_be32(uint8_t *p, uint32_t v) {
  p[0] = uint8_t(v >> 24);
  p[1] = uint8_t(v >> 16);
  p[2] = uint8_t(v >> 8);
  p[3] = uint8_t(v);
}

#ifdef RDK_LG_PROF  // phase timing (A/B builds only): s_memtime cycles summed over blocks
__device__ unsigned long long g_lg_prof[8];
#define LG_T(i)                                                          \
  do {                                                                   \
    __syncthreads();                                                     \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();          \
    if (t == 0) atomicAdd(&g_lg_prof[i], _n - prof_t);                   \
    prof_t = _n;                                                         \
  } while (0)
#else
#define LG_T(i) do { } while (0)
#endif

template <int MODE>
__global__ __launch_bounds__(kLgThreads, 1) void v01_crc_kernel(
    uint8_t *__restrict__ sbase, const uint64_t *__restrict__ set_offs,
    const uint32_t *__restrict__ set_lens, const uint64_t *__restrict__ row_offs,
    const uint32_t *__restrict__ row_caps, uint32_t *__restrict__ msg_pos,
    uint32_t *__restrict__ msg_out, int32_t *__restrict__ count,
    const uint32_t *__restrict__ gtab, const uint32_t *__restrict__ x2n) {
  __shared__ __attribute__((aligned(16))) uint8_t win_s[kLgWin + 64];
  __shared__ uint16_t J_s[kLgLev][kLgThreads];
  __shared__ uint32_t T_s[2048];
  __shared__ uint32_t cand_s[kLgThreads];
  __shared__ uint32_t wsum_s[kLgWaves];
  __shared__ uint32_t term_s[2];  // exit and class of the path's last thread
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  for (uint32_t i = t; i < 2048u; i += kLgThreads) T_s[i] = gtab[i];  // slicing tables 0..7
  const lds_w *T = (const lds_w *)T_s;
  const uint32_t si = blockIdx.x;
  uint8_t *set = sbase + set_offs[si];
  const uint32_t len = set_lens[si];
  const uint64_t row0 = row_offs[si];
  const uint32_t cap = row_caps[si];
  uint32_t pos = 0, nrow = 0;
  int32_t res = 0;
  bool run = true;
  constexpr int kV = int((kLgWin + kLgThreads * 16 - 1) / (kLgThreads * 16));
  u32x4 pv[kV];
  bool pref = false;
  auto issue = [&](uint32_t b0) {  // the window at b0 into pv (bytes past the set read 0)
    const uintptr_t ga = reinterpret_cast<uintptr_t>(set + b0);
    const uintptr_t al = ga & ~uintptr_t(15);
    const uint32_t sh0 = uint32_t(ga - al), av = len - b0;
    const uint32_t wl0 = av < kLgWin - sh0 ? av : kLgWin - sh0;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(al), 0,
                                                        int((sh0 + wl0 + 3u) & ~3u), 0x00020000);
#pragma unroll
    for (int it = 0; it < kV; ++it)
      pv[it] = __builtin_amdgcn_raw_buffer_load_b128(rs, (t + kLgThreads * it) * 16u, 0, 0);
  };
#ifdef RDK_LG_PROF
  unsigned long long prof_t = __builtin_amdgcn_s_memtime();
#endif
  while (run) {
    // ---- stage [base, end): 16-byte buffer loads from the aligned address below base
    // (issued during the previous window's CRC phase when that window could tell where
    // this one starts), stored once the previous window's readers are done
    const uint32_t base = pos;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(set + base)) & 15u;
    const uint32_t avail = len - base;
    const uint32_t wl = avail < kLgWin - sh ? avail : kLgWin - sh;
    if (!pref) issue(base);
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kV; ++it)
      if ((t + kLgThreads * it) * 16u < kLgWin)
        *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(
            (lds_b *)win_s + (t + kLgThreads * it) * 16u) = pv[it];
    Win W;
    W.w = (const lds_b *)win_s + sh;
    W.base = base;
    W.end = base + wl;
    W.len = len;
    W.q_idx0 = uint32_t(reinterpret_cast<uintptr_t>(W.w));
    __syncthreads();
    LG_T(0);
    // ---- A: guess the first message start in this thread's segment
    const uint32_t s0 = base + t * kLgSeg, s1 = s0 + kLgSeg;
    uint32_t c = kNone;
    if (t == 0) {
      c = base;
    } else if (s0 < W.end) {
      c = W.scan(s0, s1 < W.end ? s1 : W.end);
    }
    cand_s[t] = c;
    LG_T(1);
    // ---- B: walk from the guess to the first position past the segment
    uint32_t x = c, k = 0, cls = kOk;
    if (c != kNone) {
      while (x < s1) {
        uint32_t S = 0;
        cls = W.classify(x, S);
        if (cls != kOk) break;
        x += 12u + S;
        ++k;
      }
    }
    __syncthreads();
    LG_T(2);
    // ---- C: link to the thread whose guess is our exit; binary lifting from thread 0
    uint32_t nxt = t;
    if (c != kNone && cls == kOk && x < W.end) {
      const uint32_t m = (x - base) / kLgSeg;
      if (m < uint32_t(kLgThreads) && cand_s[m] == x) nxt = m;
    }
    J_s[0][t] = uint16_t(nxt);
    for (int lv = 1; lv < kLgLev; ++lv) {
      __syncthreads();
      J_s[lv][t] = J_s[lv - 1][J_s[lv - 1][t]];
    }
    __syncthreads();
    uint32_t cur = 0;
    for (int lv = kLgLev - 1; lv >= 0; --lv) {
      const uint32_t y = J_s[lv][cur];
      if (y <= t) cur = y;
    }
    const bool on = c != kNone && cur == t;
    const bool last = on && J_s[kLgLev - 1][0] == t;
    if (last) {
      term_s[0] = x;
      term_s[1] = cls;
    }
    LG_T(3);
    // ---- D: number the rows (block exclusive scan of the verified counts)
    const uint32_t mine = on ? k : 0u;
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d);
      if (lane >= uint32_t(d)) inc += y;
    }
    if (lane == 63u) wsum_s[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < uint32_t(kLgWaves); ++w) {
      const uint32_t y = wsum_s[w];
      before += w < wv ? y : 0u;
      total += y;
    }
    const uint32_t rb = nrow + before + inc - mine;
    const uint32_t tx = term_s[0], tc = term_s[1];
    // the next window's start is known now: overlap its loads with the CRC phase
    pref = nrow + total <= cap && tc != kDone && tc != kPartial && tc != kErr && tx != base &&
           tx < len;
    if (pref) issue(tx);
    if (on) {
      uint32_t p = c;
      for (uint32_t i = 0; i < k; ++i) {
        const uint32_t S = W.be32(p + 8u);
        const uint32_t r = rb + i;
        if (r < cap) {
          const uint32_t crc =
              ~crc_lds(W.w - base, p + 16u, p + 12u + S, 0xffffffffu, T);  // :613-641
          msg_pos[row0 + r] = p;
          if (MODE == RDK_HIP_V2_CRC_VERIFY) {
            msg_out[row0 + r] = W.be32(p + 12u) == crc ? 0u : 1u;  // :602-628
          } else {
            msg_out[row0 + r] = crc;
            if (MODE == RDK_HIP_V2_CRC_FINALIZE) put_be32(set + p + 12u, crc);  // :640-641
          }
        }
        p += 12u + S;
      }
    }
    LG_T(4);
#ifdef RDK_LG_PROF
    if (t == 0) atomicAdd(&g_lg_prof[6], 1ull);
    if (t == 0) atomicAdd(&g_lg_prof[7], (unsigned long long)(term_s[0] - base));
#endif
    nrow += total;
    if (nrow > cap) {
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
      // ---- a message larger than the window, at base (header staged: tc == kWin)
      const uint32_t S = W.be32(base + 8u);
      const uint8_t *p0 = set + base + 16u;
      const uint64_t L = uint64_t(S) - 4u;
      const uint64_t C = ((L + kLgThreads - 1) / kLgThreads + 3u) & ~uint64_t(3);
      const uint64_t pad = C * kLgThreads - L;  // virtual zero bytes in front
      const uint64_t vs = uint64_t(t) * C, ve = vs + C;
      uint32_t term = 0;
      if (ve > pad) {
        const uint64_t rs0 = vs > pad ? vs - pad : 0, re0 = ve - pad;
        const uint32_t r = crc_gbl(p0 + rs0, p0 + re0, rs0 == 0 ? 0xffffffffu : 0u, T);
        term = mulp(xpow8(uint64_t(kLgThreads - 1u - t) * C, x2n), r);
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) term ^= __shfl_xor(term, d);
      __syncthreads();
      if (lane == 0) wsum_s[wv] = term;
      __syncthreads();
      uint32_t acc = 0;
      for (uint32_t w = 0; w < uint32_t(kLgWaves); ++w) acc ^= wsum_s[w];
      const uint32_t crc = ~acc;
      if (nrow >= cap) {
        res = -(1 + int32_t(nrow));
        run = false;
      } else {
        if (t == 0) {
          msg_pos[row0 + nrow] = base;
          if (MODE == RDK_HIP_V2_CRC_VERIFY) {
            msg_out[row0 + nrow] = W.be32(base + 12u) == crc ? 0u : 1u;
          } else {
            msg_out[row0 + nrow] = crc;
            if (MODE == RDK_HIP_V2_CRC_FINALIZE) put_be32(set + base + 12u, crc);
          }
        }
        nrow += 1;
        pos = base + 12u + S;
      }
    }
    if (run && pos >= len) {  // (the walk reports kDone at len; kept for safety)
      res = int32_t(nrow);
      run = false;
    }
  }
  if (t == 0) count[si] = res;
#ifdef RDK_LG_PROF
  if (t == 0) atomicAdd(&g_lg_prof[5], 1ull);
#endif
}

}  // namespace
}  // namespace rdk

using namespace rdk;

RDK_API int rdk_hip_msgset_v01_crc(void *d_base, const uint64_t *d_set_offs,
                                   const uint32_t *d_set_lens, const uint64_t *d_row_offs,
                                   const uint32_t *d_row_caps, uint32_t *d_msg_pos,
                                   uint32_t *d_msg_out, int32_t *d_count, uint32_t n, int mode,
                                   void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_base || !d_set_offs || !d_set_lens || !d_row_offs || !d_row_caps || !d_msg_pos ||
      !d_msg_out || !d_count)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t *b = static_cast<uint8_t *>(d_base);
  const uint32_t *tab = crc_tables_dev(c->device, kCrcKind32);
  const uint32_t *x2n = crc_x2n_dev(c->device, kCrcKind32);
#define RDK_V01(M)                                                                        \
  hipLaunchKernelGGL(v01_crc_kernel<M>, dim3(n), dim3(kLgThreads), 0, s, b, d_set_offs,   \
                     d_set_lens, d_row_offs, d_row_caps, d_msg_pos, d_msg_out, d_count, tab, \
                     x2n)
  switch (mode) {
    case RDK_HIP_V2_CRC_COMPUTE: RDK_V01(RDK_HIP_V2_CRC_COMPUTE); break;
    case RDK_HIP_V2_CRC_FINALIZE: RDK_V01(RDK_HIP_V2_CRC_FINALIZE); break;
    case RDK_HIP_V2_CRC_VERIFY: RDK_V01(RDK_HIP_V2_CRC_VERIFY); break;
    default: return set_error(RDK_HIP_E_INVAL, "mode %d", mode);
  }
#undef RDK_V01
  RDK_HIP_CHECK(hipGetLastError());
#ifdef RDK_LG_PROF
  unsigned long long h[8];
  RDK_HIP_CHECK(hipStreamSynchronize(s));
  RDK_HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_lg_prof), sizeof h));
  fprintf(stderr, "lg_prof stage %llu A %llu B %llu C %llu D %llu blocks %llu windows %llu "
          "advance %llu\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
#endif
  return RDK_HIP_OK;
}
