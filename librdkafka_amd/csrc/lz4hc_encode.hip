// lz4hc_encode.hip -- LZ4F frame compression at compression.level 3..12 (LZ4HC:
// the hash-chain parser of levels 3..9 and the optimal parser of 10..12) on gfx950.
//
// Replaces rd_kafka_lz4_compress (rdkafka_lz4.c:329) -> LZ4F_makeBlock
// (lz4frame.c:739, dstCapacity = srcSize-1) -> LZ4F_compressBlockHC
// (lz4frame.c:782) -> LZ4_compress_HC_extStateHC_fastReset (lz4hc.c:896) ->
// LZ4HC_compress_hashChain (lz4hc.c:532-746), nbSearches = clTable
// (lz4hc.c:775-789).  Frames are byte-identical to the reference's (the CPU
// restatement in oracle/lz4hc_oracle.c documents why every LZ4F block is a
// fresh, prefix-only window).
//
// One wavefront per 64 KiB block, scratch in HBM (no LDS, so many blocks per
// CU hide the latency of the parse's dependent loads):
//   1. build: the hash chain for every position up to mflimit, 64 positions
//      per step (same-hash lanes found with 15 ballots), PLUS each position's
//      rank inside its hash bucket; a scan over the 32768 bucket sizes and a
//      scatter give `sorted`, the block's positions ordered by (hash, pos).
//      The chain of position p (LZ4HC_Insert + DELTANEXTU16 walk) is then the
//      contiguous run of `sorted` in front of p: one coalesced load fetches
//      64 candidates.
//   2. parse: the hash-chain state machine runs wave-uniform.  A search
//      (LZ4HC_InsertAndGetWiderMatch, lz4hc.c:234-442) evaluates 64
//      candidates at once (MINMATCH check, countBack, LZ4_count, one lane
//      each), then replays the reference's order: the first candidate (in
//      chain order) that passes the read16 prefilter at the current `longest`
//      and beats it wins, and the scan resumes after it with the new longest.
//      Level 9's pattern analysis (lz4hc.c:336-405) can only redirect the
//      walk for a repetitive 4-byte pattern (period 1 or 2); such searches
//      walk the chain one candidate at a time exactly as the reference does.
//   3. sequences are emitted by LZ4HC_encodeSequence's rules (limitedOutput);
//      a block that does not fit in srcSize-1 bytes is stored raw (bit 31).
// Block k of frame f goes to the same worst-case slot as the level-0 engine;
// lz4f_assemble_kernel (lz4_encode.hip) then builds the frame.
//
// Levels 10..12 (LZ4HC_compress_optimal, lz4hc.c:1278-1538; clTable rows
// lz4hc.c:786-788) share the build and the encoder.  Their search
// (LZ4HC_FindLongerMatch, lz4hc.c:1255) looks forward only, with pattern analysis
// and the chain swap (lz4hc.c:312-334): after a candidate that ties or beats the
// longest match, the walk moves to the chain of the position inside that match
// whose previous occurrence lies furthest back.  hc_search_swap() evaluates 64
// candidates of the current chain at once and replays them in order; a swap
// restarts it on the new chain (the sorted position list serves any position's
// chain, not only ip's).  The price table of the dynamic program lives in the
// wave's HBM scratch; its per-length loops run one length per lane.
#include <hip/hip_runtime.h>

#include <mutex>

#include "common.h"
#include "lz4_device.h"
#include "lz4_wave.h"

namespace rdk {

constexpr int kHcItems = 64;                 // block slots per frame per pass
constexpr uint32_t kHcSlot = kLz4Block + 4;  // worst-case bytes per block in a frame
constexpr int kHcHashLog = 15;               // lz4hc.h:196
constexpr uint32_t kHcNone = 0xFFFFFFFFu;
constexpr int kHcOptimalML = 18;             // lz4hc.c:74
constexpr size_t kHcTab = size_t(4) << kHcHashLog;  // head / bucket start, u32
constexpr int kHcOptNum = 1 << 12;           // LZ4_OPT_NUM, lz4hc.c:75
constexpr int kHcTrailing = 3;               // TRAILING_LITERALS, lz4hc.c:1290
constexpr size_t kHcOptBytes = size_t(kHcOptNum + 64) * 16;  // price table of the optimal parser
// + chain (u16), sorted (u32), tr (u32), opt (16 B entries)
constexpr size_t kHcScratch = kHcTab + 3 * 65536 * 2 + 65536 * 4 + kHcOptBytes;
constexpr unsigned kHcGrid = 4096;  // 16 waves per CU (the kernel fits 20)

struct HcBlock {
  uintptr_t s;       // block bytes (global)
  uint32_t *head;    // build: pos | rank << 16 per hash; then bucket start
  uint16_t *chain;   // DELTANEXTU16 per position
  // positions ordered by (hash, position), each with a fingerprint of its 4 bytes: position |
  // (their low 16 bits) << 16.  The candidates of one bucket lie side by side, so ruling
  // them out by fingerprint reads one line where their source bytes are one line each.
  uint32_t *sorted;
  uint32_t *tr;      // per position: its index in sorted | its rank << 16
  int4 *opt;         // LZ4HC_optimal_t[]: x price, y off, z mlen, w litlen (levels 10..12)
  int attempts;      // nbSearches
  int pa;            // patternAnalysis (levels 9+)
  int lane;
#ifdef RDK_HC_PROF
  mutable uint64_t pc[10];
#endif
};

#ifdef RDK_HC_PROF
#define HC_T0() const uint64_t hct0_ = __builtin_amdgcn_s_memtime()
#define HC_ADD(k) b.pc[k] += __builtin_amdgcn_s_memtime() - hct0_
#define HC_CNT(k, v) b.pc[k] += (v)
#else
#define HC_T0() do { } while (0)
#define HC_ADD(k) do { } while (0)
#define HC_CNT(k, v) do { } while (0)
#endif

__device__ __forceinline__ uint32_t hc_hash(uint32_t v) {  // HASH_FUNCTION, lz4hc.c:81
  return (v * 2654435761u) >> (32 - kHcHashLog);
}

// 16 bytes at any byte address through five aligned dword loads issued
// together; touches at most the dword holding byte a+16 (callers keep a+32 <=
// matchlimit = iend - LASTLITERALS, so nothing past the input is read)
__device__ __forceinline__ void hc_ld16(uintptr_t a, uint32_t w[4]) {
  const uintptr_t b = a & ~uintptr_t(3);
  const uint32_t sh = uint32_t(a & 3u);
  uint32_t d[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) d[j] = *(g_cu32 *)(b + 4 * j);
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
}

// LZ4_count by one lane: equal bytes from a / b, a never reaching lim.
// 32 bytes per dependent round trip while they fit, then dwords, then bytes.
__device__ __forceinline__ int hc_count(uintptr_t s, int a, int b, int lim) {
  const int a0 = a;
  while (a + 32 <= lim) {
    uint32_t x[8], y[8];
    hc_ld16(s + a, x);
    hc_ld16(s + a + 16, x + 4);
    hc_ld16(s + b, y);
    hc_ld16(s + b + 16, y + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t d = x[j] ^ y[j];
      if (d) return a + 4 * j + (__builtin_ctz(d) >> 3) - a0;
    }
    a += 32;
    b += 32;
  }
  while (a + 4 <= lim) {
    const uint32_t x = ld32u(s + a) ^ ld32u(s + b);
    if (x) return a + (__builtin_ctz(x) >> 3) - a0;
    a += 4;
    b += 4;
  }
  while (a < lim && ldb(s + a) == ldb(s + b)) { a++; b++; }
  return a - a0;
}

__device__ __forceinline__ uint32_t pat_byte(uint32_t pat, int k) { return (pat >> (8 * (k & 3))) & 0xFFu; }

// LZ4HC_countPattern (lz4hc.c:171-199): s[p+k] == byte k%4 of the pattern
__device__ int hc_count_pattern(uintptr_t s, int p, int end, uint32_t pat) {
  int k = 0;
  while (p + k < end && ldb(s + p + k) == pat_byte(pat, k)) k++;
  return k;
}

// LZ4HC_reverseCountPattern (lz4hc.c:204-219)
__device__ int hc_rcount_pattern(uintptr_t s, int p, int low, uint32_t pat) {
  const int p0 = p;
  while (p >= low + 4 && ld32u(s + p - 4) == pat) p -= 4;
  int k = 3;
  while (k >= 0 && p > low && ldb(s + p - 1) == pat_byte(pat, k)) { p--; k--; }
  return p0 - p;
}

__device__ __forceinline__ void hc_copy(uintptr_t d, uintptr_t s, int len, int lane) {
  for (int base = 0; base < len; base += 256) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + lane + 64 * j;  // (clamped, not predicated: see wave_copy_bytes)
      v[j] = ldb(s + (i < len ? i : len - 1));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + lane + 64 * j;
      if (i < len) stb(d + i, v[j]);
    }
  }
}

// n255 bytes of 255 then one `rest` byte
__device__ __forceinline__ void hc_run(uintptr_t d, int n255, int rest, int lane) {
  for (int i = lane; i < n255; i += 64) stb(d + i, 255u);
  if (lane == 0) stb(d + n255, uint32_t(rest));
}

// 1. hash chains, bucket ranks, bucket starts and the sorted position list
__device__ void hc_build(const HcBlock &b, int npos) {
  const int lane = b.lane;
  for (int i = lane; i < (1 << kHcHashLog); i += 64) b.head[i] = kHcNone;
  __threadfence_block();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  // the next step's source word is loaded during this step (it does not
  // depend on the head[] updates), leaving one dependent round trip per step
  uint32_t w_next = lane < npos ? ld32u(b.s + lane) : 0u;
  for (int base = 0; base < npos; base += 64) {
    const int p = base + lane;
    const bool valid = p < npos;
    const uint32_t h = valid ? hc_hash(w_next) : 0u;
    w_next = p + 64 < npos ? ld32u(b.s + p + 64) : 0u;
    const uint64_t eq = same_value_lanes<kHcHashLog>(h, ballot(valid));
    const uint32_t hv = valid ? b.head[h] : kHcNone;
    const uint64_t eb = eq & below;
    const uint32_t rk = (hv == kHcNone ? 0u : (hv >> 16) + 1u) + uint32_t(__popcll(eb));
    int prev;
    if (eb) prev = base + (63 - __clzll(eb));
    else prev = hv == kHcNone ? -65536 : int(hv & 0xFFFFu);
    if (valid) {
      const int d = p - prev;  // LZ4HC_Insert (lz4hc.c:125-132)
      b.chain[p] = uint16_t(d > 65535 ? 65535 : d);
      b.tr[p] = h | (rk << 16);  // the scatter below takes hash and rank from here
      if (!(eq & above)) b.head[h] = uint32_t(p) | (rk << 16);
    }
    __threadfence_block();
  }
  // bucket sizes -> exclusive prefix (in place: head[] becomes bucket start)
  constexpr int kPer = (1 << kHcHashLog) / 64;
  uint32_t *mine = b.head + lane * kPer;
  uint32_t sum = 0;
  for (int i = 0; i < kPer; ++i) {
    const uint32_t v = mine[i];
    sum += v == kHcNone ? 0u : (v >> 16) + 1u;
  }
  uint32_t incl = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  uint32_t run = incl - sum;
  for (int i = 0; i < kPer; i += 16) {
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = mine[i + j];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      mine[i + j] = run;
      run += v[j] == kHcNone ? 0u : (v[j] >> 16) + 1u;
    }
  }
  __threadfence_block();
  // scatter, four steps' loads issued before their stores
  for (int p0 = lane; p0 < npos; p0 += 256) {
    uint32_t t[4], v[4], st[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 + 64 * j;
      t[j] = p < npos ? b.tr[p] : 0u;
      v[j] = ld32u_nb(b.s + min(p, npos - 1));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = b.head[t[j] & 0x7FFFu];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 + 64 * j;
      if (p < npos) {
        const uint32_t r = t[j] >> 16;
        const uint32_t idx = st[j] + r;
        b.sorted[idx] = uint32_t(p) | (v[j] << 16);
        b.tr[p] = idx | (r << 16);
      }
    }
  }
  __threadfence_block();
}

// The chain swap's scan (lz4hc.c:315-329) over the chain deltas of the match at m:
// `dist` = the largest delta met on the accelerating schedule, `cp` = its position
// (left alone when no delta beats 1).  64 deltas per load, the schedule replayed
// on them with v_readlane.
__device__ void hc_swap_scan(const HcBlock &b, int m, int longest, int &dist, int &cp) {
  const int end = longest - kLz4MinMatch + 1;
  int step = 1, accel = 1 << 4, pos = 0;
  dist = 1;
  for (int base = 0; base < end; base += 64) {
    const uint32_t cd = base + b.lane < end ? uint32_t(b.chain[m + base + b.lane]) : 0u;
    const int lim = end < base + 64 ? end : base + 64;
    while (pos < lim) {
      const int c = int(__builtin_amdgcn_readlane(cd, pos - base));
      step = accel++ >> 4;
      if (c > dist) { dist = c; cp = pos; accel = 1 << 4; }
      pos += step;
    }
  }
}

// LZ4HC_InsertAndGetWiderMatch one candidate at a time (repetitive patterns
// where pattern analysis may redirect the walk: level 9 and the optimal parser).
__device__ int hc_search_serial(const HcBlock &b, int ip, int ilow, int ihigh, int longest,
                                int &mpos, int &spos, uint32_t pat, bool swap) {
  const uintptr_t s = b.s;
  const int br = ip - ilow;
  int attempts = b.attempts;
  int repeat = 0, src_pat_len = 0;  // 0 untested, 1 not, 2 confirmed
  int cp = 0;                       // matchChainPos
  int m = ip - int(b.chain[ip]);
  while (m >= 0 && attempts) {
    attempts--;
    int len = 0;
    {
      const int a = ilow + longest - 1, c = m - br + longest - 1;
      if (ldb(s + a) == ldb(s + c) && ldb(s + a + 1) == ldb(s + c + 1) && ld32u(s + m) == pat) {
        int back = 0;
        if (br) {
          const int lim = (ilow - ip) > -m ? (ilow - ip) : -m;
          while (back > lim && ldb(s + ip + back - 1) == ldb(s + m + back - 1)) back--;
        }
        len = 4 + hc_count(s, ip + 4, m + 4, ihigh) - back;
        if (len > longest) { longest = len; mpos = m + back; spos = ip + back; }
      }
    }
    if (swap && len == longest && m + longest <= ip) {  // lz4hc.c:312-334
      int dist;
      hc_swap_scan(b, m, longest, dist, cp);
      if (dist > 1) {
        m -= dist;
        continue;
      }
    }
    const int dnext = b.chain[m];
    if (b.pa && dnext == 1 && cp == 0) {
      const int cand = m - 1;
      if (repeat == 0) {
        if (((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24))) {
          repeat = 2;
          src_pat_len = hc_count_pattern(s, ip + 4, ihigh, pat) + 4;
        } else {
          repeat = 1;
        }
      }
      if (repeat == 2 && cand >= 0 && ld32u(s + cand) == pat) {
        const int fwd = hc_count_pattern(s, cand + 4, ihigh, pat) + 4;
        int bwd = hc_rcount_pattern(s, cand, 0, pat);
        if (bwd > cand) bwd = cand;
        const int seg = bwd + fwd;
        if (seg >= src_pat_len && fwd <= src_pat_len) {
          m = cand + fwd - src_pat_len;
        } else {
          m = cand - bwd;
          if (br == 0) {
            const int maxml = seg < src_pat_len ? seg : src_pat_len;
            if (longest < maxml) {
              if (ip - m > 65535) break;
              longest = maxml; mpos = m; spos = ip;
            }
            m -= int(b.chain[m]);
          }
        }
        continue;
      }
    }
    m -= int(b.chain[m + cp]);
  }
  return longest;
}

// LZ4HC_countBack (lz4hc.c:140-152) by one lane: equal bytes walking back from ip-1 / c-1,
// at most -lim of them (lim <= 0), four per dependent round trip.  Returns -count.
__device__ __forceinline__ int hc_count_back(uintptr_t s, int ip, int c, int lim) {
  int back = 0;
  while (back - 4 >= lim) {
    const uint32_t x = ld32u_nb(s + ip + back - 4) ^ ld32u_nb(s + c + back - 4);
    if (x) return back - (__builtin_clz(x) >> 3);
    back -= 4;
  }
  while (back > lim && ldb(s + ip + back - 1) == ldb(s + c + back - 1)) back--;
  return back;
}

// LZ4HC_InsertAndGetWiderMatch, 64 chain candidates per step; reads no further than the
// reference does (the last positions of a block, where hc_search()'s windows would run over)
__device__ int hc_search_edge(const HcBlock &b, int ip, int ilow, int ihigh, int longest, int &mpos,
                         int &spos) {
  const uintptr_t s = b.s;
  const int lane = b.lane;
  // (ip <= mflimit: the branch-free 8-byte read stays inside the block, and the table entry
  // is in flight together with the pattern)
  const uint32_t pat = ld32u_nb(s + ip);
  const uint32_t t = b.tr[ip];  // one load instead of rank -> hash -> bucket start
  if (b.pa && ((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24)))
    return hc_search_serial(b, ip, ilow, ihigh, longest, mpos, spos, pat, false);
  const int br = ip - ilow;
  const int r = int(t >> 16);
  const int top = int(t & 0xFFFFu) - 1;  // sorted[top] = latest earlier same-hash
  const int total = r < b.attempts ? r : b.attempts;
  for (int c0 = 0; c0 < total; c0 += 64) {
    const int j = c0 + lane;
    const bool valid = j < total;
    const int c = int(b.sorted[valid ? top - j : top] & 0xFFFFu);
    const bool ok32 = (ld32u_nb(s + c) == pat) & valid;  // (c < ip: inside the block as well)
    int back = 0, len = 0;
    if (ok32) {
      if (br) {
        const int lim = (ilow - ip) > -c ? (ilow - ip) : -c;
        back = hc_count_back(s, ip, c, lim);
      }
      len = 4 + hc_count(s, ip + 4, c + 4, ihigh) - back;
    }
    int k0 = 0;
    for (;;) {  // the reference's order: first improving candidate at the current longest
      // the read16 prefilter at longest-1 from the low limit (lz4hc.c:264): both of its bytes
      // lie inside the measured match when that reaches back to the low limit (always, for
      // a search without look-back), so only the other candidates have to read them
      const bool cand = ok32 && lane >= k0 && len > longest;
      const bool sure = back == -br;
      bool pass = cand && sure;
      if (ballot(cand && !sure)) {
        const bool rd = cand && !sure;
        const int a = ilow + longest - 1, q = c - br + longest - 1;
        // (a candidate that is read has q >= 0: its low limit lies inside the block)
        const uint32_t x0 = ldb(s + (rd ? a : ip)), y0 = ldb(s + (rd ? q : ip));
        const uint32_t x1 = ldb(s + (rd ? a + 1 : ip)), y1 = ldb(s + (rd ? q + 1 : ip));
        pass = pass || (rd && x0 == y0 && x1 == y1);
      }
      const uint64_t m = ballot(pass);
      if (!m) break;
      const int k = __builtin_ctzll(m);
      longest = __shfl(len, k);
      mpos = __shfl(c + back, k);
      spos = ip + __shfl(back, k);
      k0 = k + 1;
    }
  }
  return longest;
}

// 4-aligned dwords d[0..N) hold bytes from address (a & ~3): word k of the byte stream at a
template <int N>
__device__ __forceinline__ void hc_load_words(uintptr_t a, uint32_t w[N]) {
  const uintptr_t base = a & ~uintptr_t(3);
  const uint32_t sh = uint32_t(a & 3u);
  uint32_t d[N + 1];
#pragma unroll
  for (int k = 0; k <= N; ++k) d[k] = *(g_cu32 *)(base + 4 * k);
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// LZ4HC_InsertAndGetWiderMatch, 64 chain candidates per step.  One round trip fetches a
// candidate's 36 bytes (the MINMATCH test and the first 32 bytes of LZ4_count) and the 8
// bytes in front of it (countBack), on clamped addresses; the source's windows are loaded
// once, with the pattern and the table entry.  Longer matches continue from memory.
__device__ int hc_search_w(const HcBlock &b, int ip, int ilow, int ihigh, int longest, int &mpos,
                           int &spos);
__device__ int hc_search(const HcBlock &b, int ip, int ilow, int ihigh, int longest, int &mpos,
                         int &spos) {
  HC_T0();
  const int r_ = hc_search_w(b, ip, ilow, ihigh, longest, mpos, spos);
  HC_ADD(ip == ilow ? 0 : 1);
  HC_CNT(ip == ilow ? 2 : 3, 1);
  return r_;
}
__device__ int hc_search_w(const HcBlock &b, int ip, int ilow, int ihigh, int longest, int &mpos,
                           int &spos) {
  if (ip + 48 > ihigh) return hc_search_edge(b, ip, ilow, ihigh, longest, mpos, spos);
  const uintptr_t s = b.s;
  const int lane = b.lane;
  uint32_t sw[9], sb[2];
  hc_load_words<9>(s + ip, sw);  // bytes ip .. ip+36 (ip + 40 < block end)
  const uint32_t t = b.tr[ip];   // one load instead of rank -> hash -> bucket start
  const int br = ip - ilow;
  const bool wideback = br != 0 && ip >= 8;
  hc_load_words<2>(s + (wideback ? ip - 8 : ip), sb);  // bytes ip-8 .. ip
  const uint32_t pat = sw[0];
  if (b.pa && ((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24)))
  {
    HC_CNT(5, 1);
    return hc_search_serial(b, ip, ilow, ihigh, longest, mpos, spos, pat, false);
  }
  const int r = int(t >> 16);
  const int top = int(t & 0xFFFFu) - 1;  // sorted[top] = latest earlier same-hash
  const int total = r < b.attempts ? r : b.attempts;
  for (int c0 = 0; c0 < total; c0 += 64) {
    HC_CNT(4, 1);
    const int j = c0 + lane;
    const bool valid = j < total;
    const uint32_t se = b.sorted[valid ? top - j : top];
    // a candidate whose fingerprint differs cannot pass the MINMATCH test (lz4hc.c:266): its
    // loads go to the position itself, lines the wave holds already
    const bool fpok = valid & ((se >> 16) == (pat & 0xFFFFu));
    const int c = fpok ? int(se & 0xFFFFu) : ip;
    uint32_t cw[9], cb[2];
    hc_load_words<9>(s + c, cw);  // (c <= ip)
    const bool cback = wideback && c >= 8;
    hc_load_words<2>(s + (cback ? c - 8 : c), cb);
    const bool ok32 = (cw[0] == pat) & fpok;
    int fwd = 32;
#pragma unroll
    for (int k = 8; k >= 1; --k) {
      const uint32_t z = sw[k] ^ cw[k];
      if (z) fwd = 4 * (k - 1) + (__builtin_ctz(z) >> 3);
    }
    if (ballot(ok32 && fwd == 32)) {  // (ip + 36 < ihigh, so the 32 bytes were all countable)
      if (ok32 && fwd == 32) fwd += hc_count(s, ip + 36, c + 36, ihigh);
    }
    int back = 0;
    if (br) {
      const int lim = (ilow - ip) > -c ? (ilow - ip) : -c;  // LZ4HC_countBack (lz4hc.c:140-152)
      const uint32_t x1 = sb[1] ^ cb[1], x0 = sb[0] ^ cb[0];
      const int eqb = x1 ? int(__builtin_clz(x1) >> 3) : 4 + (x0 ? int(__builtin_clz(x0) >> 3) : 4);
      back = -(eqb < -lim ? eqb : -lim);
      const bool slow = ok32 && (cback ? (eqb == 8 && lim < -8) : true);
      if (ballot(slow)) {
        if (slow) back = cback ? hc_count_back(s, ip - 8, c - 8, lim + 8) - 8 : hc_count_back(s, ip, c, lim);
      }
    }
    const int len = ok32 ? 4 + fwd - back : 0;
    int k0 = 0;
    for (;;) {  // the reference's order: first improving candidate at the current longest
      // the read16 prefilter (lz4hc.c:264) compares the bytes at offsets o and o+1 from ip,
      // o = longest-1 - look-back.  The measured match covers offsets [back, back+len): o+1
      // lies below its end for a candidate that beats `longest` (len > longest, back >= -br),
      // and o lies in it unless the backward count stopped above o -- never for the searches
      // of the hash-chain parser (o is 2, 1 and 2 for its three searches and only grows), so
      // nothing is read for the prefilter
      const bool cand = ok32 && lane >= k0 && len > longest;
      const bool sure = longest - 1 - br >= back;
      bool pass = cand && sure;
      if (ballot(cand && !sure)) {
        const bool rd = cand && !sure;
        const int a = ilow + longest - 1, q = c - br + longest - 1;
        // (a candidate that is read has q >= 0: its low limit lies inside the block)
        const uint32_t x0 = ldb(s + (rd ? a : ip)), y0 = ldb(s + (rd ? q : ip));
        const uint32_t x1 = ldb(s + (rd ? a + 1 : ip)), y1 = ldb(s + (rd ? q + 1 : ip));
        pass = pass || (rd && x0 == y0 && x1 == y1);
      }
      const uint64_t m = ballot(pass);
      if (!m) break;
      const int k = __builtin_ctzll(m);
      longest = __shfl(len, k);
      mpos = __shfl(c + back, k);
      spos = ip + __shfl(back, k);
      k0 = k + 1;
    }
  }
  return longest;
}

// Sequences are queued, one per lane (literal start | literal length << 16, offset |
// matchlength-4 << 16), and written out 64 at a time: one round trip fetches the literals of
// 64 sequences, where writing each sequence as it is found costs one per sequence.
struct HcQueue {
  uint32_t q0, q1;
  int qn;
  int n;  // block size (bounds of the literal windows and the output stores)
};

// LZ4HC_encodeSequence (lz4hc.c:462-530), limitedOutput, for the queued sequences: 0 ok,
// 1 overflow (the block is stored raw, whichever sequence overflowed)
__device__ int hc_flush(const HcBlock &b, uintptr_t d, int &op, int oend, HcQueue &q) {
  const int lane = b.lane;
  const bool ch = lane < q.qn;
  const uint32_t lstart = q.q0 & 0xFFFFu, lit = ch ? q.q0 >> 16 : 0u;
  const uint32_t off = q.q1 & 0xFFFFu, l = q.q1 >> 16;
  const uint32_t lext = ext_bytes(lit);
  const uint32_t sz = ch ? 3u + lit + lext + ext_bytes(l) : 0u;
  uint32_t tot;
  const uint32_t tp = uint32_t(op) + wave_excl_scan(sz, tot);  // token
  const uint32_t lp = tp + 1u + lext;                          // first literal
  const uint32_t fp = lp + lit;                                // offset field
  const bool ov = ch && (int(tp + 1u + lit / 255u + lit + (2u + 1u + kLz4LastLiterals)) > oend ||
                         int(fp + 2u + l / 255u + (1u + kLz4LastLiterals)) > oend);
  if (ballot(ov)) return 1;
  const uintptr_t lo = b.s & ~uintptr_t(3);
  const rsrc_t rs = block_rsrc(lo, (b.s + uint32_t(q.n) + 3u) & ~uintptr_t(3));
  const uint32_t sa = uint32_t(b.s & 3u);
  const rsrc_t wd = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(d), 0, q.n, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b8(
      uint8_t(((lit < 15u ? lit : 15u) << 4) | (l < 15u ? l : 15u)), wd, ch ? tp : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off), wd, ch ? fp : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off >> 8), wd, ch ? fp + 1u : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(l - 15u), wd,
                                       (ch && l >= 15u && l < 270u) ? fp + 2u : kNoLoad, 0, 0);
  if (ballot(ch && lit >= 15u)) {
    if (ch && lit >= 15u) put_len(d + tp + 1u, lit);
  }
  if (ballot(ch && l >= 270u)) {
    if (ch && l >= 270u) put_len(d + fp + 2u, l);
  }
  const bool need_win = ch && lit != 0u && lit <= 16u;
  if (ballot(need_win)) {  // up to 16 literals: one 20-byte window per lane
    uint32_t w[5];
    load5(rs, need_win ? ((lstart + sa) & ~3u) : kNoLoad, w);
    const uint32_t sh = (lstart + sa) & 3u;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
#pragma unroll
    for (uint32_t k = 0; k < 16u; ++k)
      __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v[k >> 2] >> (8u * (k & 3u))), wd,
                                           (need_win && k < lit) ? lp + k : kNoLoad, 0, 0);
  }
  uint64_t longm = ballot(ch && lit > 16u);  // long runs: the whole wave copies them
  while (longm) {
    const int j = __builtin_ctzll(longm);
    longm &= longm - 1;
    hc_copy(d + __builtin_amdgcn_readlane(lp, j), b.s + __builtin_amdgcn_readlane(lstart, j),
            int(__builtin_amdgcn_readlane(lit, j)), lane);
  }
  op += int(tot);
  q.qn = 0;
  return 0;
}

// queue the sequence (literals anchor..ip, match of ml bytes at ref) and step over it
__device__ __forceinline__ int hc_encode(const HcBlock &b, uintptr_t d, int &op, int oend, int &ip,
                                         int &anchor, int ml, int ref, HcQueue &q) {
  if (q.qn == 64 && hc_flush(b, d, op, oend, q)) return 1;
  const bool me = b.lane == q.qn;
  q.q0 = me ? uint32_t(anchor) | (uint32_t(ip - anchor) << 16) : q.q0;
  q.q1 = me ? uint32_t(ip - ref) | (uint32_t(ml - kLz4MinMatch) << 16) : q.q1;
  q.qn++;
  ip += ml;
  anchor = ip;
  return 0;
}

// Whether the main loop's search at p (longest = MINMATCH-1) certainly finds
// nothing: none of its first min(rank, attempts) chain candidates repeats the
// 4 bytes at p (the only way such a search can succeed; lz4hc.c:264-266).
// Positions it cannot settle cheaply (long buckets, level-9 repetitive
// patterns) report false and get the full search.
constexpr int kHcSure = 8;  // candidates a position may have and still be settled here
__device__ __forceinline__ bool hc_sure_miss(const HcBlock &b, int p, int mflimit) {
  // every load is unconditional on a clamped address (a predicated load is waited for at
  // once): two dependent round trips per 64 positions (the position's table entry, then its
  // candidates' fingerprints), not one per candidate.  A position up to mflimit has 11 block
  // bytes behind it, so the 8-byte read stays inside.
  const bool in = p <= mflimit;
  const int pc = in ? p : mflimit;
  const uint32_t pat = ld32u_nb(b.s + pc);
  const uint32_t t = b.tr[pc];
  const bool rep = b.pa && ((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24));
  const int r = int(t >> 16);
  const int total = r < b.attempts ? r : b.attempts;
  const int top = int(t & 0xFFFFu) - 1;
  // positions that cannot be settled here read nothing of their own (their loads go to the
  // first fingerprint, one line for the wave)
  const bool open = !in || rep || total > kHcSure;
  const int nt = open ? 0 : total;
  // a candidate whose fingerprint differs from the position's cannot repeat its 4 bytes; one
  // that matches it is left to the full search
  uint32_t w[kHcSure];
#pragma unroll
  for (int j = 0; j < kHcSure; ++j) w[j] = b.sorted[j < nt ? top - j : 0] >> 16;
  bool miss = true;
#pragma unroll
  for (int j = 0; j < kHcSure; ++j)
    if (j < nt && w[j] == (pat & 0xFFFFu)) miss = false;
  return !open && miss;  // (total == 0: nothing to test)
}

// LZ4HC_compress_hashChain (lz4hc.c:532-746).  Returns the compressed size or
// 0 when the block does not fit in n-1 bytes.  n >= 13.
__device__ int hc_compress_block(const HcBlock &b, uintptr_t dst, int n, bool prebuilt) {
  const int mflimit = n - kLz4MFLimit, matchlimit = n - kLz4LastLiterals, oend = n - 1;
#ifdef RDK_HC_PROF
  const uint64_t t0 = wall_clock64();
#endif
  if (!prebuilt) hc_build(b, mflimit + 1);
#ifdef RDK_HC_PROF
  const uint64_t t1 = wall_clock64();
  int nskip = 0;
  for (int k = 0; k < 10; ++k) b.pc[k] = 0;
#endif
  int ip = 0, anchor = 0, op = 0, unused = 0;
  HcQueue q = {0u, 0u, 0, n};
  int ml, ml0, ml2, ml3, start0, ref0, ref = 0, start2 = 0, ref2 = 0, start3 = 0, ref3 = 0;
  int wbase = 0, wend = 0;  // positions [wbase, wend) have a sure-miss bit in wmiss
  uint64_t wmiss = 0;
  while (ip <= mflimit) {
    if (ip >= wend) {  // 64 positions settled in parallel, one per lane
      wbase = ip;
      wend = ip + 64;
      HC_T0();
      wmiss = ballot(hc_sure_miss(b, ip + b.lane, mflimit));
      HC_ADD(6);
      HC_CNT(7, 1);
    }
    const uint64_t run = ~(wmiss >> (ip - wbase));
    if (!(run & 1u)) {  // the reference steps ip++ over each of these (lz4hc.c:568)
#ifdef RDK_HC_PROF
      nskip += run ? __builtin_ctzll(run) : wend - ip;
#endif
      ip += run ? __builtin_ctzll(run) : wend - ip;
      continue;
    }
    ml = hc_search(b, ip, ip, matchlimit, kLz4MinMatch - 1, ref, unused);
    if (ml < kLz4MinMatch) { ip++; continue; }
    start0 = ip; ref0 = ref; ml0 = ml;
  search2:
    if (ip + ml <= mflimit)
      ml2 = hc_search(b, ip + ml - 2, ip, matchlimit, ml, ref2, start2);
    else
      ml2 = ml;
    if (ml2 == ml) {
      if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref, q)) return 0;
      continue;
    }
    if (start0 < ip && start2 < ip + ml0) { ip = start0; ref = ref0; ml = ml0; }
    if (start2 - ip < 3) { ml = ml2; ip = start2; ref = ref2; goto search2; }
  search3:
    if (start2 - ip < kHcOptimalML) {
      int nml = ml > kHcOptimalML ? kHcOptimalML : ml;
      if (ip + nml > start2 + ml2 - kLz4MinMatch) nml = start2 - ip + ml2 - kLz4MinMatch;
      const int corr = nml - (start2 - ip);
      if (corr > 0) { start2 += corr; ref2 += corr; ml2 -= corr; }
    }
    if (start2 + ml2 <= mflimit)
      ml3 = hc_search(b, start2 + ml2 - 3, start2, matchlimit, ml2, ref3, start3);
    else
      ml3 = ml2;
    if (ml3 == ml2) {
      if (start2 < ip + ml) ml = start2 - ip;
      if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref, q)) return 0;
      ip = start2;
      if (hc_encode(b, dst, op, oend, ip, anchor, ml2, ref2, q)) return 0;
      continue;
    }
    if (start3 < ip + ml + 3) {
      if (start3 >= ip + ml) {
        if (start2 < ip + ml) {
          const int corr = ip + ml - start2;
          start2 += corr; ref2 += corr; ml2 -= corr;
          if (ml2 < kLz4MinMatch) { start2 = start3; ref2 = ref3; ml2 = ml3; }
        }
        if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref, q)) return 0;
        ip = start3; ref = ref3; ml = ml3;
        start0 = start2; ref0 = ref2; ml0 = ml2;
        goto search2;
      }
      start2 = start3; ref2 = ref3; ml2 = ml3;
      goto search3;
    }
    if (start2 < ip + ml) {
      if (start2 - ip < kHcOptimalML) {
        if (ml > kHcOptimalML) ml = kHcOptimalML;
        if (ip + ml > start2 + ml2 - kLz4MinMatch) ml = start2 - ip + ml2 - kLz4MinMatch;
        const int corr = ml - (start2 - ip);
        if (corr > 0) { start2 += corr; ref2 += corr; ml2 -= corr; }
      } else {
        ml = start2 - ip;
      }
    }
    if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref, q)) return 0;
    ip = start2; ref = ref2; ml = ml2;
    start2 = start3; ref2 = ref3; ml2 = ml3;
    goto search3;
  }
  if (hc_flush(b, dst, op, oend, q)) return 0;
  {  // last literals (lz4hc.c:709-734)
    const int run = n - anchor;
    if (op + 1 + (run + 255 - 15) / 255 + run > oend) return 0;
    if (run >= 15) {
      const int a = run - 15;
      if (b.lane == 0) stb(dst + op, 15u << 4);
      hc_run(dst + op + 1, a / 255, a % 255, b.lane);
      op += 1 + a / 255 + 1;
    } else {
      if (b.lane == 0) stb(dst + op, uint32_t(run) << 4);
      op += 1;
    }
    hc_copy(dst + op, b.s + anchor, run, b.lane);
    op += run;
  }
#ifdef RDK_HC_PROF
  if (b.lane == 0 && blockIdx.x < 4)
    printf("HCPROF blk %d n %d build_us %.1f parse_us %.1f skipped %d out %d | s1 cyc %llu n %llu | s2 cyc %llu n %llu | steps %llu serial %llu | miss cyc %llu n %llu\n", int(blockIdx.x), n,
           double(t1 - t0) / 100.0, double(wall_clock64() - t1) / 100.0, nskip, op,
           (unsigned long long)b.pc[0], (unsigned long long)b.pc[2], (unsigned long long)b.pc[1], (unsigned long long)b.pc[3],
           (unsigned long long)b.pc[4], (unsigned long long)b.pc[5], (unsigned long long)b.pc[6], (unsigned long long)b.pc[7]);
#endif
  return op;
}

// ------------------------------------------------------------ levels 10..12
// LZ4HC_InsertAndGetWiderMatch as LZ4HC_FindLongerMatch drives it (forward only,
// chain swap on) for a pattern that is not one repeated byte, so that pattern
// analysis never redirects the walk.  64 candidates of the current chain per step.
__device__ int hc_search_swap(const HcBlock &b, int ip, int ihigh, int longest, int &mpos,
                              const uint32_t sw[9], uint32_t t_first, bool wide) {
  const uintptr_t s = b.s;
  const int lane = b.lane;
  const uint32_t pat = sw[0];
  int attempts = b.attempts;
  int q = ip, cp = 0;  // the walk follows the chain of position q = candidate + cp
  uint32_t t = t_first;  // tr[q]
  for (;;) {
    const int r = int(t >> 16), top = int(t & 0xFFFFu) - 1;
    const int total = r < attempts ? r : attempts;
    bool swapped = false;
    for (int c0 = 0; c0 < total; c0 += 64) {
      const int j = c0 + lane;
      const bool inq = j < total;
      const int m = int(b.sorted[inq ? top - j : top] & 0xFFFFu) - cp;  // (clamped, not predicated)
      const bool valid = inq && m >= 0;
      bool ok32;
      int len = 0;
      if (wide) {  // the candidate's 36 bytes in one round trip (m < ip, ip + 48 <= ihigh)
        uint32_t cw[9];
        hc_load_words<9>(s + (valid ? m : ip), cw);
        ok32 = valid && cw[0] == pat;
        int fwd = 32;
#pragma unroll
        for (int k = 8; k >= 1; --k) {
          const uint32_t z = sw[k] ^ cw[k];
          if (z) fwd = 4 * (k - 1) + (__builtin_ctz(z) >> 3);
        }
        if (ballot(ok32 && fwd == 32)) {
          if (ok32 && fwd == 32) fwd += hc_count(s, ip + 36, m + 36, ihigh);
        }
        len = ok32 ? 4 + fwd : 0;
      } else {
        ok32 = valid && ld32u(s + m) == pat;
        if (ok32) len = 4 + hc_count(s, ip + 4, m + 4, ihigh);
      }
      int k0 = 0;
      for (;;) {  // the reference's order: the next candidate that ties or beats `longest`
        bool pass = ok32 && lane >= k0 && len >= longest;
        if (pass && len == longest) {
          // only a count cut short by ihigh can tie; the read16 prefilter (lz4hc.c:284)
          // then decides whether the reference measured this candidate at all
          const int a = ip + longest - 1, c = m + longest - 1;
          pass = ldb(s + a) == ldb(s + c) && ldb(s + a + 1) == ldb(s + c + 1);
        }
        const uint64_t mk = ballot(pass);
        if (!mk) break;
        const int k = __builtin_ctzll(mk);
        const int lk = __shfl(len, k), mm = __shfl(m, k);
        if (lk > longest) { longest = lk; mpos = mm; }
        if (mm + longest <= ip) {  // chain swap, lz4hc.c:312-334
          int dist, ncp = cp;
          hc_swap_scan(b, mm, longest, dist, ncp);
          if (dist > 1) {
            cp = ncp;
            attempts -= c0 + k + 1;
            q = mm + cp;
            swapped = true;
            break;
          }
        }
        k0 = k + 1;
      }
      if (swapped) break;
      if (ballot(inq && !valid)) return longest;  // the chain left the block: the walk ends
    }
    if (!swapped || attempts <= 0) break;  // chain or attempts used up
    t = b.tr[q];
  }
  return longest;
}

// LZ4HC_FindLongerMatch (lz4hc.c:1255-1275), favorCompressionRatio: the length
// (0 when nothing beats min_len) and the offset
__device__ int hc_longer(const HcBlock &b, int ip, int ihigh, int min_len, int &off) {
  // the source's 36 bytes (the pattern first) and the table entry in one round trip; the
  // last positions of a block, where the windows would run over its end, read as the
  // reference does
  const bool wide = ip + 48 <= ihigh;
  uint32_t sw[9];
  if (wide) {
    hc_load_words<9>(b.s + ip, sw);
  } else {
#pragma unroll
    for (int k = 1; k < 9; ++k) sw[k] = 0;
    sw[0] = ld32u(b.s + ip);
  }
  const uint32_t t0 = b.tr[ip];
  const uint32_t pat = sw[0];
  int mpos = 0, spos = ip, len;
  if (((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24)))
    len = hc_search_serial(b, ip, ip, ihigh, min_len, mpos, spos, pat, true);
  else
    len = hc_search_swap(b, ip, ihigh, min_len, mpos, sw, t0, wide);
  if (len <= min_len) return 0;
  off = ip - mpos;
  return len;
}

// LZ4HC_literalsPrice / LZ4HC_sequencePrice (lz4hc.c:1224-1247), in bytes
__device__ __forceinline__ int hc_lit_price(int litlen) {
  return litlen + (litlen >= 15 ? 1 + (litlen - 15) / 255 : 0);
}
__device__ __forceinline__ int hc_seq_price(int litlen, int mlen) {
  return 3 + hc_lit_price(litlen) + (mlen >= 19 ? 1 + (mlen - 19) / 255 : 0);
}

// opt[] accessors: entries are written by one lane (or one entry per lane) and read
// back by the whole wave; hc_opt_sync() between a write and a dependent read.
__device__ __forceinline__ int4 hc_opt_ld(const HcBlock &b, int i) { return b.opt[i]; }
__device__ __forceinline__ void hc_opt_st(const HcBlock &b, int i, int price, int off, int mlen,
                                          int litlen) {
  if (b.lane == 0) b.opt[i] = make_int4(price, off, mlen, litlen);
}
__device__ __forceinline__ void hc_opt_sync() { __threadfence_block(); }

// opt[last+1 .. last+3]: literals after the last match (lz4hc.c:1354-1362, :1451-1458)
__device__ __forceinline__ void hc_opt_trailing(const HcBlock &b, int last, int last_price) {
  if (b.lane >= 1 && b.lane <= kHcTrailing)
    b.opt[last + b.lane] = make_int4(last_price + hc_lit_price(b.lane), 0, 1, b.lane);
}

// LZ4HC_compress_optimal (lz4hc.c:1278-1538), limitedOutput.  Returns the compressed
// size or 0 when the block does not fit in n-1 bytes.  n >= 13.
__device__ int hc_optimal_block(const HcBlock &b, uintptr_t dst, int n, int sufficient, bool full,
                                bool prebuilt) {
  const int mflimit = n - kLz4MFLimit, matchlimit = n - kLz4LastLiterals, oend = n - 1;
  const int lane = b.lane;
  if (!prebuilt) hc_build(b, mflimit + 1);
  if (sufficient >= kHcOptNum) sufficient = kHcOptNum - 1;
  int ip = 0, anchor = 0, op = 0;
  HcQueue q = {0u, 0u, 0, n};
  while (ip <= mflimit) {
    const int llen = ip - anchor;
    int best_mlen, best_off, cur, last_pos, foff = 0;
    const int flen = hc_longer(b, ip, matchlimit, kLz4MinMatch - 1, foff);
    if (flen == 0) { ip++; continue; }
    if (flen > sufficient) {  // good enough: immediate encoding (lz4hc.c:1318-1326)
      if (hc_encode(b, dst, op, oend, ip, anchor, flen, ip - foff, q)) return 0;
      continue;
    }
    // prices of the first positions: literals (lz4hc.c:1329-1338), then the first match at
    // every length (:1340-1352), one entry per lane
    for (int base = 0; base <= flen; base += 64) {
      const int r = base + lane;
      if (r < kLz4MinMatch) b.opt[r] = make_int4(hc_lit_price(llen + r), 0, 1, llen + r);
      else if (r <= flen) b.opt[r] = make_int4(hc_seq_price(llen, r), foff, r, llen);
    }
    last_pos = flen;
    hc_opt_trailing(b, last_pos, hc_seq_price(llen, flen));
    hc_opt_sync();
    bool direct = false;
    for (cur = 1; cur < last_pos; cur++) {  // lz4hc.c:1365-1459
      const int cpos = ip + cur;
      if (cpos > mflimit) break;
      const int4 oc = hc_opt_ld(b, cur);
      const int p1 = hc_opt_ld(b, cur + 1).x, p4 = hc_opt_ld(b, cur + kLz4MinMatch).x;
      // not useful to search here if the next position is as cheap (:1372-1381)
      if (full ? (p1 <= oc.x && p4 < oc.x + 3) : (p1 <= oc.x)) continue;
      int noff = 0;
      const int nlen = hc_longer(b, cpos, matchlimit, full ? kLz4MinMatch - 1 : last_pos - cur, noff);
      if (!nlen) continue;
      if (nlen > sufficient || nlen + cur >= kHcOptNum) {  // immediate encoding (:1391-1398)
        best_mlen = nlen;
        best_off = noff;
        last_pos = cur + 1;
        direct = true;
        break;
      }
      // literals after cur (:1401-1413), one length per lane
      if (lane >= 1 && lane < kLz4MinMatch) {
        const int price = oc.x - hc_lit_price(oc.w) + hc_lit_price(oc.w + lane);
        if (price < b.opt[cur + lane].x) b.opt[cur + lane] = make_int4(price, 0, 1, oc.w + lane);
      }
      // the match at cur at every length (:1416-1449), one length per lane
      int ll, pbase;
      if (oc.z == 1) {
        ll = oc.w;
        pbase = cur > ll ? hc_opt_ld(b, cur - ll).x : 0;
      } else {
        ll = 0;
        pbase = oc.x;
      }
      int new_last = last_pos;
      for (int base = kLz4MinMatch; base <= nlen; base += 64) {
        const int ml = base + lane;
        if (ml <= nlen) {
          const int pos = cur + ml;
          const int price = pbase + hc_seq_price(ll, ml);
          if (pos > last_pos + kHcTrailing || price <= b.opt[pos].x) {
            if (ml == nlen && last_pos < pos) new_last = pos;
            b.opt[pos] = make_int4(price, noff, ml, ll);
          }
        }
      }
      // only the lane of the last length can have moved last_pos
      last_pos = int(__builtin_amdgcn_readlane(new_last, (nlen - kLz4MinMatch) & 63));
      hc_opt_sync();
      hc_opt_trailing(b, last_pos, hc_opt_ld(b, last_pos).x);
      hc_opt_sync();
    }
    if (!direct) {
      const int4 ol = hc_opt_ld(b, last_pos);
      best_mlen = ol.z;
      best_off = ol.y;
      cur = last_pos - best_mlen;
    }
    {  // reverse traversal: the cheapest path becomes a forward list (lz4hc.c:1470-1484)
      int cand = cur, sel_ml = best_mlen, sel_off = best_off;
      for (;;) {
        const int4 o = hc_opt_ld(b, cand);
        hc_opt_st(b, cand, o.x, sel_off, sel_ml, o.w);
        sel_ml = o.z;
        sel_off = o.y;
        if (o.z > cand) break;
        cand -= o.z;
      }
      hc_opt_sync();
    }
    {  // encode the recorded sequences in order (lz4hc.c:1487-1498), 64 entries per load
      int r = 0, rb = -64;
      int4 e = make_int4(0, 0, 0, 0);
      while (r < last_pos) {
        if (r >= rb + 64) {
          rb = r;
          e = b.opt[rb + lane];  // entries past last_pos are never used
        }
        const int ml = int(__builtin_amdgcn_readlane(e.z, r - rb));
        if (ml == 1) { ip++; r++; continue; }
        const int off = int(__builtin_amdgcn_readlane(e.y, r - rb));
        r += ml;
        if (hc_encode(b, dst, op, oend, ip, anchor, ml, ip - off, q)) return 0;
      }
    }
  }
  if (hc_flush(b, dst, op, oend, q)) return 0;
  {  // last literals (lz4hc.c:1501-1526)
    const int run = n - anchor;
    if (op + 1 + (run + 255 - 15) / 255 + run > oend) return 0;
    if (run >= 15) {
      const int a = run - 15;
      if (lane == 0) stb(dst + op, 15u << 4);
      hc_run(dst + op + 1, a / 255, a % 255, lane);
      op += 1 + a / 255 + 1;
    } else {
      if (lane == 0) stb(dst + op, uint32_t(run) << 4);
      op += 1;
    }
    hc_copy(dst + op, b.s + anchor, run, lane);
    op += run;
  }
  return op;
}

// real_items = n * (blocks of the longest frame): the slot-major items at or past it are the
// empty block slots of short frames, and a chunk made of them only is skipped.
__global__ __launch_bounds__(256) void lz4hc_count_items_kernel(const uint32_t *__restrict__ in_lens,
                                                                uint32_t n, uint32_t *real_items) {
  __shared__ uint32_t wmax[4];
  uint32_t m = 0;
  for (uint32_t f = threadIdx.x; f < n; f += 256u) {
    const uint32_t nb = (in_lens[f] + kLz4Block - 1) / kLz4Block;
    m = nb > m ? nb : m;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t o = uint32_t(__shfl_xor(int(m), d));
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) m = wmax[w] > m ? wmax[w] : m;
    const uint64_t r = uint64_t(m < uint32_t(kHcItems) ? m : uint32_t(kHcItems)) * n;
    *real_items = uint32_t(r);
  }
}

// The build phase for the first block of every item of [it0, it1), with the hash heads on
// chip: one workgroup per block, head[] (last position and bucket rank per hash, 128 KiB) in
// LDS.  Wave 0 runs the ordered pass over the positions (hash chain delta and rank inside the
// hash bucket, 64 positions per step); all waves then turn the bucket sizes into bucket
// starts and scatter the positions into `sorted`.  Everything that goes to memory is a
// coalesced stream except the u16 scatter into the block's own 128 KiB `sorted`.  (A wave
// that builds in its own HBM scratch, hc_build(), reads and rewrites a random 64-byte line
// of a 128 KiB table per position: with thousands of waves resident that was most of the
// engine's memory traffic.)
constexpr int kHcBuildThreads = 1024;
constexpr int kHcAhead = 8;  // source words in flight per lane of the ordered pass

__global__ __launch_bounds__(kHcBuildThreads) void lz4hc_build_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint32_t n, uint8_t *scratch, uint32_t it0, uint32_t it1,
    const uint32_t *__restrict__ real_items) {
  if (it0 >= *real_items) return;  // every item of this chunk is an empty block slot
  __shared__ uint32_t head[1 << kHcHashLog];
  __shared__ uint32_t part[kHcBuildThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int kWaves = kHcBuildThreads / 64;
  for (uint32_t it = it0 + blockIdx.x; it < it1; it += gridDim.x) {
    const uint32_t f = it % n, k = it / n;
    const uint32_t len = in_lens[f];
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    if (k >= nb) continue;
    const uint32_t bn = (len - k * kLz4Block) < kLz4Block ? (len - k * kLz4Block) : kLz4Block;
    if (bn < uint32_t(kLz4MFLimit + 1)) continue;
    const int npos = int(bn) - kLz4MFLimit + 1;  // positions 0 .. mflimit
    const uintptr_t s = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kLz4Block;
    uint8_t *sc = scratch + size_t(it - it0) * kHcScratch;
    uint16_t *chain = reinterpret_cast<uint16_t *>(sc + kHcTab);
    uint32_t *sorted = reinterpret_cast<uint32_t *>(chain + 65536);
    uint32_t *tr = sorted + 65536;
    for (int i = tid; i < (1 << kHcHashLog); i += kHcBuildThreads) head[i] = kHcNone;
    __syncthreads();
    if (wave == 0) {
      const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
      const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
      // the source words of the next kHcAhead steps are in flight (they do not depend on
      // the head[] updates), so a step waits on LDS only; a position below npos has at
      // least 11 block bytes behind it, so the branch-free 8-byte read stays inside
      // (kept as raw dword pairs and aligned at the use, so that no step waits for a
      // load issued after its own)
      uint32_t wl[kHcAhead], wh[kHcAhead];
      const uint32_t sh = uint32_t((s + lane) & 3u);
#pragma unroll
      for (int j = 0; j < kHcAhead; ++j) {
        const uintptr_t a = (s + min(lane + 64 * j, npos - 1)) & ~uintptr_t(3);
        wl[j] = *(g_cu32 *)a;
        wh[j] = *(g_cu32 *)(a + 4);
      }
      for (int base0 = 0; base0 < npos; base0 += 64 * kHcAhead) {
#pragma unroll
        for (int j = 0; j < kHcAhead; ++j) {
          const int base = base0 + 64 * j;
          const int p = base + lane;
          const bool valid = p < npos;
          const uint32_t h = valid ? hc_hash(__builtin_amdgcn_alignbyte(wh[j], wl[j], sh)) : 0u;
          {  // (clamped, not predicated: a predicated load is waited for at once)
            const uintptr_t a = (s + min(p + 64 * kHcAhead, npos - 1)) & ~uintptr_t(3);
            wl[j] = *(g_cu32 *)a;
            wh[j] = *(g_cu32 *)(a + 4);
          }
          const uint64_t eq = same_value_lanes<kHcHashLog>(h, ballot(valid));
          const uint32_t hv = valid ? head[h] : kHcNone;
          const uint64_t eb = eq & below;
          const uint32_t rk = (hv == kHcNone ? 0u : (hv >> 16) + 1u) + uint32_t(__popcll(eb));
          int prev;
          if (eb) prev = base + (63 - __clzll(eb));
          else prev = hv == kHcNone ? -65536 : int(hv & 0xFFFFu);
          if (valid) {
            const int d = p - prev;  // LZ4HC_Insert (lz4hc.c:125-132)
            chain[p] = uint16_t(d > 65535 ? 65535 : d);
            tr[p] = h | (rk << 16);  // the scatter below takes hash and rank from here
            if (!(eq & above)) head[h] = uint32_t(p) | (rk << 16);
          }
        }
      }
    }
    __syncthreads();
    // bucket sizes -> bucket starts: every wave sums its quarter of the table, then scans it
    // row by row from the sum of the quarters before it
    constexpr int kRows = (1 << kHcHashLog) / 64 / kWaves;
    uint32_t *mine = head + wave * kRows * 64;
    uint32_t sum = 0;
    for (int r = 0; r < kRows; ++r) {
      const uint32_t v = mine[r * 64 + lane];
      sum += v == kHcNone ? 0u : (v >> 16) + 1u;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d);
    if (lane == 0) part[wave] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int w = 0; w < wave; ++w) run += part[w];
    for (int r = 0; r < kRows; ++r) {
      const uint32_t v = mine[r * 64 + lane];
      const uint32_t c = v == kHcNone ? 0u : (v >> 16) + 1u;
      uint32_t tot;
      const uint32_t excl = wave_excl_scan(c, tot);
      mine[r * 64 + lane] = run + excl;
      run += tot;
    }
    __syncthreads();
    // scatter, four steps' loads issued before their stores
    for (int p0 = tid; p0 < npos; p0 += 4 * kHcBuildThreads) {
      uint32_t t[4], v0[4], v1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = p0 + kHcBuildThreads * j;
        t[j] = p < npos ? tr[p] : 0u;
        // the position's 4 bytes for its fingerprint (clamped, not predicated)
        const uintptr_t a = (s + min(p, npos - 1)) & ~uintptr_t(3);
        v0[j] = *(g_cu32 *)a;
        v1[j] = *(g_cu32 *)(a + 4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = p0 + kHcBuildThreads * j;
        if (p < npos) {
          const uint32_t r = t[j] >> 16;
          const uint32_t idx = head[t[j] & 0x7FFFu] + r;
          sorted[idx] = uint32_t(p) |
                        (__builtin_amdgcn_alignbyte(v1[j], v0[j], uint32_t((s + p) & 3u)) << 16);
          tr[p] = idx | (r << 16);
        }
      }
    }
    __syncthreads();  // head[] is reused by the next item
  }
}

// OPT: the optimal parser (levels 10..12), a kernel of its own so that its registers do
// not cost the hash-chain parser its residency.  Items [it0, it1) come from a work queue;
// item `it` has its tables at scratch + (it - it0) * kHcScratch, built by lz4hc_build_kernel
// for its first block (frames of more than 64 blocks: the wave builds the further ones
// itself, in the same tables).
// (four waves per SIMD: a 4096-item chunk is resident at once)
template <bool OPT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void lz4hc_compress_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t n, int attempts, int sufficient,
    uint8_t *scratch, uint32_t *__restrict__ next_item, uint32_t it0, uint32_t it1,
    const uint32_t *__restrict__ real_items) {
  if (it0 >= *real_items) return;  // every item of this chunk is an empty block slot
  HcBlock b;
  b.lane = threadIdx.x;
  b.attempts = attempts;
  // the optimal parser always searches with pattern analysis (lz4hc.c:1267), the
  // hash-chain parser from level 9 (lz4hc.c:544)
  b.pa = OPT ? 1 : attempts > 128;
  // Work queue over (block slot, frame) items, slot-major: every wave takes
  // the next item when it finishes one, so the parse's uneven cost per block
  // spreads over the whole grid; the empty slots of short frames come last
  // and cost one atomic each.
  for (;;) {
    uint32_t it = 0;
    if (b.lane == 0) it = atomicAdd(next_item, 1u);
    it = it0 + uni(it);
    if (it >= it1) break;
    uint8_t *sc = scratch + size_t(it - it0) * kHcScratch;
    b.head = reinterpret_cast<uint32_t *>(sc);
    b.chain = reinterpret_cast<uint16_t *>(sc + kHcTab);
    b.sorted = reinterpret_cast<uint32_t *>(b.chain + 65536);
    b.tr = b.sorted + 65536;
    b.opt = reinterpret_cast<int4 *>(b.tr + 65536);
    const uint32_t f = it % n, kk = it / n;
    const uint32_t len = uni(in_lens[f]);
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    for (uint32_t k = kk; k < nb; k += kHcItems) {
      const uint32_t bn = (len - k * kLz4Block) < kLz4Block ? (len - k * kLz4Block) : kLz4Block;
      b.s = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kLz4Block;
      const uintptr_t slot = reinterpret_cast<uintptr_t>(out) + out_offs[f] + 7u + uint64_t(k) * kHcSlot;
      // LZ4_minLength: shorter blocks are all literals and never fit in n-1
      // (the optimal parser has no such test, but its main loop never runs below 13 bytes
      // and its last-literals run cannot fit either)
      int csize = 0;
      if (bn >= uint32_t(kLz4MFLimit + 1))
        csize = OPT ? hc_optimal_block(b, slot + 4u, int(bn), sufficient, attempts == 16384, k == kk)
                    : hc_compress_block(b, slot + 4u, int(bn), k == kk);
      if (b.lane == 0) {
        const uint32_t w = csize ? uint32_t(csize) : (bn | 0x80000000u);  // LZ4F_makeBlock
        stb(slot, w & 0xFFu); stb(slot + 1, (w >> 8) & 0xFFu);
        stb(slot + 2, (w >> 16) & 0xFFu); stb(slot + 3, w >> 24);
      }
    }
  }
}

struct FuseCrc;
void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s, const FuseCrc *fuse);

// The hash/chain tables (kHcScratch bytes per item of a chunk) and the work-queue counters
// live in the calling thread's kScratchHc region: calls on different streams are ordered by
// scratch_acquire / scratch_release, so two streams never share the tables.  A batch runs
// in chunks of kHcGrid items: the build kernel, then the parser on one wave per item.
int lz4hc_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, int level, hipStream_t s) {
  if (!n) return 0;
  if (n > (0xFFFFFFFFu / kHcItems) - kHcGrid) return set_error(RDK_HIP_E_INVAL, "too many frames");
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  const uint32_t items = n * uint32_t(kHcItems);
  const uint32_t chunk = items < kHcGrid ? items : kHcGrid;  // a single drop-in frame: 64 items
  const uint32_t nchunks = (items + chunk - 1) / chunk;
  const size_t counters = (size_t(nchunks + 1) * sizeof(uint32_t) + 255) & ~size_t(255);
  int rc = scratch_acquire(c, kScratchHc, size_t(kHcScratch) * chunk + counters, s);
  if (rc) return rc;
  uint8_t *p = c->d_stage[kScratchHc];
  // clTable (lz4hc.c:775-789): nbSearches, and the optimal parser's sufficient length
  if (level > 12) level = 12;  // MIN(LZ4HC_CLEVEL_MAX, cLevel), lz4hc.c:798
  const int attempts = level >= 12 ? 16384 : level == 11 ? 512 : level == 10 ? 96 : 1 << (level - 1);
  const int sufficient = level >= 12 ? kHcOptNum : level == 11 ? 128 : level == 10 ? 64 : 0;
  uint32_t *next_item = reinterpret_cast<uint32_t *>(p + size_t(kHcScratch) * chunk);
  RDK_HIP_CHECK(hipMemsetAsync(next_item, 0, size_t(nchunks) * sizeof(uint32_t), s));
  uint32_t *real_items = next_item + nchunks;
  hipLaunchKernelGGL(lz4hc_count_items_kernel, dim3(1), dim3(256), 0, s, d_in_lens, n, real_items);
  for (uint32_t ci = 0; ci < nchunks; ++ci) {
    const uint32_t it0 = ci * chunk, it1 = it0 + chunk < items ? it0 + chunk : items;
    const unsigned grid = it1 - it0;
    hipLaunchKernelGGL(lz4hc_build_kernel, dim3(grid), dim3(kHcBuildThreads), 0, s, d_in, d_in_offs,
                       d_in_lens, n, p, it0, it1, real_items);
    if (sufficient)
      hipLaunchKernelGGL(lz4hc_compress_blocks_kernel<true>, dim3(grid), dim3(64), 0, s, d_in,
                         d_in_offs, d_in_lens, d_out, d_out_offs, n, attempts, sufficient, p,
                         next_item + ci, it0, it1, real_items);
    else
      hipLaunchKernelGGL(lz4hc_compress_blocks_kernel<false>, dim3(grid), dim3(64), 0, s, d_in,
                         d_in_offs, d_in_lens, d_out, d_out_offs, n, attempts, sufficient, p,
                         next_item + ci, it0, it1, real_items);
  }
  lz4f_assemble_launch(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, s, nullptr);
  RDK_HIP_CHECK(hipGetLastError());
  return scratch_release(c, kScratchHc, s);
}

}  // namespace rdk
