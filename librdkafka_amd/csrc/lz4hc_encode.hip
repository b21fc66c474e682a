// lz4hc_encode.hip -- LZ4F frame compression at compression.level 3..9 (LZ4HC
// hash chain) on gfx950.
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
#include <hip/hip_runtime.h>

#include <mutex>

#include "common.h"
#include "lz4_device.h"

namespace rdk {

constexpr int kHcItems = 64;                 // block slots per frame per pass
constexpr uint32_t kHcSlot = kLz4Block + 4;  // worst-case bytes per block in a frame
constexpr int kHcHashLog = 15;               // lz4hc.h:196
constexpr uint32_t kHcNone = 0xFFFFFFFFu;
constexpr int kHcOptimalML = 18;             // lz4hc.c:74
constexpr size_t kHcTab = size_t(4) << kHcHashLog;  // head / bucket start, u32
constexpr size_t kHcScratch = kHcTab + 3 * 65536 * 2 + 65536 * 4;  // + chain, rank, sorted (u16), tr (u32)
constexpr unsigned kHcGrid = 4096;  // 16 waves per CU (the kernel fits 20)

struct HcBlock {
  uintptr_t s;       // block bytes (global)
  uint32_t *head;    // build: pos | rank << 16 per hash; then bucket start
  uint16_t *chain;   // DELTANEXTU16 per position
  uint16_t *rank;    // index of the position inside its hash bucket
  uint16_t *sorted;  // positions ordered by (hash, position)
  uint32_t *tr;      // per position: its index in sorted | its rank << 16
  int attempts;      // nbSearches
  int pa;            // patternAnalysis (levels 9+)
  int lane;
};

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
      const int i = base + lane + 64 * j;
      v[j] = i < len ? ldb(s + i) : 0u;
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
    if (valid) b.tr[p] = h;  // the scatter below reads the hash back from here
    uint64_t eq = ballot(valid);
#pragma unroll
    for (int bit = 0; bit < kHcHashLog; ++bit) {
      const bool on = (h >> bit) & 1u;
      const uint64_t m = ballot(on);
      eq &= on ? m : ~m;
    }
    const uint32_t hv = valid ? b.head[h] : kHcNone;
    const uint64_t eb = eq & below;
    const uint32_t rk = (hv == kHcNone ? 0u : (hv >> 16) + 1u) + uint32_t(__popcll(eb));
    int prev;
    if (eb) prev = base + (63 - __clzll(eb));
    else prev = hv == kHcNone ? -65536 : int(hv & 0xFFFFu);
    if (valid) {
      const int d = p - prev;  // LZ4HC_Insert (lz4hc.c:125-132)
      b.chain[p] = uint16_t(d > 65535 ? 65535 : d);
      b.rank[p] = uint16_t(rk);
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
    uint32_t h[4], r[4], st[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 + 64 * j;
      h[j] = p < npos ? b.tr[p] : 0u;
      r[j] = p < npos ? uint32_t(b.rank[p]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = b.head[h[j]];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 + 64 * j;
      if (p < npos) {
        const uint32_t idx = st[j] + r[j];
        b.sorted[idx] = uint16_t(p);
        b.tr[p] = idx | (r[j] << 16);
      }
    }
  }
  __threadfence_block();
}

// LZ4HC_InsertAndGetWiderMatch one candidate at a time (repetitive patterns
// at level 9, where pattern analysis may redirect the walk).
__device__ int hc_search_serial(const HcBlock &b, int ip, int ilow, int ihigh, int longest,
                                int &mpos, int &spos, uint32_t pat) {
  const uintptr_t s = b.s;
  const int br = ip - ilow;
  int attempts = b.attempts;
  int repeat = 0, src_pat_len = 0;  // 0 untested, 1 not, 2 confirmed
  int m = ip - int(b.chain[ip]);
  while (m >= 0 && attempts) {
    attempts--;
    {
      const int a = ilow + longest - 1, c = m - br + longest - 1;
      if (ldb(s + a) == ldb(s + c) && ldb(s + a + 1) == ldb(s + c + 1) && ld32u(s + m) == pat) {
        int back = 0;
        if (br) {
          const int lim = (ilow - ip) > -m ? (ilow - ip) : -m;
          while (back > lim && ldb(s + ip + back - 1) == ldb(s + m + back - 1)) back--;
        }
        const int len = 4 + hc_count(s, ip + 4, m + 4, ihigh) - back;
        if (len > longest) { longest = len; mpos = m + back; spos = ip + back; }
      }
    }
    const int dnext = b.chain[m];
    if (b.pa && dnext == 1) {
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
    m -= dnext;
  }
  return longest;
}

// LZ4HC_InsertAndGetWiderMatch, 64 chain candidates per step
__device__ int hc_search(const HcBlock &b, int ip, int ilow, int ihigh, int longest, int &mpos,
                         int &spos) {
  const uintptr_t s = b.s;
  const int lane = b.lane;
  const uint32_t pat = ld32u(s + ip);
  if (b.pa && ((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24)))
    return hc_search_serial(b, ip, ilow, ihigh, longest, mpos, spos, pat);
  const int br = ip - ilow;
  const uint32_t t = b.tr[ip];  // one load instead of rank -> hash -> bucket start
  const int r = int(t >> 16);
  const int top = int(t & 0xFFFFu) - 1;  // sorted[top] = latest earlier same-hash
  const int total = r < b.attempts ? r : b.attempts;
  for (int c0 = 0; c0 < total; c0 += 64) {
    const int j = c0 + lane;
    const bool valid = j < total;
    const int c = valid ? int(b.sorted[top - j]) : 0;
    const bool ok32 = valid && ld32u(s + c) == pat;
    int back = 0, len = 0;
    if (ok32) {
      if (br) {  // LZ4HC_countBack (lz4hc.c:140-152)
        const int lim = (ilow - ip) > -c ? (ilow - ip) : -c;
        while (back > lim && ldb(s + ip + back - 1) == ldb(s + c + back - 1)) back--;
      }
      len = 4 + hc_count(s, ip + 4, c + 4, ihigh) - back;
    }
    int k0 = 0;
    for (;;) {  // the reference's order: first improving candidate at the current longest
      bool pass = false;
      if (ok32 && lane >= k0 && len > longest) {
        const int a = ilow + longest - 1, q = c - br + longest - 1;
        pass = ldb(s + a) == ldb(s + q) && ldb(s + a + 1) == ldb(s + q + 1);
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

// LZ4HC_encodeSequence (lz4hc.c:462-530), limitedOutput: 0 ok, 1 overflow
__device__ int hc_encode(const HcBlock &b, uintptr_t d, int &op, int oend, int &ip, int &anchor,
                         int ml, int ref) {
  const int lane = b.lane;
  int o = op;
  const int tok = o++;
  const int lit = ip - anchor;
  if (o + lit / 255 + lit + (2 + 1 + kLz4LastLiterals) > oend) return 1;
  uint32_t token;
  if (lit >= 15) {
    const int l = lit - 15;
    token = 15u << 4;
    hc_run(d + o, l / 255, l % 255, lane);
    o += l / 255 + 1;
  } else {
    token = uint32_t(lit) << 4;
  }
  hc_copy(d + o, b.s + anchor, lit, lane);
  o += lit;
  const int off = ip - ref;
  if (lane == 0) {
    stb(d + o, uint32_t(off) & 0xFFu);
    stb(d + o + 1, (uint32_t(off) >> 8) & 0xFFu);
  }
  o += 2;
  int l = ml - kLz4MinMatch;
  if (o + l / 255 + (1 + kLz4LastLiterals) > oend) return 1;
  if (l >= 15) {
    token += 15u;
    l -= 15;
    hc_run(d + o, l / 255, l % 255, lane);
    o += l / 255 + 1;
  } else {
    token += uint32_t(l);
  }
  if (lane == 0) stb(d + tok, token);
  ip += ml;
  anchor = ip;
  op = o;
  return 0;
}

// Whether the main loop's search at p (longest = MINMATCH-1) certainly finds
// nothing: none of its first min(rank, attempts) chain candidates repeats the
// 4 bytes at p (the only way such a search can succeed; lz4hc.c:264-266).
// Positions it cannot settle cheaply (long buckets, level-9 repetitive
// patterns) report false and get the full search.
__device__ __forceinline__ bool hc_sure_miss(const HcBlock &b, int p, int mflimit) {
  if (p > mflimit) return false;
  const uint32_t pat = ld32u(b.s + p);
  if (b.pa && ((pat & 0xFFFFu) == (pat >> 16)) && ((pat & 0xFFu) == (pat >> 24))) return false;
  const uint32_t t = b.tr[p];
  const int r = int(t >> 16);
  const int total = r < b.attempts ? r : b.attempts;
  if (total == 0) return true;
  if (total > 8) return false;
  const int top = int(t & 0xFFFFu) - 1;
  int c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = j < total ? int(b.sorted[top - j]) : -1;
  bool miss = true;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (c[j] >= 0 && ld32u(b.s + c[j]) == pat) miss = false;
  return miss;
}

// LZ4HC_compress_hashChain (lz4hc.c:532-746).  Returns the compressed size or
// 0 when the block does not fit in n-1 bytes.  n >= 13.
__device__ int hc_compress_block(const HcBlock &b, uintptr_t dst, int n) {
  const int mflimit = n - kLz4MFLimit, matchlimit = n - kLz4LastLiterals, oend = n - 1;
#ifdef RDK_HC_PROF
  const uint64_t t0 = wall_clock64();
#endif
  hc_build(b, mflimit + 1);
#ifdef RDK_HC_PROF
  const uint64_t t1 = wall_clock64();
  int nskip = 0;
#endif
  int ip = 0, anchor = 0, op = 0, unused = 0;
  int ml, ml0, ml2, ml3, start0, ref0, ref = 0, start2 = 0, ref2 = 0, start3 = 0, ref3 = 0;
  int wbase = 0, wend = 0;  // positions [wbase, wend) have a sure-miss bit in wmiss
  uint64_t wmiss = 0;
  while (ip <= mflimit) {
    if (ip >= wend) {  // 64 positions settled in parallel, one per lane
      wbase = ip;
      wend = ip + 64;
      wmiss = ballot(hc_sure_miss(b, ip + b.lane, mflimit));
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
      if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref)) return 0;
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
      if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref)) return 0;
      ip = start2;
      if (hc_encode(b, dst, op, oend, ip, anchor, ml2, ref2)) return 0;
      continue;
    }
    if (start3 < ip + ml + 3) {
      if (start3 >= ip + ml) {
        if (start2 < ip + ml) {
          const int corr = ip + ml - start2;
          start2 += corr; ref2 += corr; ml2 -= corr;
          if (ml2 < kLz4MinMatch) { start2 = start3; ref2 = ref3; ml2 = ml3; }
        }
        if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref)) return 0;
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
    if (hc_encode(b, dst, op, oend, ip, anchor, ml, ref)) return 0;
    ip = start2; ref = ref2; ml = ml2;
    start2 = start3; ref2 = ref3; ml2 = ml3;
    goto search3;
  }
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
    printf("HCPROF blk %d n %d build_us %.1f parse_us %.1f skipped %d out %d\n", int(blockIdx.x), n,
           double(t1 - t0) / 100.0, double(wall_clock64() - t1) / 100.0, nskip, op);
#endif
  return op;
}

__global__ __launch_bounds__(64) void lz4hc_compress_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t n, int attempts, uint8_t *scratch,
    uint32_t *__restrict__ next_item) {
  HcBlock b;
  b.lane = threadIdx.x;
  uint8_t *sc = scratch + size_t(blockIdx.x) * kHcScratch;
  b.head = reinterpret_cast<uint32_t *>(sc);
  b.chain = reinterpret_cast<uint16_t *>(sc + kHcTab);
  b.rank = b.chain + 65536;
  b.sorted = b.rank + 65536;
  b.tr = reinterpret_cast<uint32_t *>(b.sorted + 65536);
  b.attempts = attempts;
  b.pa = attempts > 128;  // lz4hc.c:544
  // Work queue over (block slot, frame) items, slot-major: every wave takes
  // the next item when it finishes one, so the parse's uneven cost per block
  // spreads over the whole grid; the empty slots of short frames come last
  // and cost one atomic each.
  const uint32_t items = n * uint32_t(kHcItems);
  for (;;) {
    uint32_t it = 0;
    if (b.lane == 0) it = atomicAdd(next_item, 1u);
    it = uni(it);
    if (it >= items) break;
    const uint32_t f = it % n, kk = it / n;
    const uint32_t len = uni(in_lens[f]);
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    for (uint32_t k = kk; k < nb; k += kHcItems) {
      const uint32_t bn = (len - k * kLz4Block) < kLz4Block ? (len - k * kLz4Block) : kLz4Block;
      b.s = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kLz4Block;
      const uintptr_t slot = reinterpret_cast<uintptr_t>(out) + out_offs[f] + 7u + uint64_t(k) * kHcSlot;
      // LZ4_minLength: shorter blocks are all literals and never fit in n-1
      const int csize = bn >= uint32_t(kLz4MFLimit + 1) ? hc_compress_block(b, slot + 4u, int(bn)) : 0;
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

// The hash/chain tables (kHcScratch bytes per wave) and the work-queue counter live in
// the calling thread's kScratchHc region: calls on different streams are ordered by
// scratch_acquire / scratch_release, so two streams never share the tables.
int lz4hc_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, int level, hipStream_t s) {
  if (!n) return 0;
  if (n > (0xFFFFFFFFu / kHcItems) - kHcGrid) return set_error(RDK_HIP_E_INVAL, "too many frames");
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  const uint64_t items = uint64_t(n) * kHcItems;
  const unsigned grid = unsigned(items < kHcGrid ? items : kHcGrid);
  // a single drop-in frame needs 64 slices, a large batch the full grid
  int rc = scratch_acquire(c, kScratchHc, size_t(kHcScratch) * grid + 256, s);
  if (rc) return rc;
  uint8_t *p = c->d_stage[kScratchHc];
  const int attempts = 1 << (level - 1);  // clTable rows 3..9: 4 .. 256
  uint32_t *next_item = reinterpret_cast<uint32_t *>(p + size_t(kHcScratch) * grid);
  RDK_HIP_CHECK(hipMemsetAsync(next_item, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(lz4hc_compress_blocks_kernel, dim3(grid), dim3(64), 0, s, d_in, d_in_offs,
                     d_in_lens, d_out, d_out_offs, n, attempts, p, next_item);
  lz4f_assemble_launch(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, s, nullptr);
  RDK_HIP_CHECK(hipGetLastError());
  return scratch_release(c, kScratchHc, s);
}

}  // namespace rdk
