// snappy.hip -- snappy compression and decompression on gfx950.
//
// Replaces, for whole batches of MessageSets at a time, the codec behind
// rd_kafka_msgset_writer_compress_snappy (rdkafka_msgset_writer.c:1041) =
// rd_kafka_snappy_compress_iov (snappy.c:1488) -> sn_compress (:1408) ->
// compress_fragment (:957), and behind the reader's snappy case
// (rdkafka_msgset_reader.c:299-390) = rd_kafka_snappy_uncompress (snappy.c:1572)
// -> decompress_all_tags (:1226).
//
// COMPRESS.  sn_compress cuts the input into 64 KiB fragments and zeroes the hash
// table for each (get_hash_table, snappy.c:790), so fragments are independent: one
// wavefront per fragment, its u16 table (up to 2^14 entries, 32 KiB) in LDS.
// compress_fragment's greedy parse is emulated exactly, so streams are byte-identical
// to snappy.c's:
//   * the search evaluates 64 consecutive probes at once; the skip schedule
//     (bytes_between_hash_lookups = skip++ >> 5, :1019) is reproduced by a lane prefix
//     sum; a probe's candidate is the latest earlier probe of the step with the same
//     hash (14 ballots) or else the table entry; the first verifying probe wins and
//     only probes up to it update the table, last writer per hash;
//   * find_match_length, the literal copy and the copy elements of long matches
//     (emit_copy, :718) move 64 bytes / write 64 elements per wave step;
//   * after a copy the table takes ip-1 and the position behind the copy is tested at
//     once (:1071-1088).
// Fragment k of stream f is compressed into a slot of the caller's output buffer
// (4-byte size + payload; a fragment of this compressor grows by at most 1/64 + 8
// bytes, so the slots fit rd_kafka_snappy_max_compressed_length); an assemble kernel
// writes the varint32 length and slides the fragments together.
//
// DECOMPRESS.  A snappy stream has no block index, so one wavefront decodes one
// stream, 64 compressed bytes per step, with the discovery / pointer-doubling walk /
// lane-per-byte expansion scheme of the LZ4 block decoder (lz4_decode_fast.h): every
// lane parses the element that would start at its byte (tag + up to 3 bytes), the
// real elements are the orbit of the entry position under "next element", and the
// output is painted 64 bytes at a time from the input (literals), the wave's LDS
// history ring, or the already written output.  Elements whose header needs a fifth
// byte (literals of 16 MiB and more, 4-byte offsets) are parsed by a scalar routine.
// Every condition under which decompress_all_tags / writer_append* fail is checked
// (offset 0 or beyond the produced bytes, output or input overrun, a length that
// does not match the preamble), so the verdict is the reference's: 0 or -EIO.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "lz4_device.h"
#include "lz4_wave.h"
#include "win_ring.h"

namespace rdk {

typedef __attribute__((address_space(3))) uint16_t sn_lds_u16;
typedef __attribute__((address_space(3))) uint8_t sn_lds_u8;
typedef __amdgpu_buffer_rsrc_t sn_rsrc_t;

constexpr uint32_t kSnBlock = 65536;          // kblock_size, snappy.c:774
constexpr uint32_t kSnMaxTable = 1u << 14;    // kmax_hash_table_size, snappy.c:781
constexpr uint32_t kSnSlot = kSnBlock + 2048; // bytes per staged fragment (size word + payload)
constexpr uint32_t kSnSlot0 = 8;              // room for the varint32 in front of slot 0
constexpr int kSnItems = 64;                  // fragment slots per stream per pass
constexpr uint32_t kSnMul = 0x1e35a7bdu;      // hash_bytes, snappy.c:606
constexpr int kSnEIO = -5;
constexpr int kSnDstSize = -1001;             // RDK_HIP_SNAPPY_E_DSTSIZE

__device__ __forceinline__ uint32_t sn_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d);
    if (lane >= d) v += t;
  }
  return v;
}

// equal bytes a[i] == b[i], i < limit, 64 per wave step (find_match_length, snappy.c:823)
__device__ __forceinline__ uint32_t sn_count(uintptr_t a, uintptr_t b, uint32_t limit, int lane) {
  uint32_t cnt = 0;
  while (cnt < limit) {
    const uint32_t l = cnt + uint32_t(lane);
    const bool ok = l < limit && ldb(a + l) == ldb(b + l);
    const uint64_t m = ballot(ok);
    const uint32_t run = m == ~0ull ? 64u : uint32_t(__builtin_ctzll(~m));
    cnt += run;
    if (run < 64u) break;
  }
  return cnt;
}

__device__ __forceinline__ void sn_copy(uintptr_t d, uintptr_t s, uint32_t len, int lane) {
  for (uint32_t base = 0; base < len; base += 256u) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + uint32_t(lane) + 64u * j;
      v[j] = ldb(s + (i < len ? i : len - 1u));  // (clamped, not predicated)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + uint32_t(lane) + 64u * j;
      if (i < len) stb(d + i, v[j]);
    }
  }
}

// emit_literal (snappy.c:652-695): returns the bytes written
__device__ __forceinline__ uint32_t sn_emit_literal(uintptr_t d, uintptr_t lit, uint32_t len, int lane) {
  const uint32_t n = len - 1u;
  uint32_t hdr;
  if (n < 60u) {
    hdr = 1u;
    if (lane == 0) stb(d, n << 2);
  } else {
    const uint32_t count = n < 0x100u ? 1u : n < 0x10000u ? 2u : n < 0x1000000u ? 3u : 4u;
    hdr = 1u + count;
    if (lane == 0) stb(d, (59u + count) << 2);
    if (uint32_t(lane) < count) stb(d + 1u + uint32_t(lane), (n >> (8u * uint32_t(lane))) & 0xFFu);
  }
  sn_copy(d + hdr, lit, len, lane);
  return hdr + len;
}

// emit_copy (snappy.c:718-741): 64-byte copies while 68 or more remain, a 60-byte copy when
// 65..67 remain, then the rest (emit_copy_less_than64, :697).  Returns the bytes written.
__device__ __forceinline__ uint32_t sn_emit_copy(uintptr_t d, uint32_t offset, uint32_t len, int lane) {
  const uint32_t k64 = len >= 68u ? (len - 4u) / 64u : 0u;
  for (uint32_t j = uint32_t(lane); j < k64; j += 64u) {
    stb(d + 3u * j, 2u + (63u << 2));
    stb(d + 3u * j + 1u, offset & 0xFFu);
    stb(d + 3u * j + 2u, offset >> 8);
  }
  uint32_t o = 3u * k64, rem = len - 64u * k64;
  if (lane == 0) {
    if (rem > 64u) {
      stb(d + o, 2u + (59u << 2));
      stb(d + o + 1u, offset & 0xFFu);
      stb(d + o + 2u, offset >> 8);
    }
  }
  if (rem > 64u) { o += 3u; rem -= 60u; }
  const bool small = rem < 12u && offset < 2048u;
  if (lane == 0) {
    if (small) {
      stb(d + o, 1u + ((rem - 4u) << 2) + ((offset >> 8) << 5));
      stb(d + o + 1u, offset & 0xFFu);
    } else {
      stb(d + o, 2u + ((rem - 1u) << 2));
      stb(d + o + 1u, offset & 0xFFu);
      stb(d + o + 2u, offset >> 8);
    }
  }
  return o + (small ? 2u : 3u);
}

// compress_fragment (snappy.c:957-1103).  table[0, tsize) is zero.  Returns the size.
__device__ uint32_t sn_compress_fragment(uintptr_t src, uint32_t n, uintptr_t dst, sn_lds_u16 *table,
                                         uint32_t tsize, int lane) {
  const uint32_t shift = 32u - uint32_t(31 - __builtin_clz(tsize));
  uint32_t ip = 0, next_emit = 0, op = 0;
  if (n >= 15u) {
    const uint32_t ip_limit = n - 15u;
    ip = 1;
    bool running = true;
    while (running) {
      // ---- step 1: scan forward for a 4-byte match (:1011-1031)
      uint32_t cand = 0;
      {
        uint32_t fwd = ip, cbase = 0;
        for (;;) {
          const uint32_t c = cbase + uint32_t(lane);
          const uint32_t s = (32u + c) >> 5;
          const uint32_t incl = sn_incl_scan(s, lane);
          const uint32_t P = fwd + incl - s, Pn = fwd + incl;
          const bool valid = Pn <= ip_limit;  // next_ip > ip_limit ends the fragment (:1021)
          const uint64_t vmask = ballot(valid);
          const uint32_t seq = valid ? ld32u(src + P) : 0u;
          const uint32_t h = (seq * kSnMul) >> shift;
          uint64_t eq = same_value_lanes<14>(h, vmask);
          const uint64_t lower = eq & ((1ull << lane) - 1ull);
          const int pred = lower ? 63 - __builtin_clzll(lower) : 0;
          const uint32_t predP = uint32_t(__shfl(int(P), pred));
          const uint32_t cd = lower ? predP : uint32_t(table[h]);
          const bool m = valid && ld32u(src + cd) == seq;
          const uint64_t mm = ballot(m);
          const int f = mm ? __builtin_ctzll(mm) : 64;
          const int e = ~vmask ? __builtin_ctzll(~vmask) : 64;
          if (f < e) {
            const uint64_t upto = (2ull << f) - 1ull;
            const uint64_t later = eq & ~((2ull << lane) - 1ull) & upto;
            if (lane <= f && !later) table[h] = uint16_t(P);
            ip = uint32_t(__builtin_amdgcn_readlane(int(P), f));
            cand = uint32_t(__builtin_amdgcn_readlane(int(cd), f));
            break;
          }
          if (e < 64) { running = false; break; }
          {
            const uint64_t later = eq & ~((2ull << lane) - 1ull);
            if (!later) table[h] = uint16_t(P);
          }
          fwd = uint32_t(__builtin_amdgcn_readlane(int(Pn), 63));
          cbase += 64u;
        }
      }
      if (!running) break;
      asm volatile("" ::: "memory");
      // ---- step 2: the bytes before the match are a literal (:1039)
      op += sn_emit_literal(dst + op, src + next_emit, ip - next_emit, lane);
      // ---- step 3: copies while the position behind the last copy matches (:1054-1088)
      for (;;) {
        const uint32_t matched = 4u + sn_count(src + cand + 4u, src + ip + 4u, n - (ip + 4u), lane);
        op += sn_emit_copy(dst + op, ip - cand, matched, lane);
        ip += matched;
        next_emit = ip;
        if (ip >= ip_limit) { running = false; break; }
        const uint32_t h1 = (ld32u(src + ip - 1u) * kSnMul) >> shift;
        if (lane == 0) table[h1] = uint16_t(ip - 1u);
        asm volatile("" ::: "memory");
        const uint32_t seq = ld32u(src + ip);
        const uint32_t h = (seq * kSnMul) >> shift;
        const uint32_t mi = uni(uint32_t(table[h]));
        asm volatile("" ::: "memory");
        if (lane == 0) table[h] = uint16_t(ip);
        asm volatile("" ::: "memory");
        if (ld32u(src + mi) == seq) { cand = mi; continue; }
        ip++;
        break;
      }
    }
  }
  if (next_emit < n) op += sn_emit_literal(dst + op, src + next_emit, n - next_emit, lane);  // :1097
  return op;
}

// ===================================================================== windows
// compress_fragment in WINDOWS of 64 consecutive positions, one per lane (the scheme of the
// exact LZ4 engine, lz4_encode.hip).  Every lane loads its own 36 source bytes and its table
// candidate's 36 bytes once (from the LDS source ring, or from memory for candidates further
// back than the ring), verifies the 4-byte match and measures it (28 bytes from registers,
// up to 92 from the ring).  The sequential loop's path over those per-lane results -- which
// positions are probed and inserted, the first verifying probe, the ip-1 insertion and the
// immediate re-test behind a copy (:1071-1088) -- is the orbit of the entry lane under
// next(m) = first verified lane >= m + len(m), hopped on the scalar unit (the parallel
// walk).  The skip schedule leaves stride 1 after probe 31 of a search (skip++ >> 5 from
// 32, :1019): the walk is cut at the first lane a search would reach with a higher probe
// index, and sn_generic_search() continues from there probe by probe, 64 probes per step.
// Windows outside the conditions under which the shortcut is exact (a candidate that a lane
// of the same window inserted, a length that is not final, the end of the fragment) are
// replayed one copy at a time by the scalar walk.  tests/sim/snappy_window_sim.cpp is the
// same walk with the lanes as arrays.
constexpr int kSnStride1 = 31;     // highest probe index of a search the windows handle
constexpr int kSnRegLen = 28;      // match bytes a lane measures from its two register windows
constexpr int kSnMaxLen = 92;      // ... and with up to 64 more bytes from the source ring
constexpr uint32_t kSnShortLit = 16;  // literal runs copied by their own lane

enum SnMode { SN_SEARCH = 0, SN_POSTMATCH = 1, SN_FORCED = 2 };
enum SnStatus { SN_CONTINUE = 0, SN_LAST = 1 };

struct SnFrag : SrcRing {  // + the fragment's source and its LDS ring (win_ring.h)
  uintptr_t dst;
  rsrc_t w;       // the fragment's output slot (byte stores; parked lanes write nothing)
  int n, ip_limit;
  uint32_t shift;  // 32 - log2(table size)
  int ip;          // next probe (SN_SEARCH) / end of the last copy (SN_POSTMATCH)
  int cnt;         // probes already made in the current search
  int anchor, op;  // next_emit, bytes written
  int mode;        // how the next window starts
  uint32_t q0, q1;  // the element queue, one copy per lane (sn_flush_elements)
  int qn;           // copies queued
};

// The search loop of :1015-1031 from probe index `cbase` at position `fwd`, 64 probes per
// step.  true: a probe verified, P / cand are set and the table holds every probe up to P;
// false: next_ip passed ip_limit (the remainder follows).
__device__ __forceinline__ bool sn_generic_search(const SnFrag &b, uint32_t fwd, uint32_t cbase,
                                                  sn_lds_u16 *table, int lane, int &P_out,
                                                  int &cand_out) {
  for (;;) {
    const uint32_t c = cbase + uint32_t(lane);
    const uint32_t s = (32u + c) >> 5;
    const uint32_t incl = sn_incl_scan(s, lane);
    const uint32_t P = fwd + incl - s, Pn = fwd + incl;
    const bool valid = int(Pn) <= b.ip_limit;
    const uint64_t vmask = ballot(valid);
    // (a valid probe and every table entry have 15 fragment bytes behind them: the
    // branch-free 8-byte reads stay inside; a load under a lane predicate would be waited
    // for at once)
    const uint32_t sv = ld32u_nb(b.src + (valid ? P : 0u));
    const uint32_t seq = valid ? sv : 0u;
    const uint32_t h = (seq * kSnMul) >> b.shift;
    uint64_t eq = same_value_lanes<14>(h, vmask);
    const uint64_t lower = eq & ((1ull << lane) - 1ull);
    const int pred = lower ? 63 - __builtin_clzll(lower) : 0;
    const uint32_t predP = uint32_t(__shfl(int(P), pred));
    const uint32_t cd = lower ? predP : uint32_t(table[h]);
    const uint32_t cv = ld32u_nb(b.src + (valid ? cd : 0u));
    const bool m = valid && cv == seq;
    const uint64_t mm = ballot(m);
    const int f = ffs64(mm);
    const int e = ffs64(~vmask);
    if (f < e) {
      const uint64_t upto = (2ull << f) - 1ull;
      const uint64_t later = eq & ~((2ull << lane) - 1ull) & upto;
      if (lane <= f && !later) table[h] = uint16_t(P);
      P_out = __builtin_amdgcn_readlane(int(P), f);
      cand_out = __builtin_amdgcn_readlane(int(cd), f);
      return true;
    }
    if (e < 64) return false;
    {
      const uint64_t later = eq & ~((2ull << lane) - 1ull);
      if (!later) table[h] = uint16_t(P);
    }
    fwd = uint32_t(__builtin_amdgcn_readlane(int(Pn), 63));
    cbase += 64u;
  }
}

// bytes emit_copy (:718) writes for a copy of `len` bytes at `off`
__device__ __forceinline__ uint32_t sn_copy_size(uint32_t len, uint32_t off) {
  const uint32_t k64 = len >= 68u ? (len - 4u) >> 6 : 0u;
  uint32_t rem = len - (k64 << 6), o = 3u * k64;
  if (rem > 64u) { o += 3u; rem -= 60u; }
  return o + ((rem < 12u && off < 2048u) ? 2u : 3u);
}

// Write out the queued copies (lane q < qn holds one: literal start | literal length << 16,
// offset | copy length << 16; a copy of a fragment is shorter than 65536 bytes): the literal
// element in front of the copy (tag, length bytes, literal bytes) and the copy element(s) at
// wave-prefix-sum positions.
__device__ __forceinline__ void sn_flush_elements(SnFrag &b, int lane) {
  const bool ch = lane < b.qn;
  const uint32_t lstart = b.q0 & 0xFFFFu, lit = ch ? b.q0 >> 16 : 0u;
  const uint32_t off = b.q1 & 0xFFFFu, ml = b.q1 >> 16;
  const uint32_t ln = lit - 1u;
  const uint32_t lhdr = lit == 0u ? 0u : ln < 60u ? 1u : ln < 256u ? 2u : 3u;  // emit_literal (:652)
  const uint32_t sz = ch ? lhdr + lit + sn_copy_size(ml, off) : 0u;
  uint32_t tot;
  const uint32_t tp = uint32_t(b.op) + wave_excl_scan(sz, tot);  // the literal tag
  const uint32_t lp = tp + lhdr;                                   // first literal byte
  const uint32_t cp = lp + lit;                                    // the copy element
  const bool haslit = ch && lit != 0u;
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(ln < 60u ? ln << 2 : (58u + lhdr) << 2), b.w,
                                       haslit ? tp : kNoLoad, 0, 0);
  if (ballot(haslit && lhdr > 1u)) {  // literals of more than 60 bytes: length bytes
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(ln), b.w, (haslit && lhdr > 1u) ? tp + 1u : kNoLoad, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(ln >> 8), b.w, (haslit && lhdr > 2u) ? tp + 2u : kNoLoad, 0, 0);
  }
  // the copy element (emit_copy_less_than64, :697); copies of more than 64 bytes below
  const bool one = ch && ml <= 64u;
  const bool c2 = ml < 12u && off < 2048u;
  __builtin_amdgcn_raw_buffer_store_b8(
      uint8_t(c2 ? 1u + ((ml - 4u) << 2) + ((off >> 8) << 5) : 2u + ((ml - 1u) << 2)), b.w,
      one ? cp : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off), b.w, one ? cp + 1u : kNoLoad, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(off >> 8), b.w, (one && !c2) ? cp + 2u : kNoLoad, 0, 0);
  uint64_t bigm = ballot(ch && ml > 64u);  // rare: the whole wave writes the elements (:718)
  while (bigm) {
    const int j = __builtin_ctzll(bigm);
    bigm &= bigm - 1;
    sn_emit_copy(b.dst + __builtin_amdgcn_readlane(cp, j), __builtin_amdgcn_readlane(off, j),
                 __builtin_amdgcn_readlane(ml, j), lane);
  }
  // up to 16 literals: one 20-byte window per lane, from the ring while it still holds them
  const uint32_t la = (lstart + b.sa) & ~3u;
  const bool need_win = haslit && lit <= kSnShortLit && int(la) >= b.H - int(kRingBytes);
  if (ballot(need_win)) {
    uint32_t wv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      wv[k] = *(ring_lds_u32 *)((ring_lds_u8 *)b.ring + ((la + 4u * uint32_t(k)) & (kRingBytes - 1u)));
    const uint32_t sh = (lstart + b.sa) & 3u;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], sh);
#pragma unroll
    for (uint32_t k = 0; k < kSnShortLit; ++k)
      __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v[k >> 2] >> (8u * (k & 3u))), b.w,
                                           (need_win && k < lit) ? lp + k : kNoLoad, 0, 0);
  }
  uint64_t longm = ballot(haslit && !need_win);  // long runs: the whole wave copies them
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
}

__device__ __forceinline__ int sn_window_step(SnFrag &b, int w0, int forced_cand, sn_lds_u16 *table,
                                              int lane) {
  const int mode = b.mode;
  // ---------------------------------------------------------------- per lane
  const int i = w0 + lane;
  const bool act = i < b.ip_limit;  // a probe here has next_ip <= ip_limit; a re-test has ip < ip_limit
  while (b.H < w0 + int(b.sa) + 64 + kSnMaxLen + 8) ring_fill(b, lane);
  uint32_t xd[9], yt[9];
  // (the window's 64 lanes read consecutive positions: all straight unless the window
  // straddles the end of the ring)
  const uint32_t wb = (uint32_t(w0) + b.sa) & (kRingBytes - 1u);
  if (wb >= 4u && wb + 64u + 32u <= kRingBytes)
    ring_load9_straight(b, (uint32_t(i) + b.sa) & ~3u, xd);
  else
    ring_load9(b, (uint32_t(i) + b.sa) & ~3u, xd);
  const uint32_t shi = (uint32_t(i) + b.sa) & 3u;
  const uint32_t seq = __builtin_amdgcn_alignbyte(xd[2], xd[1], shi);
  const uint32_t h = (seq * kSnMul) >> b.shift;
  int tc = act ? int(table[h]) : 0;
  if (mode == SN_FORCED && lane == 0) tc = forced_cand;
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
  uint64_t eq = same_value_lanes<14>(h, ACT);
  if (!act) eq = 0;
  const uint64_t DUP = ballot((eq & ((1ull << lane) - 1ull)) != 0);
#pragma unroll
  for (int k = 0; k < 9; ++k) yt[k] = far ? g[k] : yt[k];
  const uint32_t shc = (uint32_t(tc) + b.sa) & 3u;
  const bool tver = act && seq == __builtin_amdgcn_alignbyte(yt[2], yt[1], shc);
  const uint64_t VT = ballot(tver);
  // first differing bit behind the 4 hashed bytes: trailing-zero counts over dword pairs
  // (64 exactly when a pair is equal: only then the next pair counts)
  uint32_t cz[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint32_t z0 = __builtin_amdgcn_alignbyte(xd[2 * k + 3], xd[2 * k + 2], shi) ^
                        __builtin_amdgcn_alignbyte(yt[2 * k + 3], yt[2 * k + 2], shc);
    const uint32_t z1 = __builtin_amdgcn_alignbyte(xd[2 * k + 4], xd[2 * k + 3], shi) ^
                        __builtin_amdgcn_alignbyte(yt[2 * k + 4], yt[2 * k + 3], shc);
    const uint64_t w = (uint64_t(z1) << 32) | z0;
    cz[k] = w ? uint32_t(__builtin_ctzll(w)) : 64u;
  }
  uint32_t fd = cz[1] + (cz[1] >> 6) * cz[2];
  fd = (cz[0] + (cz[0] >> 6) * fd) >> 3;
  int len = 4 + int(fd < uint32_t(kSnRegLen - 4) ? fd : uint32_t(kSnRegLen - 4));
  // a match that fills the register window is measured on from the ring, 4 bytes a step, up
  // to kSnMaxLen; `sat` = the length is still not final and has to be finished from memory if
  // the parse takes this match
  bool more = tver && len == kSnRegLen && !far;
  if (ballot(more)) {
    const uint32_t vi = uint32_t(i) + b.sa, vc = uint32_t(tc) + b.sa;
#pragma unroll 1
    for (int j = 0; j < (kSnMaxLen - kSnRegLen) / 4; ++j) {
      if (!ballot(more)) break;
      const uint32_t pi = vi + uint32_t(len), pc = vc + uint32_t(len);
      ring_lds_u8 *rb = (ring_lds_u8 *)b.ring;
      const uint32_t a0 = *(ring_lds_u32 *)(rb + (pi & (kRingBytes - 4u)));
      const uint32_t a1 = *(ring_lds_u32 *)(rb + ((pi + 4u) & (kRingBytes - 4u)));
      const uint32_t c0 = *(ring_lds_u32 *)(rb + (pc & (kRingBytes - 4u)));
      const uint32_t c1 = *(ring_lds_u32 *)(rb + ((pc + 4u) & (kRingBytes - 4u)));
      const uint32_t z = __builtin_amdgcn_alignbyte(a1, a0, pi & 3u) ^
                         __builtin_amdgcn_alignbyte(c1, c0, pc & 3u);
      if (more) {
        len += z ? int(__builtin_ctz(z) >> 3) : 4;
        if (z) more = false;
      }
    }
  }
  if (len > b.n - i) len = b.n - i;  // find_match_length stops at the end of the input (:823)
  const bool sat = tver && i + len < b.n && (len == kSnMaxLen || (far && len == kSnRegLen));
  const int NA = ~ACT ? __builtin_ctzll(~ACT) : 64;  // first lane that may not be probed

  // one readlane per copy fetches the lane's candidate, match length and `sat`
  const uint32_t pk = uint32_t(tc) | (uint32_t(len) << 16) | (sat ? 1u << 27 : 0u);
  const uint64_t VD = VT | DUP;  // lanes >= NA have neither bit

  const int anchor_in = b.anchor;
  uint64_t INS = 0, chosen = 0;
  int L_cand = 0, L_len = 0;  // per lane: the copy that starts here
  int anchor = b.anchor, cnt = b.cnt;
  int q = 0, x = 0, cand = 0, ipn = 0;
  bool inwin = false, ver = false;
  int st = SN_CONTINUE;
  b.mode = SN_SEARCH;

  // ------------------------------------------------------------ parallel walk
  bool fast_done = false;
  int seq_prev = 0;  // per lane: where the literal of a copy that starts here begins
  if (NA == 64) {
    const int e = mode == SN_POSTMATCH ? 1 : 0;
    const int tl = lane + len;
    const uint64_t fm = tl >= 64 ? 0ull : VT & (~0ull << tl);
    const int J0 = fm ? __builtin_ctzll(fm) : 64;
    // the orbit of the entry lane under J0, hop by hop on the scalar unit (one v_readlane
    // and a handful of scalar instructions per copy)
    const uint64_t em = VT & ~bits_below(e);
    uint64_t ch = 0;
    for (int pos = em ? __builtin_ctzll(em) : 64; pos < 64; pos = __builtin_amdgcn_readlane(J0, pos))
      ch |= 1ull << pos;
    // per lane: the end of the previous chosen copy (0: none).  Chosen copies do not
    // overlap, so their ends grow with the lane: a running maximum, shifted by one lane
    // (the tests below are one vector compare each; their lane masks are combined on the
    // scalar unit.  A copy never ends at position 0, and pend == i + 1 puts the re-test
    // inside the window exactly for lanes below 63.)
    const int mend = i + len;
    const int pend = wave_excl_max(__builtin_amdgcn_inverse_ballot_w64(ch) ? mend : 0);
    const uint64_t Mv = ballot(pend <= i) & (~0ull << e);  // not inside a chosen copy
    uint64_t Tm = ballot(pend == i) & ~uint64_t(w0 == 0);
    uint64_t Rm = ballot(pend == i + 1) & bits_below(63);
    if (mode == SN_POSTMATCH) {
      Tm |= 2ull;
      Rm |= 1ull;
    }
    // probe index of every searched lane: its distance from the last re-tested lane
    const uint64_t lt = Tm & ((1ull << lane) - 1ull);
    const int idx = lt ? lane - 1 - (63 - __builtin_clzll(lt)) : b.cnt + lane;
    const uint64_t over =
        ballot(idx > kSnStride1) & Mv & ~Tm & ~uint64_t(mode == SN_FORCED);  // (FORCED: lane 0)
    const int Z = over ? __builtin_ctzll(over) : 64;
    ch &= bits_below(Z);
    const uint64_t ins = (Mv | Rm) & bits_below(Z);
    const uint64_t Bsat = ballot(sat), Bend = ballot(mend >= b.ip_limit);
    const uint64_t Bdup = ballot((eq & ins & ((1ull << lane) - 1ull)) != 0);
    const uint64_t badm = bits_below(Z) & ((ch & (Bsat | Bend)) | (Mv & Bdup));
    if (!badm) {
      fast_done = true;
      seq_prev = pend > anchor_in ? pend : anchor_in;  // (a chosen end lies behind the anchor)
      INS = ins;
      chosen = ch;
      L_cand = tc;
      L_len = len;
      int end = -1;
      if (ch) {
        const int cl = 63 - __builtin_clzll(ch);
        end = cl + __builtin_amdgcn_readlane(len, cl);  // lane after the last copy
        anchor = w0 + end;
      }
      if (Z < 64) {
        b.ip = w0 + Z;
        b.cnt = kSnStride1 + 1;
      } else if (end >= 64) {
        b.ip = w0 + end;
        b.mode = SN_POSTMATCH;
      } else {
        b.ip = w0 + 64;
        b.cnt = Tm ? 63 - (63 - __builtin_clzll(Tm)) : b.cnt + 64;
      }
    }
  }

  // ------------------------------------------------------------- scalar walk
  // One loop iteration per copy: the pending match (:1054-1062), then the ip-1 insertion and
  // the re-test of ip (:1071-1088), then the search for the next match (:1015-1031).
#define RDK_SN_LOOKUP(lx)                                                                   \
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
  if (!fast_done) {
    bool have = false;  // a verified match at lane x is pending
    bool post = false;  // a copy just ended at ipn
    if (mode == SN_POSTMATCH) {
      ipn = w0 + 1;
      post = true;
    } else if (mode == SN_FORCED) {
      x = 0;  // lane 0's candidate was set to forced_cand above
      have = true;
    }
    for (;;) {
      if (have) {
        have = false;
        const int P = w0 + x;
        const uint32_t pkx = uint32_t(__builtin_amdgcn_readlane(int(pk), x));
        if (!inwin) cand = int(pkx & 0xFFFFu);
        int fl;
        if (inwin) {
          fl = win_count_fwd(b, P + 4, cand + 4, b.n - (P + 4), lane);
        } else {
          const int lx = int((pkx >> 16) & 0xFFu);
          fl = lx - 4;
          if (pkx & (1u << 27))  // length not final: finish it from the ring / memory
            fl += win_count_fwd(b, P + lx, cand + lx, b.n - P - lx, lane);
        }
        if (lane == x) {
          L_cand = cand;
          L_len = 4 + fl;
        }
        chosen |= 1ull << x;
        ipn = P + 4 + fl;
        anchor = ipn;
        if (ipn >= b.ip_limit) {  // :1062
          st = SN_LAST;
          break;
        }
        post = true;
      }
      if (post) {
        post = false;
        const int r = ipn - 1 - w0;
        if (r >= 63) {  // the re-test position lies beyond this window
          b.ip = ipn;
          b.mode = SN_POSTMATCH;
          break;
        }
        x = r + 1;
        INS |= 3ull << r;  // table[hash(ip-1)] = ip-1 (:1071) and the re-tested ip itself
        if ((DUP >> x) & 1ull) {
          RDK_SN_LOOKUP(x);
        } else {
          inwin = false;
          ver = (VT >> x) & 1ull;
        }
        if (ver) {  // immediate copy: no literal
          have = true;
          continue;
        }
        q = x + 1;
        cnt = 0;
      }
      // search from lane q, whose probe index is cnt; lanes from xlim on have a probe index
      // above kSnStride1
      const int xlim = q + (kSnStride1 + 1) - cnt;
      uint64_t cm = q < 64 ? VD & (~0ull << q) : 0ull;
      if (xlim < 64) cm &= bits_below(xlim);
      if (!cm) {  // no candidate left in this window
        int stop = NA;  // <= 64
        int why = NA < 64 ? 1 : 0;  // 1: remainder, 0: window end
        if (xlim <= stop) {         // 2: strides above 1 from here on
          stop = xlim;
          why = 2;
        }
        INS |= bits_range(q, stop);
        if (why == 1) {
          st = SN_LAST;
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
        RDK_SN_LOOKUP(x);
        have = ver;
      } else {  // x has no earlier lane with its hash: its table candidate verified (VT)
        inwin = false;
        have = true;
      }
    }
  }
#undef RDK_SN_LOOKUP

  // ------------------------------------------------------------ table update
  // every inserted lane; the latest position per hash wins
  if (st != SN_LAST) {
    const bool ins = __builtin_amdgcn_inverse_ballot_w64(INS);
    const uint64_t later = eq & INS & ~bits_below(lane + 1);
    if (ins && !later) table[h] = uint16_t(i);
    asm volatile("" ::: "memory");
  }
  // ----------------------------------------------------------------- elements
  // A window holds a handful of copies, far fewer than lanes: they are queued, one per lane
  // of the queue registers, and written out 64 at a time (sn_flush_elements).
  {
    const bool ch = __builtin_amdgcn_inverse_ballot_w64(chosen);
    int prev = seq_prev;  // where this copy's literal starts (the parallel walk has it already)
    if (!fast_done) {
      const uint64_t lowc = chosen & ((1ull << lane) - 1ull);
      const int pl = lowc ? 63 - __builtin_clzll(lowc) : lane;
      const int pend = __shfl(i + L_len, pl);  // end of the previous chosen copy
      prev = lowc ? pend : anchor_in;
    }
    const uint32_t lit = uint32_t(i - prev);
    const uint32_t off = uint32_t(i - L_cand), ml = uint32_t(L_len);
    const int cnt = __builtin_popcountll(chosen);
    if (cnt) {
      if (b.qn + cnt > 64) sn_flush_elements(b, lane);
      // chosen lane -> queue lane qn + its rank among the chosen lanes: a forward permute
      // (scatter); the other lanes send to a lane outside the accepted range
      const int rank = int(__builtin_amdgcn_mbcnt_hi(uint32_t(chosen >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(uint32_t(chosen), 0u)));
      const int tgt = ch ? b.qn + rank : ((b.qn + cnt) & 63);
      const uint32_t r0 = uint32_t(__builtin_amdgcn_ds_permute(tgt << 2, int(uint32_t(prev) | (lit << 16))));
      const uint32_t r1 = uint32_t(__builtin_amdgcn_ds_permute(tgt << 2, int(off | (ml << 16))));
      const bool acc = lane >= b.qn && lane < b.qn + cnt;
      b.q0 = acc ? r0 : b.q0;
      b.q1 = acc ? r1 : b.q1;
      b.qn += cnt;
    }
  }
  b.anchor = anchor;
  return st;
}

// compress_fragment (snappy.c:957-1103) in windows; table[0, tsize) is zero.  `cap` = bytes
// of the output slot.  Returns the size.
__device__ uint32_t sn_window_fragment(uintptr_t src, uint32_t n, uintptr_t dst, uint32_t cap,
                                       sn_lds_u16 *table, ring_lds_u32 *ring, uint32_t tsize, int lane) {
  SnFrag b;
  ring_init(b, src, n, ring, lane);
  b.dst = dst;
  b.w = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(dst), 0, int(cap), 0x00020000);
  b.n = int(n);
  b.ip_limit = int(n) - 15;  // kinput_margin_bytes (:965)
  b.shift = 32u - uint32_t(31 - __builtin_clz(tsize));
  b.ip = 1;
  b.cnt = 0;
  b.anchor = 0;
  b.op = 0;
  b.mode = SN_SEARCH;
  b.q0 = b.q1 = 0;
  b.qn = 0;
  if (n >= 15u) {
    int forced = 0;
    for (;;) {
      int w0;
      if (b.mode == SN_SEARCH && b.cnt > kSnStride1) {  // strides above 1: probe by probe
        int P, cand;
        if (!sn_generic_search(b, uint32_t(b.ip), uint32_t(b.cnt), table, lane, P, cand)) break;
        asm volatile("" ::: "memory");
        b.mode = SN_FORCED;
        forced = cand;
        w0 = P;
      } else {
        w0 = b.mode == SN_POSTMATCH ? b.ip - 1 : b.ip;
      }
      if (sn_window_step(b, w0, forced, table, lane) == SN_LAST) break;
    }
    sn_flush_elements(b, lane);
  }
  uint32_t op = uint32_t(b.op);
  if (uint32_t(b.anchor) < n)  // emit_remainder (:1097)
    op += sn_emit_literal(dst + op, src + uint32_t(b.anchor), n - uint32_t(b.anchor), lane);
  return op;
}

// One wavefront per fragment; items are slot-major so that every shader engine is busy.
template <bool WINDOWS>
__global__ __launch_bounds__(64) void snappy_compress_fragments_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t n) {
  // the source ring (windowed engine) sits in front of the hash table
  constexpr uint32_t kRingLds = WINDOWS ? kRingBytes : 0u;
  __shared__ __attribute__((aligned(16))) uint8_t lds_mem[kRingLds + 2u * kSnMaxTable];
  sn_lds_u16 *table = (sn_lds_u16 *)reinterpret_cast<uint16_t *>(lds_mem + kRingLds);
  const int lane = threadIdx.x;
  const uint32_t items = n * uint32_t(kSnItems);
  for (uint32_t it = blockIdx.x; it < items; it += gridDim.x) {
    const uint32_t f = it % n, kk = it / n;
    const uint32_t len = uni(in_lens[f]);
    const uint32_t nb = (len + kSnBlock - 1u) / kSnBlock;
    for (uint32_t k = kk; k < nb; k += uint32_t(kSnItems)) {
      const uint32_t fn = len - k * kSnBlock < kSnBlock ? len - k * kSnBlock : kSnBlock;
      uint32_t tsize = 256;  // get_hash_table, snappy.c:790-807
      while (tsize < kSnMaxTable && tsize < fn) tsize <<= 1;
      for (uint32_t i = uint32_t(lane); i < tsize / 2u; i += 64u) ((ring_lds_u32 *)table)[i] = 0;
      asm volatile("" ::: "memory");
      const uintptr_t src = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kSnBlock;
      const uintptr_t slot =
          reinterpret_cast<uintptr_t>(out) + out_offs[f] + kSnSlot0 + uint64_t(k) * kSnSlot;
      // (the output resource ends inside rd_kafka_snappy_max_compressed_length of the stream)
      const uint32_t sz = WINDOWS ? sn_window_fragment(src, fn, slot + 4u, fn + fn / 6u + 16u, table,
                                                       (ring_lds_u32 *)lds_mem, tsize, lane)
                                  : sn_compress_fragment(src, fn, slot + 4u, table, tsize, lane);
      if (lane == 0) {
        stb(slot, sz & 0xFFu); stb(slot + 1, (sz >> 8) & 0xFFu);
        stb(slot + 2, (sz >> 16) & 0xFFu); stb(slot + 3, sz >> 24);
      }
    }
  }
}

// One workgroup per stream: the varint32 of the input length (varint_encode32, snappy.c:297),
// then the fragments slid together (destination always below source).
constexpr uint32_t kSnAsmThreads = 1024;  // 16 KiB per read-then-write step of the slide

__global__ __launch_bounds__(kSnAsmThreads) void snappy_assemble_kernel(
    const uint32_t *__restrict__ in_lens, uint8_t *out, const uint64_t *__restrict__ out_offs,
    uint32_t *__restrict__ out_lens, uint32_t n) {
  const int t = threadIdx.x;
  for (uint32_t f = blockIdx.x; f < n; f += gridDim.x) {
    const uint32_t len = in_lens[f];
    const uint32_t nb = (len + kSnBlock - 1u) / kSnBlock;
    const uintptr_t ob = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    uint32_t vl = 1;
    for (uint32_t v = len; v >= 128u; v >>= 7) vl++;
    uint64_t pos = vl;
    for (uint32_t k = 0; k < nb; ++k) {
      const uintptr_t slot = ob + kSnSlot0 + uint64_t(k) * kSnSlot;
      const uint32_t sz = ldb(slot) | (ldb(slot + 1) << 8) | (ldb(slot + 2) << 16) | (ldb(slot + 3) << 24);
      __syncthreads();  // everyone has read the size word before it may be overwritten
      const uintptr_t from = slot + 4u, to = ob + pos;
      for (uint32_t base = 0; base < sz; base += kSnAsmThreads * 16u) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t i = base + uint32_t(t) + kSnAsmThreads * j;
          v[j] = ldb(from + (i < sz ? i : sz - 1u));  // (clamped, not predicated)
        }
        __syncthreads();  // chunk fully read before any lane writes (dst < src)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t i = base + uint32_t(t) + kSnAsmThreads * j;
          if (i < sz) stb(to + i, v[j]);
        }
        __syncthreads();
      }
      pos += sz;
    }
    if (t == 0) {
      uint32_t v = len, i = 0;
      for (; v >= 128u; v >>= 7) stb(ob + i++, (v & 127u) | 128u);
      stb(ob + i, v);
      out_lens[f] = uint32_t(pos);
    }
    __syncthreads();
  }
}

// ===================================================================== decompress
constexpr uint32_t kSnRing = 4096;            // LDS history per wavefront
constexpr uint32_t kSnRingMask = kSnRing - 1u;
constexpr int kSnDecWaves = 4;                // wavefronts per workgroup
constexpr uint32_t kSnLitTag = 0x80000000u;
constexpr uint32_t kSnNoAccess = 0x80000000u; // out-of-range buffer offset (reads 0, stores nothing)
constexpr uint32_t kSnComplex = 0xFFFFFFFFu;  // header needs a fifth byte
constexpr uint32_t kSnBad = 0xFFFFFFFEu;      // no element can start here

__device__ __forceinline__ sn_rsrc_t sn_make_rsrc(uintptr_t base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), 0, int(bytes), 0x00020000);
}
__device__ __forceinline__ uint64_t sn_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint32_t sn_incl_max(uint32_t v) {
  int x = int(v);
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true));
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true));
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true));
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true));
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));
  return uint32_t(x);
}
__device__ __forceinline__ uint32_t sn_excl_sum(uint32_t v, uint32_t &total) {
  int x = int(v);
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  total = uint32_t(__builtin_amdgcn_readlane(x, 63));
  return uint32_t(x) - v;
}

struct SnDec {
  sn_lds_u8 *ring, *map;  // map: [0, 64) per-piece scratch, [64, 128) stores of parked lanes
  // rin spans the whole dwords that hold the stream (a range-checked dword that is only
  // partly inside a buffer reads as zero, and a stream may end in a 2-byte element):
  // offsets into it are stream positions + din
  sn_rsrc_t rin;
  g_u8 *out;  // output; every position written or read lies below the checked length
  uint32_t din;
  // the fetched, not yet written piece: the byte as each of the three sources delivered it,
  // and which one holds it (literal, history ring, else far history)
  uint32_t pn, poc, plb, pfb, prb;
  bool plit, prk;
};

// a start position no piece below `end` contains
__device__ __forceinline__ uint32_t c_none(uint32_t end) { return end + 0x40000000u; }

__device__ __forceinline__ void sn_set_out(SnDec &d, uintptr_t dst) {
  // wave-uniform base: the output is addressed as scalar base + lane offset
  d.out = (g_u8 *)((uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(uint64_t(dst) >> 32)))) << 32) |
                   uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(dst)))));
}

// Output reaches memory a whole kSnOutChunk at a time, from the history ring, as one 16-byte
// store per lane (aligned when the destination is): memory takes whole sectors well and
// pieces of a few bytes badly.
constexpr uint32_t kSnOutChunk = 1024;
typedef uint32_t sn_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t sn_u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) sn_u32x4 sn_lds_u32x4;
typedef __attribute__((address_space(1))) sn_u32x4_a1 sn_g_u32x4;

// ring -> memory: output [c0, c0 + n), c0 a multiple of kSnOutChunk, n <= kSnOutChunk
__device__ __forceinline__ void sn_write_out(const SnDec &d, uint32_t c0, uint32_t n, int lane) {
  const uint32_t l16 = 16u * uint32_t(lane), o = c0 + l16;
  if (l16 + 16u <= n) {
    *(sn_g_u32x4 *)(d.out + o) = *(sn_lds_u32x4 *)(d.ring + (o & kSnRingMask));
  } else if (l16 < n) {  // the last, partial 16 bytes
    for (uint32_t j = 0; j < n - l16; ++j) d.out[o + j] = d.ring[(o + j) & kSnRingMask];
  }
}

// the output's last, incomplete chunk
__device__ __forceinline__ void sn_write_tail(const SnDec &d, uint32_t op, int lane) {
  sn_write_out(d, op & ~(kSnOutChunk - 1u), op & (kSnOutChunk - 1u), lane);
}

__device__ __forceinline__ void sn_retire(SnDec &d, int lane) {
  __builtin_amdgcn_sched_barrier(0);  // keep the wait for the piece's loads down here
  // (through empty asm statements: a select between fields of `d` would otherwise become one
  // load through a selected address, which puts the fields into scratch memory)
  uint32_t a = d.plb, b = d.prb, c = d.pfb;
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
  const uint32_t v = d.plit ? a : (d.prk ? b : c);
  if (uint32_t(lane) < d.pn) d.ring[(d.poc + uint32_t(lane)) & kSnRingMask] = uint8_t(v);
  asm volatile("" ::: "memory");
  // (a piece is at most 64 bytes: it completes at most one chunk)
  if (((d.poc + d.pn) ^ d.poc) & ~(kSnOutChunk - 1u))
    sn_write_out(d, d.poc & ~(kSnOutChunk - 1u), kSnOutChunk, lane);
  d.pn = 0;
}

// fetch output bytes [pc, pc+nvalid): lane l's byte comes from `src` (tag | input position, or
// an output position below its own; all ones in a lane without a byte)
__device__ __forceinline__ void sn_flush(SnDec &d, uint32_t src, uint32_t pc, uint32_t nvalid, int lane) {
  for (;;) {  // sources inside the piece: pointer jumping (unconditional shuffle, then select)
    const bool intra = int32_t(src) >= int32_t(pc);  // (a tagged source is negative)
    if (!sn_ballot(intra)) break;
    const uint32_t v = uint32_t(__builtin_amdgcn_ds_bpermute(int((src - pc) << 2), int(src)));
    src = intra ? v : src;
  }
  sn_retire(d, lane);  // the ring must hold everything before pc
  const bool lit = int32_t(src) < 0;
  const uint32_t q = src & ~kSnLitTag;
  const bool rk = q + kSnRing >= pc;  // a copy source still in the history ring
  // (a lane without a byte stays out of the input's range: positions are below 2^31 - din)
  d.plb = __builtin_amdgcn_raw_buffer_load_b8(d.rin, lit ? q + d.din : kSnNoAccess, 0, 0);
  // Far history was stored at least (kSnRing - kSnOutChunk) / 64 pieces ago, each of which
  // ended in sn_retire's wait for its loads.  The load relies on gfx950 handling one
  // wavefront's vector-memory operations in program order (a store issued before a load that
  // has been waited for has completed) -- the same reasoning, and the same kind of test
  // (copies around the ring edge), as in lz4_decode_fast.h.
  static_assert(kSnRing >= kSnOutChunk + 2048u, "far history must be at least 32 pieces old");
  d.pfb = d.out[(lit | rk) ? 0u : q];
  asm volatile("" ::: "memory");
  d.prb = d.ring[q & kSnRingMask];
  d.plit = lit;
  d.prk = rk;
  d.pn = nvalid;
  d.poc = pc;
}

// The element that would start at p = seg + lane, from the 4 bytes at p (char_table,
// snappy.c:1129): A = next element start (kSnComplex / kSnBad), ll / ml = literal / copy
// bytes, off = copy offset, k = header bytes.
struct SnCand {
  uint32_t A, ll, off, mk;  // mk = ml | k << 8
};

typedef uint32_t sn_u2 __attribute__((ext_vector_type(2)));

// the aligned 8 bytes that hold the 4 bytes at p = seg + lane
__device__ __forceinline__ sn_u2 sn_parse_load(const SnDec &d, uint32_t seg, int lane) {
  return __builtin_amdgcn_raw_buffer_load_b64(d.rin, (seg + uint32_t(lane) + d.din) & ~3u, 0, 0);
}

__device__ __forceinline__ SnCand sn_parse_words(const SnDec &d, sn_u2 h, uint32_t csize, uint32_t seg,
                                                 int lane) {
  const uint32_t p = seg + uint32_t(lane);
  const uint32_t w = __builtin_amdgcn_alignbyte(h.y, h.x, (p + d.din) & 3u);
  // (flat selects over values already computed: nested ones compile to divergent branches)
  const uint32_t c = w & 0xFFu, kind = c & 3u, hi = c >> 2;
  const uint32_t b1 = (w >> 8) & 0xFFu, b12 = (w >> 8) & 0xFFFFu;
  const bool islit = kind == 0u;
  const uint32_t lx = max(hi, 59u) - 59u;
  const uint32_t lext = islit ? lx : 0u;  // extra length bytes of a literal
  const uint32_t k = ((0x5321u >> (kind << 2)) & 15u) + lext;  // header bytes: 1+lext, 2, 3, 5
  const bool complex = (lext == 4u) | (kind == 3u);
  const uint32_t lvx = __builtin_amdgcn_ubfe(w, 8u, lext << 3);  // the lext bytes after the tag
  const uint32_t lv = lext == 0u ? hi : lvx;
  const uint32_t ll = islit ? lv + 1u : 0u;
  const uint32_t m1 = 4u + (hi & 7u), m2 = hi + 1u;
  const uint32_t mlc = kind == 1u ? m1 : m2;
  const uint32_t ml = islit ? 0u : mlc;
  const uint32_t o1 = ((c >> 5) << 8) | b1;
  const uint32_t off = kind == 1u ? o1 : b12;
  SnCand r;
  const bool bad = (p >= csize) | (p + k > csize);  // refill_tag cannot complete the header
  r.A = bad ? kSnBad : complex ? kSnComplex : p + k + ll;
  r.ll = ll;
  r.off = off;
  r.mk = ml | (k << 8);
  return r;
}

__device__ __forceinline__ SnCand sn_parse(const SnDec &d, uint32_t csize, uint32_t seg, int lane) {
  return sn_parse_words(d, sn_parse_load(d, seg, lane), csize, seg, lane);
}

// wave-uniform byte of the stream (slow path only)
__device__ __forceinline__ uint32_t sn_in_byte(const SnDec &d, uint32_t i) {
  return __builtin_amdgcn_readfirstlane(__builtin_amdgcn_raw_buffer_load_b8(d.rin, i + d.din, 0, 0));
}

#ifdef RDK_SN_DEBUG
#define SN_FAIL(site) (kSnEIO - 100 * (site))
#else
#define SN_FAIL(site) kSnEIO
#endif
// The elements of the stream from input position ipn up to n, which must produce exactly
// `ulen` bytes from output position 0 of d.rout (decompress_all_tags, snappy.c:1226-1312).
// Returns 0 or -EIO.
__device__ int sn_decode_elems(SnDec &d, uint32_t n, uint32_t ipn, uint32_t ulen, sn_lds_u8 *map,
                               int lane) {
  uint32_t op = 0;
  if (ipn == n) return ulen == 0u ? 0 : SN_FAIL(21);
  uint32_t seg = ipn & ~63u;
  SnCand cur = sn_parse(d, n, seg, lane);
  SnCand nxt = sn_parse(d, n, seg + 64u, lane);
  for (;;) {
    // ---- walk: which candidate lanes are the real elements of this segment
    const uint32_t x0 = ipn - seg;
    uint64_t M;
    bool mem;
    for (;;) {
      const bool stop = (cur.A - seg >= 64u) | (cur.A == n);  // bad, complex, leaves, or ends the stream
      // successor lane as a permute address (lane * 4); 256: none.  A level marks every
      // reached lane's successor (lanes that mark nothing mark the entry lane, which is
      // reached anyway) and squares the successor map.
      uint32_t J = stop ? 256u : (cur.A - seg) << 2;
      bool R = uint32_t(lane) == x0;
#pragma unroll
      for (int level = 0; level < 5; ++level) {
        const bool send = R & (J < 256u);
        const int t = __builtin_amdgcn_ds_permute(int(send ? J : x0 << 2), 1);
        R = R | (t != 0);
        const uint32_t jj = uint32_t(__builtin_amdgcn_ds_bpermute(int(J), int(J)));
        J = J < 256u ? jj : 256u;
      }
      mem = R;
      // (ballots straight from one compare each; a member's A is never 0)
      const uint32_t ra = R ? cur.A : 0u;
      M = sn_ballot(ra != 0u);
      const uint64_t cx = sn_ballot(ra >= kSnBad);  // kSnBad or kSnComplex among the members
      if (!cx) break;
      if (sn_ballot(ra == kSnBad)) return SN_FAIL(4);
      // header with a fifth byte: literal of 2^24 bytes or more, or a 4-byte offset
      const uint32_t xc = uint32_t(__builtin_ctzll(cx));
      const uint32_t p = seg + xc;
      const uint32_t c = sn_in_byte(d, p);
      const uint32_t v = sn_in_byte(d, p + 1u) | (sn_in_byte(d, p + 2u) << 8) |
                         (sn_in_byte(d, p + 3u) << 16) | (sn_in_byte(d, p + 4u) << 24);
      const bool me = uint32_t(lane) == xc;
      if ((c & 3u) == 3u) {  // copy with a 4-byte offset
        cur.A = me ? p + 5u : cur.A;
        cur.ll = me ? 0u : cur.ll;
        cur.off = me ? v : cur.off;
        cur.mk = me ? ((c >> 2) + 1u) | (5u << 8) : cur.mk;
      } else {
        const uint64_t nx = uint64_t(p) + 5u + uint64_t(v) + 1u;
        if (nx > n) return SN_FAIL(5);  // premature end of input (:1283)
        cur.A = me ? uint32_t(nx) : cur.A;
        cur.ll = me ? v + 1u : cur.ll;
        cur.off = me ? 0u : cur.off;
        cur.mk = me ? (5u << 8) : cur.mk;
      }
    }
    const uint32_t xl = uint32_t(63 - __builtin_clzll(M));
    const uint32_t a_last = uni(__builtin_amdgcn_readlane(cur.A, xl));
    if (a_last > n) return SN_FAIL(6);  // the last literal runs past the input
    const bool done = a_last == n;
    // ---- the segment's elements, one per member lane, in lane order
    const uint32_t ll = cur.ll, ml = cur.mk & 0xFFu, off = cur.off, k = cur.mk >> 8;
    const uint32_t len = mem ? ll + ml : 0u;
    // (the members' literals are disjoint pieces of an input below 2^31 bytes, so the sum of
    // their lengths cannot wrap)
    uint32_t T;
    const uint32_t ostart = op + sn_excl_sum(len, T);
    if (uint64_t(op) + T > ulen) return SN_FAIL(7);  // writer_append* : no room (:572, :543)
    // writer_append_from_self: offset 0 or beyond the produced bytes (:548)
    if (sn_ballot((mem ? ml : 0u) != 0u) & sn_ballot(ostart <= off - 1u)) return SN_FAIL(8);
    // ---- output [op, op+T) in pieces of 64 bytes, lane per byte
    const uint32_t op_new = uni(op + T);
    const uint32_t ls = seg + uint32_t(lane) + k;  // first literal byte
    // every member has bytes; their fields are packed into the low lanes in stream order (a
    // segment holds at most 32 elements): first byte that is not a literal, literal position
    // minus output position, copy offset
    const uint64_t Mn = sn_ballot(len != 0u);
    const uint32_t slot = len != 0u ? __builtin_amdgcn_mbcnt_hi(uint32_t(Mn >> 32),
                                                                __builtin_amdgcn_mbcnt_lo(uint32_t(Mn), 0u))
                                    : 63u;
    const uint32_t f_cpy = uint32_t(__builtin_amdgcn_ds_permute(int(slot << 2), int(ostart + ll)));
    const uint32_t f_dl = uint32_t(__builtin_amdgcn_ds_permute(int(slot << 2), int(ls - ostart)));
    const uint32_t f_of = uint32_t(__builtin_amdgcn_ds_permute(int(slot << 2), int(off)));
    const uint32_t ost = len != 0u ? ostart : c_none(op_new);
    uint32_t before = 0xFFFFFFFFu;  // elements that start before the piece, less one
    for (uint32_t c = op; c < op_new; c = uni(c + 64u)) {
      // the starts in this piece are scattered into the map; a lane's element is the count of
      // starts up to its byte
      map[lane] = 0;
      asm volatile("" ::: "memory");
      const uint32_t rel0 = ost - c;
      map[rel0 < 64u ? rel0 : 64u + uint32_t(lane)] = 1;
      asm volatile("" ::: "memory");
      const uint64_t sb = sn_ballot(map[lane] != 0);
      const uint64_t s1 = sb >> 1;
      const uint32_t cntb = __builtin_amdgcn_mbcnt_hi(uint32_t(s1 >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(uint32_t(s1), 0u));
      const int idx4 = int((cntb << 2) + uni((before + uint32_t(sb & 1ull)) << 2));
      before = uni(before + uint32_t(__builtin_popcountll(sb)));
      const uint32_t g_cpy = uint32_t(__builtin_amdgcn_ds_bpermute(idx4, int(f_cpy)));
      const uint32_t g_dl = uint32_t(__builtin_amdgcn_ds_bpermute(idx4, int(f_dl)));
      const uint32_t g_of = uint32_t(__builtin_amdgcn_ds_bpermute(idx4, int(f_of)));
      const uint32_t o = c + uint32_t(lane);
      const uint32_t s_lit = (o + g_dl) | kSnLitTag, s_mat = o - g_of;
      const uint32_t s = o < g_cpy ? s_lit : s_mat;
      const uint32_t left = op_new - c;
      const uint32_t nv = left < 64u ? left : 64u;
      sn_flush(d, uint32_t(lane) < nv ? s : 0xFFFFFFFFu, c, nv, lane);
    }
    op = op_new;
    if (done) {
      sn_retire(d, lane);
      sn_write_tail(d, op, lane);
      return op == ulen ? 0 : SN_FAIL(20);  // eof && writer_check_length (:1403)
    }
    ipn = a_last;
    const uint32_t nseg = ipn & ~63u;
    if (nseg == seg + 64u) {
      cur = nxt;
    } else {
      cur = sn_parse(d, n, nseg, lane);
    }
    seg = nseg;
    nxt = sn_parse(d, n, seg + 64u, lane);
  }
}

// Decode the stream at `src` (n bytes) into `dst` (cap bytes).  Returns 0 or -EIO like
// rd_kafka_snappy_uncompress; *ulen_out = the declared length (0 when unreadable).
__device__ int sn_decode_stream(uintptr_t src, uint32_t n, uintptr_t dst, uint32_t cap,
                                uint32_t *ulen_out, sn_lds_u8 *ring, sn_lds_u8 *map, int lane) {
  if (n >= 0x80000000u) return SN_FAIL(1);  // input positions carry a tag in bit 31
  SnDec d;
  d.ring = ring;
  d.map = map;
  d.din = uint32_t(src & 3u);
  d.rin = sn_make_rsrc(src - d.din, (d.din + n + 3u) & ~3u);
  d.pn = d.poc = d.plb = d.pfb = d.prb = 0;
  d.plit = d.prk = false;
  // read_uncompressed_length (snappy.c:1193-1218)
  uint32_t ulen = 0, ip0 = 0;
  for (uint32_t shift = 0;; shift += 7u) {
    if (shift >= 32u || ip0 >= n) return SN_FAIL(2);
    const uint32_t c = sn_in_byte(d, ip0++);
    ulen |= (c & 0x7Fu) << shift;
    if (c < 128u) break;
  }
  *ulen_out = ulen;
  if (ulen > 0x7FFFFFF0u) return SN_FAIL(3);  // positions are kept in 31 bits
  if (ulen > cap) return kSnDstSize;      // the caller sizes dst from the preamble
  sn_set_out(d, dst);
  return sn_decode_elems(d, n, ip0, ulen, map, lane);
}

// ---- decoding a stream by its fragments
// A compressor emits one run of elements per 64 KiB fragment of its input (sn_compress,
// snappy.c:1408-1484), so in the streams it makes no element crosses a multiple of 64 KiB of
// output and no copy reaches in front of its fragment.  A parse-only pass over the stream
// (one wave per stream, nothing written) checks exactly that and notes where in the input
// each fragment starts; the fragments are then decoded independently, which fills the chip
// where one wave per stream leaves it nearly idle.  A stream that is anything else --
// malformed, a single fragment, elements or copies that cross -- is decoded serially as
// before, and that decoder alone decides its verdict.
constexpr uint32_t kSnFragMax = 64;  // fragments per stream the split handles (4 MiB)

struct SnSplit {
  int32_t split;            // 1: decode by fragments; 0: decode the stream serially
  uint32_t ulen, ip0, nfrag;
  uint32_t ip[kSnFragMax];  // input position of fragment k's first element (k >= 1)
};

constexpr uint32_t kSnPoison = 0x04000000u;  // a length no stream that splits can reach
constexpr int kSnScanGroup = 4;              // segments whose lists are collapsed together

// The elements of one 64-byte segment reached from lane x0, with output positions from `op`:
// false when one of them keeps the stream from being split (it crosses a 64 KiB boundary of
// the output, copies from before its fragment, or cannot be parsed); records the input
// position of every element that starts a fragment.
__device__ bool sn_scan_members(const SnCand &cur, uint32_t n, uint32_t seg, uint32_t x0, uint32_t op,
                                SnSplit *t, uint32_t &found, int lane) {
  const bool stop = (cur.A - seg >= 64u) | (cur.A == n);
  uint32_t J = stop ? 256u : (cur.A - seg) << 2;  // successor as a permute address; 256: none
  bool R = uint32_t(lane) == x0;
#pragma unroll
  for (int level = 0; level < 5; ++level) {
    const bool send = R & (J < 256u);
    const int tt = __builtin_amdgcn_ds_permute(int(send ? J : x0 << 2), 1);
    R = R | (tt != 0);
    const uint32_t jj = uint32_t(__builtin_amdgcn_ds_bpermute(int(J), int(J)));
    J = J < 256u ? jj : 256u;
  }
  const bool mem = R;
  const uint32_t ra = R ? cur.A : 0u;                // (a member's A is never 0)
  if (sn_ballot(ra >= kSnBad)) return false;         // kSnBad or kSnComplex
  const uint32_t ml = cur.mk & 0xFFu, off = cur.off;
  const uint32_t len = mem ? cur.ll + ml : 0u;
  uint32_t T;
  const uint32_t ostart = op + sn_excl_sum(len, T);
  const uint32_t in_frag = ostart & (kSnBlock - 1u);
  // (one vector compare per ballot, the lane masks combined on the scalar unit; a lane that
  // is no member has len 0)
  const uint64_t crosses = sn_ballot(in_frag + len > kSnBlock);
  // offset 0, or in front of the fragment
  const uint64_t reaches = sn_ballot((mem ? ml : 0u) != 0u) & sn_ballot(in_frag <= off - 1u);
  if (crosses | reaches) return false;
  const uint64_t Fm = sn_ballot(len != 0u) & sn_ballot(in_frag == 0u) & sn_ballot(ostart != 0u);
  if (__builtin_amdgcn_inverse_ballot_w64(Fm)) t->ip[ostart >> 16] = seg + uint32_t(lane);
  found += uint32_t(__builtin_popcountll(Fm));
  return true;
}

// Whether a stream can be decoded by fragments, and where each fragment's input starts
// (every 64 KiB of output begins at an element boundary and no copy reaches across one:
// what the block-by-block writer, snappy.c:1344, produces).
//
// One wavefront follows the stream's elements from segment to segment. A segment's step
// (entry lane -> output bytes, exit position, largest copy offset on the way) does not
// depend on where the stream enters it, so the elements of a segment are collapsed by
// pointer doubling for every entry lane at once, kSnScanGroup segments side by side (their
// shuffles overlap); the dependent part per segment is then a handful of lane reads. Only a
// segment whose output touches a 64 KiB boundary, or holds an offset larger than the
// distance to the fragment's start, has its elements looked at one by one.
__device__ bool sn_scan_stream(uintptr_t src, uint32_t n, uint32_t cap, SnSplit *t, int lane) {
  if (n >= 0x80000000u) return false;
  SnDec d;
  d.ring = nullptr;
  d.map = nullptr;
  d.din = uint32_t(src & 3u);
  d.rin = sn_make_rsrc(src - d.din, (d.din + n + 3u) & ~3u);
  d.out = nullptr;
  d.pn = d.poc = d.plb = d.pfb = d.prb = 0;
  d.plit = d.prk = false;
  uint32_t ulen = 0, ip0 = 0;
  for (uint32_t shift = 0;; shift += 7u) {
    if (shift >= 32u || ip0 >= n) return false;
    const uint32_t c = sn_in_byte(d, ip0++);
    ulen |= (c & 0x7Fu) << shift;
    if (c < 128u) break;
  }
  const uint32_t nfrag = (ulen + kSnBlock - 1u) / kSnBlock;
  if (ulen > cap || nfrag < 2u || nfrag > kSnFragMax || ip0 == n) return false;
  constexpr int G = kSnScanGroup;
  uint32_t op = 0, ipn = ip0, found = 0;
  uint32_t base = ipn & ~63u;
  sn_u2 pf[G];
#pragma unroll
  for (int g = 0; g < G; ++g) pf[g] = sn_parse_load(d, base + 64u * uint32_t(g), lane);
  for (bool more = true; more;) {
    SnCand c[G];
    uint32_t P4[G], W[G], MX[G], L[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t seg = base + 64u * uint32_t(g);
      c[g] = sn_parse_words(d, pf[g], n, seg, lane);
      pf[g] = sn_parse_load(d, seg + 64u * uint32_t(G), lane);  // the next group's
      const uint32_t ml = c[g].mk & 0xFFu;
      const bool stop = (c[g].A - seg >= 64u) | (c[g].A == n);
      const bool poison = (c[g].A >= kSnBad) | ((ml != 0u) & (c[g].off == 0u));
      L[g] = poison ? kSnPoison : c[g].ll + ml;
      // a list: successor (the last element of the segment points at itself), bytes up to
      // the successor, largest copy offset from here on
      P4[g] = (stop ? uint32_t(lane) : c[g].A - seg) << 2;
      W[g] = stop ? 0u : L[g];
      MX[g] = ml != 0u ? c[g].off : 0u;
    }
    // (an element takes at least two bytes: at most 32 to a segment)
#pragma unroll
    for (int level = 0; level < 5; ++level) {
      uint32_t w2[G], m2[G], p2[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        w2[g] = uint32_t(__builtin_amdgcn_ds_bpermute(int(P4[g]), int(W[g])));
        m2[g] = uint32_t(__builtin_amdgcn_ds_bpermute(int(P4[g]), int(MX[g])));
        p2[g] = uint32_t(__builtin_amdgcn_ds_bpermute(int(P4[g]), int(P4[g])));
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        W[g] += w2[g];
        MX[g] = max(MX[g], m2[g]);
        P4[g] = p2[g];
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t seg = base + 64u * uint32_t(g);
      if (more && (ipn & ~63u) == seg) {
        const uint32_t x = ipn - seg;
        const uint32_t last = uni(__builtin_amdgcn_readlane(P4[g], x)) >> 2;
        const uint32_t T = uni(__builtin_amdgcn_readlane(W[g], x)) + uni(__builtin_amdgcn_readlane(L[g], last));
        const uint32_t mx = uni(__builtin_amdgcn_readlane(MX[g], x));
        const uint32_t a_last = uni(__builtin_amdgcn_readlane(c[g].A, last));
        if (T > ulen - op || a_last > n) return false;  // (a poisoned length is beyond ulen)
        const uint32_t in0 = op & (kSnBlock - 1u);
        if ((in0 + T > kSnBlock) | (mx > in0)) {
          if (!sn_scan_members(c[g], n, seg, x, op, t, found, lane)) return false;
        } else if (in0 == 0u && op != 0u) {
          if (lane == 0) t->ip[op >> 16] = ipn;
          ++found;
        }
        op = uni(op + T);
        ipn = a_last;
        more = a_last != n;
      }
    }
    const uint32_t nbase = ipn & ~63u;
    if (more && nbase != base + 64u * uint32_t(G)) {  // a literal ran past the group
#pragma unroll
      for (int g = 0; g < G; ++g) pf[g] = sn_parse_load(d, nbase + 64u * uint32_t(g), lane);
    }
    base = nbase;
  }
  if (op != ulen || found != nfrag - 1u) return false;
  if (lane == 0) {
    t->ulen = ulen;
    t->ip0 = ip0;
    t->nfrag = nfrag;
  }
  return true;
}

__global__ __launch_bounds__(64 * kSnDecWaves) void snappy_scan_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, const uint32_t *__restrict__ out_caps,
    uint32_t *__restrict__ out_lens, int32_t *__restrict__ status, SnSplit *__restrict__ tab,
    uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = uni(threadIdx.x >> 6);
  const uint32_t wpb = blockDim.x >> 6;
  for (uint32_t f = blockIdx.x * wpb + w; f < n; f += gridDim.x * wpb) {
    const uintptr_t src = reinterpret_cast<uintptr_t>(in) + in_offs[f];
    SnSplit *t = tab + f;
    const bool ok = sn_scan_stream(src, uni(in_lens[f]), uni(out_caps[f]), t, lane);
    if (lane == 0) {
      t->split = ok ? 1 : 0;
      if (ok) {  // the fragments only report failures
        status[f] = 0;
        out_lens[f] = t->ulen;
      }
    }
  }
}

// items (fragment slot k, stream f), slot-major: fragment k of a split stream, or (k == 0) a
// whole stream that is decoded serially
__global__ __launch_bounds__(64 * kSnDecWaves) void snappy_uncompress_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *out, const uint64_t *__restrict__ out_offs,
    const uint32_t *__restrict__ out_caps, uint32_t *__restrict__ out_lens,
    int32_t *__restrict__ status, const SnSplit *__restrict__ tab, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t rings[kSnDecWaves][kSnRing];
  __shared__ __attribute__((aligned(16))) uint8_t maps[kSnDecWaves][128];
  const int lane = threadIdx.x & 63;
  const uint32_t w = uni(threadIdx.x >> 6);
  sn_lds_u8 *ring = (sn_lds_u8 *)rings[w];
  sn_lds_u8 *map = (sn_lds_u8 *)maps[w];
  const uint32_t wpb = blockDim.x >> 6;
  const uint64_t items = uint64_t(n) * kSnFragMax;
  for (uint64_t it = uint64_t(blockIdx.x) * wpb + w; it < items; it += uint64_t(gridDim.x) * wpb) {
    const uint32_t f = uint32_t(it % n), k = uint32_t(it / n);
    const SnSplit *t = tab + f;
    const uintptr_t src = reinterpret_cast<uintptr_t>(in) + in_offs[f];
    const uintptr_t dst = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    if (uni(uint32_t(t->split))) {
      const uint32_t nfrag = uni(t->nfrag);
      if (k >= nfrag) continue;
      const uint32_t nin = uni(in_lens[f]), ulen = uni(t->ulen);
      const uint32_t ipk = k ? uni(t->ip[k]) : uni(t->ip0);
      const uint32_t ipe = k + 1u < nfrag ? uni(t->ip[k + 1u]) : nin;
      const uint32_t flen = k + 1u < nfrag ? kSnBlock : ulen - k * kSnBlock;
      SnDec d;
      d.ring = ring;
      d.map = map;
      d.din = uint32_t(src & 3u);
      d.rin = sn_make_rsrc(src - d.din, (d.din + nin + 3u) & ~3u);
      sn_set_out(d, dst + uint64_t(k) * kSnBlock);
      d.pn = d.poc = d.plb = d.pfb = d.prb = 0;
      d.plit = d.prk = false;
      const int r = sn_decode_elems(d, ipe, ipk, flen, map, lane);
      if (r != 0 && lane == 0) status[f] = r;
    } else if (k == 0) {
      uint32_t ulen = 0;
      const int r = sn_decode_stream(src, uni(in_lens[f]), dst, uni(out_caps[f]), &ulen, ring, map, lane);
      if (lane == 0) {
        status[f] = r;
        out_lens[f] = ulen;
      }
    }
  }
}

// ------------------------------------------------------------------ host side
size_t snappy_max_compressed_length(size_t len) { return 32 + len + len / 6; }  // snappy.c:639

int snappy_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                           uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                           uint32_t n, hipStream_t s) {
  if (!n) return 0;
  if (n > 0xFFFFFFFFu / kSnItems) return set_error(RDK_HIP_E_INVAL, "too many streams");
  const uint64_t items = uint64_t(n) * kSnItems;
  const unsigned grid = unsigned(items < 65536u ? items : 65536u);
  // RDK_HIP_SNAPPY_SEQ=1 selects the one-copy-at-a-time engine (A/B runs)
  static const bool seq = [] { const char *e = getenv("RDK_HIP_SNAPPY_SEQ"); return e && *e == '1'; }();
  if (seq)
    hipLaunchKernelGGL(snappy_compress_fragments_kernel<false>, dim3(grid), dim3(64), 0, s, d_in,
                       d_in_offs, d_in_lens, d_out, d_out_offs, n);
  else
    hipLaunchKernelGGL(snappy_compress_fragments_kernel<true>, dim3(grid), dim3(64), 0, s, d_in,
                       d_in_offs, d_in_lens, d_out, d_out_offs, n);
  hipLaunchKernelGGL(snappy_assemble_kernel, dim3(n < 4096u ? n : 4096u), dim3(kSnAsmThreads), 0, s, d_in_lens,
                     d_out, d_out_offs, d_out_lens, n);
  RDK_HIP_CHECK(hipGetLastError());
  return 0;
}

int snappy_uncompress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                             uint8_t *d_out, const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                             uint32_t *d_out_lens, int32_t *d_status, uint32_t n, hipStream_t s) {
  if (!n) return 0;
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  // the per-stream fragment tables live in the decoder's scratch region (stream-ordered)
  int rc = scratch_acquire(c, kScratchDecode, size_t(n) * sizeof(SnSplit), s);
  if (rc) return rc;
  SnSplit *tab = reinterpret_cast<SnSplit *>(c->d_stage[kScratchDecode]);
  const unsigned wg = (n + kSnDecWaves - 1) / kSnDecWaves;
  hipLaunchKernelGGL(snappy_scan_kernel, dim3(wg < 2048u ? wg : 2048u), dim3(64 * kSnDecWaves), 0, s,
                     d_in, d_in_offs, d_in_lens, d_out_caps, d_out_lens, d_status, tab, n);
  const uint64_t wgi = (uint64_t(n) * kSnFragMax + kSnDecWaves - 1) / kSnDecWaves;
  hipLaunchKernelGGL(snappy_uncompress_kernel, dim3(unsigned(wgi < 2048u ? wgi : 2048u)),
                     dim3(64 * kSnDecWaves), 0, s, d_in, d_in_offs, d_in_lens, d_out, d_out_offs,
                     d_out_caps, d_out_lens, d_status, tab, n);
  RDK_HIP_CHECK(hipGetLastError());
  return scratch_release(c, kScratchDecode, s);
}

}  // namespace rdk

using namespace rdk;

// rd_kafka_snappy_max_compressed_length (snappy.c:639)
RDK_API size_t rdk_hip_snappy_max_compressed_length(size_t len) {
  return snappy_max_compressed_length(len);
}

RDK_API int rdk_hip_snappy_compress(const void *d_in, const uint64_t *d_in_offs,
                                    const uint32_t *d_in_lens, void *d_out,
                                    const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                                    void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_lens)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  return snappy_compress_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n,
                                static_cast<hipStream_t>(stream));
}

RDK_API int rdk_hip_snappy_uncompress(const void *d_in, const uint64_t *d_in_offs,
                                      const uint32_t *d_in_lens, void *d_out,
                                      const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                                      uint32_t *d_out_lens, int32_t *d_status, uint32_t n,
                                      void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_caps || !d_out_lens ||
      !d_status)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  return snappy_uncompress_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                  static_cast<uint8_t *>(d_out), d_out_offs, d_out_caps, d_out_lens,
                                  d_status, n, static_cast<hipStream_t>(stream));
}
