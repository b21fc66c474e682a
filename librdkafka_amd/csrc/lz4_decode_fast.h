// lz4_decode_fast.h -- batched LZ4 block decoder (independent blocks).
//
// Included by lz4_decode.hip.  decode_block_fast() decodes one independent
// block (LZ4_decompress_safe_usingDict with noDict, lz4.c:2307 ->
// LZ4_decompress_generic lz4.c:1654-2068) without the per-sequence wave
// round trips of the exact decoder.  The compressed block is cut into fixed
// 64-byte segments; per segment:
//
//   1. DISCOVERY: for every byte position p of the segment, lane p%64 parses
//      the sequence that WOULD start at p: token and literal length bytes from
//      the 4 bytes at p, offset and match length bytes from a gather of the 4
//      bytes behind the literals.  Branch-free, two loads, issued one and two
//      segments ahead of their use.
//   2. WALK: the true sequences are the orbit of the entry position under
//      "next start"; it is marked by pointer doubling (5 levels cover the at
//      most 22 sequences a segment can hold), in LDS, with no scalar chain.
//   3. EXPANSION: the member lanes are in stream order, so a lane prefix sum over
//      their lengths places every sequence in the output.  The segment's
//      output is built in pieces of 64 bytes, lane per byte: sequence starts are
//      scattered into a 64-byte LDS map and max-scanned, each lane fetches its
//      sequence's fields (two ds_bpermute) and then its byte -- from the input
//      (literals), the wave's LDS history ring, or the already written output
//      in HBM; sources inside the piece are resolved by pointer jumping.  A
//      fetched piece is written one piece later so its loads overlap the next
//      piece's address work.
//
// The fast path only returns a result when the block is PROVABLY accepted
// by the reference with this output: every condition under which
// LZ4_decompress_generic would return an error (or could even take a
// different branch that matters) is checked -- offset 0, a match before the
// block start, length bytes read too close to the input end (lz4.c:1625
// read_variable_length limits), the end-of-block literal / match margins
// (MFLIMIT, LASTLITERALS, lz4.c:1850-1880 / 1986-2004), the last sequence
// ending exactly at the input end, the caller's capacity.  Anything else
// returns kFastFallback and the block is re-decoded from scratch by the
// exact decoder (decode_block), which then decides the verdict.
// (textually included inside namespace rdk, after the ring definitions)
#pragma once

constexpr int kFastFallback = -100;
constexpr uint32_t kLitTag = 0x80000000u;
constexpr uint32_t kSeqComplex = 0xFFFFFFFFu;  // header longer than the lane window
constexpr uint32_t kSeqBad = 0xFFFFFFFEu;      // the reference would reject it
constexpr uint32_t kNoAccess = 0x80000000u;    // out-of-range buffer offset (reads 0)

typedef __amdgpu_buffer_rsrc_t rsrc_t;
// lane mask of a predicate, straight from the compare (no 0/1 round trip through a VGPR)
__device__ __forceinline__ uint64_t fballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ rsrc_t make_rsrc(uintptr_t base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), 0, int(bytes),
                                           0x00020000);
}

struct FastDec {
  lds_u8 *ring;      // kRing bytes of the newest output
  lds_u8 *map;       // 128 bytes: [0, 64) per-piece scratch, [64, 128) stores of parked lanes
  rsrc_t rin;        // compressed block [0, csize)
  g_u8 *out;         // block output; every position written or read lies below the checked end
  uint32_t csize;
  // the previous piece, fetched but not yet written: its HBM loads stay in
  // flight while the next piece's sources are worked out
  uint32_t pn, poc;  // live bytes (0: none) and output position
  uint32_t plb, pfb, prb;  // the byte as each of the three sources delivered it
  bool plit, prk;          // which one holds it: literal, history ring, else far history
};

// ring byte of output position x (the ring starts at a multiple of its size in LDS, so the
// position's low bits are ORed into the base)
__device__ __forceinline__ lds_u8 *ring_at(const FastDec &d, uint32_t x) {
  return (lds_u8 *)(uintptr_t)(uint32_t(uintptr_t(d.ring)) | (x & kRingMask));
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m, uint32_t add) {
  return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), add));
}
// value of lane `idx` (modulo 64), any lane pattern
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t idx) {
  return uint32_t(__builtin_amdgcn_ds_bpermute(int(idx << 2), int(v)));
}

// Output reaches memory a whole kOutChunk at a time, from the history ring, as one aligned
// 16-byte store per lane: memory takes whole sectors well and pieces of a few bytes at
// arbitrary alignment badly (every partly written sector is first read back from HBM; the
// decoder fetched four times its output that way).
constexpr uint32_t kOutChunk = 1024;
typedef uint32_t fd_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t fd_u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) fd_u32x4 fd_lds_u32x4;
typedef __attribute__((address_space(1))) fd_u32x4_a1 fd_g_u32x4;

// ring -> memory: output [c0, c0 + n), c0 a multiple of kOutChunk, n <= kOutChunk
__device__ __forceinline__ void fast_write_out(const FastDec &d, uint32_t c0, uint32_t n, int lane) {
  const uint32_t o = c0 + 16u * uint32_t(lane), l16 = 16u * uint32_t(lane);
  if (l16 + 16u <= n) {
    *(fd_g_u32x4 *)(d.out + o) = *(fd_lds_u32x4 *)ring_at(d, o);
  } else if (l16 < n) {  // the block's last, partial 16 bytes
    for (uint32_t j = 0; j < n - l16; ++j) d.out[o + j] = *ring_at(d, o + j);
  }
}

// Write the pending piece into the history ring, and the chunk it completes to HBM.
__device__ __forceinline__ void fast_retire(FastDec &d, int lane) {
  __builtin_amdgcn_sched_barrier(0);  // keep the wait for the piece's loads down here
  // (the three values pass through empty asm statements: a select between fields of `d`
  // would otherwise be turned into one load through a selected address, which puts the
  // fields into scratch memory)
  uint32_t a = d.plb, b = d.prb, c = d.pfb;
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
  const uint32_t v = d.plit ? a : (d.prk ? b : c);
  if (uint32_t(lane) < d.pn) *ring_at(d, d.poc + uint32_t(lane)) = uint8_t(v);
  asm volatile("" ::: "memory");
  // (a piece is at most 64 bytes: it completes at most one chunk)
  if (((d.poc + d.pn) ^ d.poc) & ~(kOutChunk - 1u)) fast_write_out(d, d.poc & ~(kOutChunk - 1u), kOutChunk, lane);
  d.pn = 0;
}

// Fetch output bytes [pc, pc+nvalid): lane l's byte comes from `src` (kLitTag | input
// position, or an output position below its own; all ones in a lane without a byte).
// They are written by the next retire.
__device__ __forceinline__ void fast_flush(FastDec &d, uint32_t src, uint32_t pc, uint32_t nvalid,
                                           int lane) {
  // match sources inside this piece: pointer jumping, each step halves the
  // remaining hops (sources always point to lower lanes).  The shuffle is
  // unconditional: under a lane predicate its source lanes would read zeros.
  for (;;) {
    // (a literal source has the tag bit set: the signed compare keeps it out)
    const bool intra = int32_t(src) >= int32_t(pc);
    if (!fballot(intra)) break;
    const uint32_t v = lane_read(src, src - pc);
    src = intra ? v : src;
  }
  fast_retire(d, lane);  // the ring must hold everything before pc
  const bool lit = int32_t(src) < 0;
  const uint32_t q = src & ~kLitTag;
  const bool rk = q + kRing >= pc;  // a match source still in the history ring
  // a literal's position is in range of the input only with its tag taken off; a lane
  // without a byte (all ones) stays out of range either way
  d.plb = __builtin_amdgcn_raw_buffer_load_b8(d.rin, src ^ kLitTag, 0, 0);
  // Far history left the ring for memory at least (kRing - kOutChunk) / 64 pieces ago (the
  // static_assert below keeps that at 32 or more), each of which ended in fast_retire's wait
  // for its three loads.  The load below relies on two properties of gfx950 that the
  // language does not promise: vector-memory operations of one wavefront reach the CU's
  // cache in program order, and vmcnt retires in order, so a store issued before a load
  // that has since been waited for has itself completed.  The bytes were stored by other
  // lanes of this same wavefront through this same cache, which a store updates.
  // tests/test_gpu_lz4.py (matches around the history ring edge) exercises exactly these
  // sources.
  static_assert(kRing >= kOutChunk + 2048u, "far history must be at least 32 pieces old");
  d.pfb = d.out[(lit | rk) ? 0u : q];
  asm volatile("" ::: "memory");  // ring bytes stored by other lanes
  d.prb = *ring_at(d, q);
  d.plit = lit;
  d.prk = rk;
  d.pn = nvalid;
  d.poc = pc;
}

// Candidate sequence of lane `lane` of segment [seg, seg+64): the sequence
// that would start at p = seg+lane.
//   A: next sequence start, kSeqComplex, or kSeqBad
//   B: literal length | match length << 16 (match length 0: last sequence)
//   C: offset | (literal start - p) << 16
struct SegCand {
  uint32_t A, B, C;
};

typedef uint32_t seg_u2 __attribute__((ext_vector_type(2)));

// discovery, first load: the aligned 8 bytes holding the 4 bytes at p
__device__ __forceinline__ seg_u2 seg_load_head(rsrc_t rin, uint32_t seg, int lane) {
  return __builtin_amdgcn_raw_buffer_load_b64(rin, (seg + uint32_t(lane)) & ~3u, 0, 0);
}

// Token and literal length of the candidate at p: ll, header bytes k, flags
struct SegHead {
  uint32_t tok, ll, k, lit_end;
  bool bad, complex;
};

// CHECKED = false: for a segment whose last candidate ends its length bytes before the
// limits below (seg + 63 + 4 < csize - 15), where none of them can trip
template <bool CHECKED = true>
__device__ __forceinline__ SegHead seg_head(seg_u2 h, uint32_t csize, uint32_t seg, int lane) {
  const uint32_t p = seg + uint32_t(lane);
  const uint32_t w0 = __builtin_amdgcn_alignbyte(h.y, h.x, p & 3u);
  SegHead r;
  r.tok = w0 & 0xFFu;
  uint32_t ll = r.tok >> 4;
  const uint32_t b1 = (w0 >> 8) & 0xFFu, b2 = (w0 >> 16) & 0xFFu, b3 = w0 >> 24;
  const bool e0 = ll == 15u;          // length bytes follow
  const bool e1 = e0 & (b1 == 255u);
  const bool e2 = e1 & (b2 == 255u);
  const bool e3 = e2 & (b3 == 255u);  // the run continues past the 4 bytes
  ll += (e0 ? b1 : 0u) + (e1 ? b2 : 0u) + (e2 ? b3 : 0u);
  r.k = 1u + uint32_t(e0) + uint32_t(e1) + uint32_t(e2);
  // read_variable_length(iend-15, initial_check): error if ip >= iend-15; a 255 read at
  // ip >= iend-15 stops the reference's loop early (loop_error, tolerated for literals)
  // where this parse would go on
  const uint32_t lim = csize - 15u;
  r.bad = CHECKED && ((e0 & ((p + 1u >= lim) | (csize < 16u))) | (e1 & (p + 2u >= lim)) |
                      (e2 & (p + 3u >= lim)) | (e3 & (p + 4u >= lim)) | (p >= csize));
  r.complex = e3;
  r.ll = ll;
  r.lit_end = p + r.k + ll;
  return r;
}

// discovery, second load: the aligned 8 bytes holding the 4 bytes behind the literals
__device__ __forceinline__ seg_u2 seg_load_tail(rsrc_t rin, const SegHead &hd) {
  return __builtin_amdgcn_raw_buffer_load_b64(rin, hd.lit_end & ~3u, 0, 0);
}

__device__ __forceinline__ SegCand seg_finish(const SegHead &hd, seg_u2 g, uint32_t csize) {
  const uint32_t dw = __builtin_amdgcn_alignbyte(g.y, g.x, hd.lit_end & 3u);
  const bool last = hd.lit_end == csize;  // literals-only last sequence
  const uint32_t off = dw & 0xFFFFu;
  uint32_t ml = hd.tok & 15u;
  const uint32_t c1 = (dw >> 16) & 0xFFu, c2 = dw >> 24;
  const bool f0 = ml == 15u;
  const bool f1 = f0 & (c1 == 255u);
  const bool f2 = f1 & (c2 == 255u);  // the run continues past the 4 bytes
  ml += (f0 ? c1 : 0u) + (f1 ? c2 : 0u) + uint32_t(kLz4MinMatch);
  // read_variable_length(iend-LASTLITERALS+1): error once ip >= iend-4, for every byte read
  const uint32_t m0 = hd.lit_end + 2u;
  const bool mbad = (off == 0u) |  // the reference writes garbage for offset 0
                    (f0 & ((m0 + 1u >= csize - 4u) | (csize < 5u))) | (f1 & (m0 + 2u >= csize - 4u));
  const bool bad = hd.bad | (!last & !hd.complex & mbad);
  const bool complex = hd.complex | (!last & f2);
  const uint32_t next = last ? csize : m0 + uint32_t(f0) + uint32_t(f1);
  SegCand c;
  c.A = bad ? kSeqBad : (complex ? kSeqComplex : next);
  c.B = (hd.ll & 0xFFFFu) | ((last ? 0u : ml) << 16);
  c.C = (last ? 0u : off) | (hd.k << 16);
  return c;
}

__device__ __forceinline__ SegCand seg_parse(const FastDec &d, uint32_t seg, int lane) {
  const SegHead hd = seg_head(seg_load_head(d.rin, seg, lane), d.csize, seg, lane);
  return seg_finish(hd, seg_load_tail(d.rin, hd), d.csize);
}

// Byte `i` of the compressed block, wave-uniform (slow path only).
__device__ __forceinline__ uint32_t in_byte(rsrc_t rin, uint32_t i) {
  return __builtin_amdgcn_readfirstlane(__builtin_amdgcn_raw_buffer_load_b8(rin, i, 0, 0));
}

// Scalar parse of the sequence at p whose header does not fit a lane
// window (long literal / match length runs).  Same checks as seg_parse.
__device__ __forceinline__ SegCand seq_slow(rsrc_t rin, uint32_t csize, uint32_t p) {
  SegCand c;
  uint32_t tok = in_byte(rin, p), ll = tok >> 4, k = 1u;
  bool bad = false;
  if (ll == 15u) {
    if (p + 1u >= csize - 15u || csize < 16u) bad = true;
    uint32_t b;
    do {
      if (p + k >= csize) { bad = true; break; }
      b = in_byte(rin, p + k);
      if (b == 255u && p + k + 1u >= csize - 15u) bad = true;
      ll += b;
      ++k;
    } while (b == 255u);
  }
  const uint32_t lit_end = p + k + ll;
  uint32_t ml = 0, off = 0, next = csize;
  if (!bad && lit_end != csize) {
    if (lit_end + 2u > csize) bad = true;
    else {
      off = in_byte(rin, lit_end) | (in_byte(rin, lit_end + 1u) << 8);
      if (off == 0u) bad = true;
      ml = tok & 15u;
      uint32_t m = lit_end + 2u;
      if (ml == 15u) {
        uint32_t b;
        do {
          if (m >= csize || m + 1u >= csize - 4u || csize < 5u) { bad = true; break; }
          b = in_byte(rin, m);
          ml += b;
          ++m;
        } while (b == 255u);
      }
      ml += uint32_t(kLz4MinMatch);
      next = m;
    }
  }
  if (ll > 0xFFFFu || ml > 0xFFFFu) bad = true;
  c.A = bad ? kSeqBad : next;
  c.B = (ll & 0xFFFFu) | (ml << 16);
  c.C = off | (k << 16);
  return c;
}

// inclusive max over lanes 0..lane (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  int x = int(v);
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true));   // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true));   // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true));   // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true));   // row_shr:8
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return uint32_t(x);
}

// exclusive prefix sum over lanes (DPP), `total` = wave sum
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t &total) {
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

// Decode one independent block, a whole 64-byte input segment at a time (see the file
// comment).  Returns the decoded size or kFastFallback.
__device__ int decode_block_fast(uintptr_t src, uint32_t csize, uintptr_t dst, uint32_t oend,
                                 uint32_t realcap, lds_u8 *ring, lds_u8 *map, int lane) {
  if (csize < 16u || csize > 65536u || oend > 65536u || oend < 64u) return kFastFallback;
  FastDec d;
  d.ring = ring;
  d.map = map;
  d.rin = make_rsrc(src, csize);
  // wave-uniform base: the output is addressed as scalar base + lane offset
  d.out = (g_u8 *)(
      (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(uint64_t(dst) >> 32)))) << 32) |
      uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(dst)))));
  d.csize = csize;
  d.pn = d.poc = d.plb = d.pfb = d.prb = 0;
  d.plit = d.prk = false;
  const uint32_t olimit = realcap < 65536u ? realcap : 65536u;
  uint32_t op = 0, ipn = 0;
  // the last non-final sequence decides the end-of-block margins
  uint32_t last_cpy = 0, last_lit_end = 0, last_mend = 0;
  bool have_last = false;
  uint32_t seg = 0;
  SegCand cur = seg_parse(d, 0u, lane);
  // discovery pipeline: the head of segment seg+64 is parsed and its tail gather issued
  // before this segment is expanded; the head bytes of seg+128 are in flight
  seg_u2 h2 = seg_load_head(d.rin, 64u, lane);
  for (;;) {
    const SegHead nhd = seg + 64u + 63u + 4u + 15u < csize
                            ? seg_head<false>(h2, csize, seg + 64u, lane)
                            : seg_head<true>(h2, csize, seg + 64u, lane);
    const seg_u2 ng = seg_load_tail(d.rin, nhd);
    h2 = seg_load_head(d.rin, seg + 128u, lane);
    // ---- walk: which candidate lanes are the real sequences of this segment
    const uint32_t x0 = ipn - seg;
    uint64_t M;
    bool mem;
    for (;;) {
      // bad, complex, leaves the segment, or ends the block (nothing may follow csize)
      const bool stop = (cur.A - seg >= 64u) | (cur.A == csize);
      // successor lane as a permute address (lane * 4); 256: none
      uint32_t J = stop ? 256u : (cur.A - seg) << 2;
      bool R = uint32_t(lane) == x0;
      // One level: every reached lane marks its successor (a forward permute is a scatter;
      // lanes that mark nothing mark the entry lane, which nothing else targets and which
      // is reached anyway), then the successor map is squared.
#pragma unroll
      for (int level = 0; level < 5; ++level) {
        const bool send = R & (J < 256u);
        const int t = __builtin_amdgcn_ds_permute(int(send ? J : x0 << 2), 1);
        R = R | (t != 0);
        const uint32_t jj = uint32_t(__builtin_amdgcn_ds_bpermute(int(J), int(J)));
        J = J < 256u ? jj : 256u;
      }
      mem = R;
      const uint32_t ra = R ? cur.A : 0u;
      M = fballot(ra != 0u);  // (a member's A is never 0)
      const uint64_t cx = fballot(ra >= kSeqBad);  // kSeqBad or kSeqComplex among the members
      if (!cx) break;
      if (fballot(ra == kSeqBad)) return kFastFallback;
      // header too long for the lane's bytes: parse it scalar, then walk again
      const uint32_t xc = uint32_t(__builtin_ctzll(cx));
      const SegCand sc = seq_slow(d.rin, csize, seg + xc);
      if (sc.A == kSeqBad) return kFastFallback;
      const bool me = uint32_t(lane) == xc;
      cur.A = me ? sc.A : cur.A;
      cur.B = me ? sc.B : cur.B;
      cur.C = me ? sc.C : cur.C;
    }
    const uint32_t xl = uint32_t(63 - __builtin_clzll(M));  // last member (M holds x0)
    const uint32_t a_last = uni(__builtin_amdgcn_readlane(cur.A, xl));
    const bool done = a_last == csize;  // nothing can follow: the literals-only last sequence
    // ---- the segment's sequences, one per member lane, in lane order
    const uint32_t ll = cur.B & 0xFFFFu, ml = cur.B >> 16, off = cur.C & 0xFFFFu;
    const uint32_t ls = seg + uint32_t(lane) + (cur.C >> 16);
    uint32_t T;
    const uint32_t len = mem ? ll + ml : 0u;
    const uint32_t ostart = op + wave_excl_sum(len, T);
    const uint32_t cpy = ostart + ll;
    // (ballots straight from one compare each: a ballot of a combined predicate goes
    // through a 0/1 register)
    const bool mm = (mem ? ml : 0u) != 0u;
    if (fballot((mm ? off : 0u) > cpy)) return kFastFallback;  // match < lowPrefix
    if (op + T > olimit) return kFastFallback;  // the exact path reports the size error
    const uint64_t nl = fballot(mm);
    if (nl) {
      const int j = 63 - __builtin_clzll(nl);
      last_cpy = __builtin_amdgcn_readlane(cpy, j);
      last_lit_end = __builtin_amdgcn_readlane(ls + ll, j);
      last_mend = __builtin_amdgcn_readlane(cpy + ml, j);
      have_last = true;
    }
    if (done) {
      const uint32_t lml = __builtin_amdgcn_readlane(ml, xl);
      const uint32_t lcpy = __builtin_amdgcn_readlane(cpy, xl);
      if (lml != 0u || lcpy > oend) return kFastFallback;
      if (have_last && (last_cpy > oend - uint32_t(kLz4MFLimit) ||
                        last_lit_end > csize - uint32_t(2 + 1 + kLz4LastLiterals) ||
                        last_mend > oend - uint32_t(kLz4LastLiterals)))
        return kFastFallback;
    }
    // ---- output [op, op+T) in pieces of 64 bytes, lane per byte
    const uint32_t op_new = uni(op + T);
    // the sequences that have bytes, packed into the low lanes in stream order (a sequence
    // without bytes can only be the last one)
    const uint64_t Mn = fballot(len != 0u);
    const uint32_t slot = len != 0u ? lanes_below(Mn, 0u) : 63u;  // at most 22 sequences
    const uint32_t f1 = uint32_t(__builtin_amdgcn_ds_permute(int(slot << 2), int(ll | (off << 16))));
    // (a sequence with bytes starts below 65536)
    const uint32_t f2 =
        uint32_t(__builtin_amdgcn_ds_permute(int(slot << 2), int((ostart & 0xFFFFu) | (ls << 16))));
    const uint32_t ost = len != 0u ? ostart : 0x80000000u;
    uint32_t before = 0xFFFFFFFFu;  // sequences that start before the piece, less one
    for (uint32_t c = op; c < op_new; c = uni(c + 64u)) {
      // sequence whose output starts at or before each lane's byte: the starts in this piece
      // are scattered into the map; a lane's sequence is the count of starts up to its byte
      // (compiler barriers: other lanes' LDS stores are invisible to the optimizer, which
      // would otherwise forward map[lane] = 0 to the read)
      map[lane] = 0;
      asm volatile("" ::: "memory");
      const uint32_t rel0 = ost - c;
      map[rel0 < 64u ? rel0 : 64u + uint32_t(lane)] = 1;
      asm volatile("" ::: "memory");
      const uint64_t sb = fballot(map[lane] != 0);
      const int idx4 =
          int((lanes_below(sb >> 1, 0u) << 2) + uni((before + uint32_t(sb & 1ull)) << 2));
      before = uni(before + uint32_t(__builtin_popcountll(sb)));
      const uint32_t g1 = uint32_t(__builtin_amdgcn_ds_bpermute(idx4, int(f1)));
      const uint32_t g2 = uint32_t(__builtin_amdgcn_ds_bpermute(idx4, int(f2)));
      const uint32_t o = c + uint32_t(lane);
      const uint32_t rel = (o - g2) & 0xFFFFu;
      const uint32_t s_lit = ((g2 >> 16) + rel) | kLitTag, s_mat = o - (g1 >> 16);
      const uint32_t s = rel < (g1 & 0xFFFFu) ? s_lit : s_mat;
      const uint32_t left = op_new - c;
      const uint32_t nv = left < 64u ? left : 64u;
      fast_flush(d, uint32_t(lane) < nv ? s : 0xFFFFFFFFu, c, nv, lane);
    }
    op = op_new;
    if (done) {
      fast_retire(d, lane);
      fast_write_out(d, op & ~(kOutChunk - 1u), op & (kOutChunk - 1u), lane);
      return int(op);
    }
    ipn = a_last;
    // ---- next segment (usually the one in the discovery pipeline)
    const uint32_t nseg = ipn & ~63u;
    if (nseg >= csize) return kFastFallback;  // ran off the input without a last sequence
    if (nseg == seg + 64u) {
      cur = seg_finish(nhd, ng, csize);
    } else {
      cur = seg_parse(d, nseg, lane);
      h2 = seg_load_head(d.rin, nseg + 64u, lane);
    }
    seg = nseg;
  }
}
