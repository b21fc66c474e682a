// lz4_decode_fast.h -- batched LZ4 block decoder (independent blocks).
//
// Included by lz4_decode.hip.  decode_block_fast() decodes one independent
// block (LZ4_decompress_safe_usingDict with noDict, lz4.c:2307 ->
// LZ4_decompress_generic lz4.c:1654-2068) without the per-sequence wave
// round trips of the exact decoder:
//
//   1. DISCOVERY: the compressed block is cut into fixed 64-byte segments.
//      For every byte position p of a segment, lane p%64 parses the
//      sequence that WOULD start at p (token, literal / match length bytes,
//      offset) from a 24-byte register window of its own, so a whole
//      segment's candidates cost two loads and ~40 VALU.
//   2. WALK: the true sequence chain is followed with one v_readlane per
//      sequence (next start -> lane), scalar.  Each sequence "paints" the
//      64-byte output chunk under construction: lane l of the chunk records
//      where output byte oc+l comes from (an input position for literals,
//      an earlier output position for matches).
//   3. FLUSH: a complete chunk resolves its in-chunk match sources by
//      pointer jumping (ds_bpermute, only when some offset < 64), fetches
//      every byte at once (input, the wave's 8 KiB LDS history ring, or the
//      already written output in HBM) and stores 64 contiguous bytes.
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
__device__ __forceinline__ rsrc_t make_rsrc(uintptr_t base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), 0, int(bytes),
                                           0x00020000);
}

struct FastDec {
  uintptr_t dst;
  lds_u8 *ring;      // kRing bytes of the newest output
  rsrc_t rin;        // compressed block [0, csize)
  rsrc_t rout;       // block output [0, realcap)
  uint32_t csize, oend, realcap;
  uint32_t oc;       // output position of the chunk being painted
  uint32_t dsrc;     // lane l: source of output byte oc+l (kLitTag | input pos, or output pos)
  // the previous chunk, fetched but not yet written: its HBM loads stay in
  // flight while the next chunk is painted
  uint32_t pn, poc;  // live bytes (0: none) and output position
  uint32_t plb, pfb, prb;
};

// Write the pending chunk into the history ring and to HBM.  Each lane's byte
// arrived in exactly one of its three sources (parked loads read 0).
__device__ __forceinline__ void fast_retire(FastDec &d, int lane) {
  if (!d.pn) return;
  const bool live = uint32_t(lane) < d.pn;
  const uint32_t v = d.plb | d.pfb | d.prb;
  if (live) d.ring[(d.poc + uint32_t(lane)) & kRingMask] = uint8_t(v);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v), d.rout, live ? d.poc + uint32_t(lane) : kNoAccess,
                                      0, 0);
  d.pn = 0;
}

// Resolve and fetch output bytes [oc, oc+nvalid) of the painted chunk; they
// are written by the next retire, so the loads overlap the next painting.
__device__ __forceinline__ void fast_flush(FastDec &d, uint32_t nvalid, int lane) {
  fast_retire(d, lane);  // the ring must hold everything before oc
  uint32_t src = d.dsrc;
  const bool live = uint32_t(lane) < nvalid;
  // match sources inside this chunk: pointer jumping, each step halves the
  // remaining hops (sources always point to lower lanes)
  for (;;) {
    const bool intra = live && !(src & kLitTag) && src >= d.oc;
    if (!ballot(intra)) break;
    const uint32_t v = uint32_t(__shfl(int(src), intra ? int(src - d.oc) : lane));
    if (intra) src = v;
  }
  const bool lit = (src & kLitTag) != 0u;
  const uint32_t q = src & ~kLitTag;
  const bool ring_ok = !lit && q + kRing >= d.oc;  // still in the history ring
  const bool far = live && !lit && !ring_ok;
  // far history was stored >= kRing/64 chunks (>= 64 vector-memory ops) ago:
  // with in-order vmcnt retirement it has completed, so no wait is needed
  d.plb = __builtin_amdgcn_raw_buffer_load_b8(d.rin, (live && lit) ? q : kNoAccess, 0, 0);
  d.pfb = __builtin_amdgcn_raw_buffer_load_b8(d.rout, far ? q : kNoAccess, 0, 0);
  asm volatile("" ::: "memory");  // ring bytes stored by other lanes
  d.prb = d.ring[q & kRingMask] & (ring_ok ? 0xFFu : 0u);
  d.pn = nvalid;
  d.poc = d.oc;
}

// output [a, b) takes its bytes from source positions s, s+1, ... (tag marks
// input positions); completes and flushes chunks on the way
__device__ __forceinline__ void fast_paint(FastDec &d, uint32_t a, uint32_t b, uint32_t s,
                                           uint32_t tag, int lane) {
  while (a < b) {
    const uint32_t ce = d.oc + 64u;
    const uint32_t e = b < ce ? b : ce;
    const uint32_t rel = uint32_t(lane) + d.oc - a;
    if (rel < e - a) d.dsrc = (s + rel) | tag;
    s += e - a;
    a = e;
    if (a == ce) {
      fast_flush(d, 64u, lane);
      d.oc = ce;
    }
  }
}

// Candidate sequence of lane `lane` of segment [seg, seg+64): the sequence
// that would start at p = seg+lane, parsed from 24 bytes of registers.
//   A: next sequence start, kSeqComplex, or kSeqBad
//   B: literal length | match length << 16 (match length 0: last sequence)
//   C: offset | (literal start - p) << 16
struct SegCand {
  uint32_t A, B, C;
};

// 20 bytes of a lane's window as named words (no array: a runtime-indexed
// register array would be demoted to scratch)
struct Win20 {
  uint32_t w0, w1, w2, w3, w4;
};

// 4 bytes starting `k` bytes into the window (k <= 19; bytes past 20 read 0)
__device__ __forceinline__ uint32_t win4(const Win20 &w, uint32_t k) {
  const uint32_t j = k >> 2;
  const uint32_t lo = j == 0 ? w.w0 : j == 1 ? w.w1 : j == 2 ? w.w2 : j == 3 ? w.w3 : w.w4;
  const uint32_t hi = j == 0 ? w.w1 : j == 1 ? w.w2 : j == 2 ? w.w3 : j == 3 ? w.w4 : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, k & 3u);
}

__device__ __forceinline__ SegCand seg_parse(const FastDec &d, uint32_t seg, int lane) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  const uint32_t p = seg + uint32_t(lane);
  const uint32_t a = p & ~3u, sh = p & 3u;
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(d.rin, a, 0, 0);
  const u2 x = __builtin_amdgcn_raw_buffer_load_b64(d.rin, a + 16u, 0, 0);
  Win20 w;  // bytes p .. p+19
  w.w0 = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
  w.w1 = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
  w.w2 = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
  w.w3 = __builtin_amdgcn_alignbyte(x.x, v.w, sh);
  w.w4 = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
  const uint32_t csize = d.csize;
  SegCand c;
  const uint32_t tok = w.w0 & 0xFFu;
  uint32_t ll = tok >> 4, k = 1u;
  bool complex = false, bad = false;
  if (ll == 15u) {
    // read_variable_length(iend-15, initial_check): error if ip >= iend-15
    if (p + 1u >= csize - 15u || csize < 16u) bad = true;
    uint32_t b;
    do {
      b = (win4(w, k) & 0xFFu);
      // a 255 read at ip >= iend-15 stops the reference's loop early
      // (loop_error, tolerated for literals) where this parse would go on
      if (b == 255u && p + k + 1u >= csize - 15u) bad = true;
      ll += b;
      ++k;
    } while (b == 255u && k < 4u);
    if (b == 255u) complex = true;  // run continues past the window
  }
  const uint32_t lit_end = p + k + ll;
  uint32_t ml = 0, off = 0, next;
  if (lit_end == csize) {  // literals-only last sequence
    next = csize;
  } else {
    const uint32_t r = lit_end - p;
    if (r + 3u > 20u) {
      complex = true;
      next = 0;
    } else {
      const uint32_t dw = win4(w, r);
      off = dw & 0xFFFFu;
      if (off == 0u) bad = true;  // the reference writes garbage for it
      ml = tok & 15u;
      uint32_t m = r + 2u;
      if (ml == 15u) {
        uint32_t b;
        do {
          if (m >= 20u) { complex = true; break; }
          b = win4(w, m) & 0xFFu;
          // read_variable_length(iend-LASTLITERALS+1): error once ip >= iend-4
          if (p + m + 1u >= csize - 4u || csize < 5u) bad = true;
          ml += b;
          ++m;
        } while (b == 255u);
      }
      ml += uint32_t(kLz4MinMatch);
      next = p + m;
    }
  }
  c.A = bad ? kSeqBad : (complex ? kSeqComplex : next);
  c.B = (ll & 0xFFFFu) | (ml << 16);
  c.C = off | (k << 16);
  if (p >= csize) c.A = kSeqBad;  // no sequence can start past the input
  return c;
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

// Decode one independent block, a whole 64-byte input segment at a time.
// The chain walk only marks which candidate lanes are real sequences (one
// v_readlane + one s_bitset per sequence); everything else is vector work
// over the segment's sequences: output offsets by a lane prefix sum, the
// reference's acceptance checks by ballot, and the output chunks painted
// lane-per-byte (LDS scatter of sequence starts + max scan).
// Returns the decoded size or kFastFallback.
__device__ int decode_block_fast(uintptr_t src, uint32_t csize, uintptr_t dst, uint32_t oend,
                                 uint32_t realcap, lds_u8 *ring, lds_u8 *map, int lane) {
  if (csize < 16u || csize > 65536u || oend > 65536u || oend < 64u) return kFastFallback;
  FastDec d;
  d.dst = dst;
  d.ring = ring;
  d.rin = make_rsrc(src, csize);
  d.rout = make_rsrc(dst, realcap);
  d.csize = csize;
  d.oend = oend;
  d.realcap = realcap;
  d.oc = 0;
  d.dsrc = 0;
  d.pn = d.poc = d.plb = d.pfb = d.prb = 0;
  uint32_t op = 0, ipn = 0;
  // the last non-final sequence decides the end-of-block margins
  uint32_t last_cpy = 0, last_lit_end = 0, last_mend = 0;
  bool have_last = false;
  uint32_t seg = 0;
  SegCand cur = seg_parse(d, 0u, lane);
  SegCand nxt = seg_parse(d, 64u, lane);
  for (;;) {
    // ---- walk: which candidate lanes are the real sequences of this segment
    uint64_t M = 0;
    uint32_t x = ipn - seg;
    bool done = false;
    while (x < 64u) {
      uint32_t a = __builtin_amdgcn_readlane(cur.A, x);
      if (a == kSeqComplex) {  // header too long for the lane window: parse it scalar
        const SegCand s = seq_slow(d.rin, csize, seg + x);
        const bool me = uint32_t(lane) == x;
        cur.A = me ? s.A : cur.A;
        cur.B = me ? s.B : cur.B;
        cur.C = me ? s.C : cur.C;
        a = s.A;
      }
      if (a == kSeqBad) return kFastFallback;
      M |= 1ull << x;
      if (a == csize) {  // nothing can follow: must be the literals-only last sequence
        done = true;
        break;
      }
      x = a - seg;
    }
    const uint32_t xl = x;  // last member (only meaningful when done)
#ifdef RDK_DEC_DEBUG
    if (lane == 0 && seg < 512)
      printf("seg %u ipn %u x %u M %016lx done %d op %u oc %u\n", seg, ipn, x, (unsigned long)M,
             int(done), op, d.oc);
#endif
    // ---- the segment's sequences, one per member lane, in lane order
    const bool mem = (M >> lane) & 1ull;
    const uint32_t ll = cur.B & 0xFFFFu, ml = cur.B >> 16, off = cur.C & 0xFFFFu;
    const uint32_t ls = seg + uint32_t(lane) + (cur.C >> 16);
    uint32_t T;
    const uint32_t ostart = op + wave_excl_sum(mem ? ll + ml : 0u, T);
    const uint32_t cpy = ostart + ll;
    if (ballot(mem && ml != 0u && off > cpy)) return kFastFallback;  // match < lowPrefix
    if (op + T > realcap) return kFastFallback;  // the exact path reports the size error
    const uint64_t nl = ballot(mem && ml != 0u);
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
    // ---- paint output [op, op+T) into 64-byte chunks, flushing full ones
    const uint32_t op_new = op + T;
    const uint32_t ffield = ll | (off << 16);
    for (uint32_t c = d.oc; c < op_new; c += 64u) {
      const uint32_t lo = op > c ? op : c;
      const uint32_t hi = op_new < c + 64u ? op_new : c + 64u;
      // member whose output starts at or before each lane's byte: starts in
      // this chunk are scattered into the map and max-scanned; lanes before
      // the chunk's first start take the member running into the chunk
      // (compiler barriers: other lanes' LDS stores are invisible to the
      // optimizer, which would otherwise forward map[lane] = 0 to the read)
      map[lane] = 0;
      asm volatile("" ::: "memory");
      if (mem && ostart >= c && ostart < c + 64u && ll + ml != 0u) map[ostart - c] = uint8_t(lane + 1);
      asm volatile("" ::: "memory");
      uint32_t v = wave_incl_max(map[lane]);
      const uint64_t before = ballot(mem && ostart < c && ll + ml != 0u);
      const uint32_t carry = before ? uint32_t(64 - __builtin_clzll(before)) : 0u;
      v = v ? v : carry;
      const int idx = int(v ? v - 1u : 0u);
      const uint32_t fo = uint32_t(__shfl(int(ostart), idx));
      const uint32_t ff = uint32_t(__shfl(int(ffield), idx));
      const uint32_t fl = uint32_t(__shfl(int(ls), idx));
      const uint32_t o = c + uint32_t(lane);
      const uint32_t rel = o - fo;
      const uint32_t s = rel < (ff & 0xFFFFu) ? ((fl + rel) | kLitTag) : (o - (ff >> 16));
      if (o >= lo && o < hi) d.dsrc = s;
#ifdef RDK_DEC_DEBUG
      if (seg == 64 && c == 64 && lane >= 10 && lane < 24)
        printf("L%d mem %d ostart %u ll %u ml %u off %u ls %u | v %u fo %u ff %08x fl %u s %08x\n",
               lane, int(mem), ostart, ll, ml, off, ls, v, fo, ff, fl, s);
#endif
      if (hi == c + 64u) {
        fast_flush(d, 64u, lane);
        d.oc = c + 64u;
      }
    }
    op = op_new;
    if (done) {
      if (op > d.oc) fast_flush(d, op - d.oc, lane);
      fast_retire(d, lane);
      return int(op);
    }
    ipn = seg + x;
    // ---- next segment (usually the prefetched one)
    const uint32_t nseg = ipn & ~63u;
    if (nseg >= csize) return kFastFallback;  // ran off the input without a last sequence
    if (nseg == seg + 64u) {
      cur = nxt;
    } else {
      cur = seg_parse(d, nseg, lane);
    }
    seg = nseg;
    nxt = seg_parse(d, seg + 64u, lane);
  }
}
