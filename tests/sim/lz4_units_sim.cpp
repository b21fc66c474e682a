// lz4_units_sim.cpp -- host model of the throughput-mode LZ4 block compressor
// (librdkafka_amd/csrc/lz4_encode_fast.hip, one workgroup per 64 KiB block).
//
// TEST INFRASTRUCTURE.  The HIP kernel keeps a block's source and its hash table in LDS
// and splits the work between a finder wavefront and parser wavefronts.  Its result is
// defined by the sequential algorithm below, and the kernel must reproduce it byte for
// byte (tests/test_gpu_lz4.py compares them); tests/test_units_sim.py checks this model
// against the reference decoder and the reference's compression ratio without a GPU.
//
//   1. Candidates, in position order, 64 positions at a time: every position i <= n-12 is
//      hashed with LZ4_hash4 (lz4.c:631, 13-bit table as LZ4_compress_generic's byU16, lz4.c:633) and takes as its candidate the
//      table's entry as it stood before its group of 64; then the whole group is entered
//      (the highest position of a group wins an entry).
//   2. The block is cut into units of `unit_windows` x 64 positions.  A unit is parsed
//      greedily on its own, starting at its first position: the next match is the first
//      position of the unit at or after the end of the last one whose candidate verifies
//      (MINMATCH equal bytes), as long as it does (up to matchlimit = n-5, lz4.c:822, so
//      it may run past the unit's end); up to 4 catch-up bytes (lz4.c:957) are taken
//      from the literals behind the unit's start or the last match.
//   3. Units are stitched in order.  The literals that a unit leaves behind its last
//      match become part of the next unit's first sequence.  Where a match has run into
//      the following units, their sequences that it covers are dropped, and one that it
//      covers in part keeps the rest of its match (same offset) if that is MINMATCH
//      bytes or more and starts no later than n-12.  The block ends with the last
//      literals (lz4.c:1141-1166).  A block that does not fit in `cap` = n-1 bytes
//      (LZ4F_makeBlock, lz4frame.c:739-761) returns 0 and is stored raw.
//
// Build: g++ -O2 -shared -fPIC -o libunitssim.so lz4_units_sim.cpp
#include <cstdint>
#include <cstring>
#include <vector>

namespace {
constexpr int kMinMatch = 4, kLastLiterals = 5, kMFLimit = 12, kHashLog = 13;

inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint32_t hash4(uint32_t s) { return (s * 2654435761u) >> (32 - kHashLog); }

struct Seq {
  int lstart, lit, off, mlen;
};

inline int ext_bytes(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

inline void put_len(std::vector<uint8_t> &o, int v) {  // v >= 15
  v -= 15;
  while (v >= 255) {
    o.push_back(255);
    v -= 255;
  }
  o.push_back(uint8_t(v));
}
}  // namespace

extern "C" int sim_lz4_units_block(const uint8_t *src, int n, uint8_t *dst, int cap,
                                   int unit_windows, long *stats /* [4] or null */) {
  if (n < kMFLimit + 1) return 0;
  const int mfl = n - kMFLimit, mlim = n - kLastLiterals;
  std::vector<uint16_t> table(1u << kHashLog, 0);
  std::vector<int> cand(n, -1);
  for (int R = 0; R <= mfl; R += 64) {
    int c[64];
    for (int l = 0; l < 64; ++l) {
      const int i = R + l;
      c[l] = i <= mfl ? int(table[hash4(rd32(src + i))]) : -1;
    }
    for (int l = 0; l < 64; ++l) {
      const int i = R + l;
      if (i <= mfl) {
        table[hash4(rd32(src + i))] = uint16_t(i);
        cand[i] = c[l] < i ? c[l] : -1;
      }
    }
  }
  const int ulen = unit_windows * 64;
  std::vector<uint8_t> o;
  o.reserve(size_t(n) + 64);
  int carry = 0;  // start of the literals not yet written == end of the last match written
  long nseq = 0, nunits = 0, dropped = 0, trimmed = 0;
  std::vector<Seq> unit;
  for (int u0 = 0; u0 < n; u0 += ulen) {
    const int u1 = u0 + ulen < n ? u0 + ulen : n;
    // ---- the unit's own parse: starts at u0, knows nothing of the units before it; a
    // match may run past the unit's end (up to matchlimit)
    unit.clear();
    int p = u0, anchor = u0;
    ++nunits;
    for (int i = u0; i < u1; ++i) {
      if (i < p || cand[i] < 0) continue;
      const int c = cand[i];
      if (rd32(src + i) != rd32(src + c)) continue;
      int len = 0;
      while (i + len < mlim && src[i + len] == src[c + len]) ++len;
      if (len < kMinMatch) continue;
      int bk = 0;
      while (bk < 4 && i - bk > anchor && c - bk > 0 && src[i - bk - 1] == src[c - bk - 1]) ++bk;
      unit.push_back(Seq{anchor, i - bk - anchor, i - c, len + bk});
      p = anchor = i + len;
    }
    // ---- stitching: `carry` may lie inside this unit (a match of an earlier unit ran
    // into it).  Sequences whose match ends at or before carry are dropped; one that
    // straddles it keeps the part of its match from carry on (same offset), unless that is
    // under MINMATCH bytes or would start past n-12; the first sequence kept takes its
    // literals from carry.
    bool first = true;
    for (Seq s : unit) {
      int ms = s.lstart + s.lit;     // match start (catch-up included)
      const int me = ms + s.mlen;    // match end
      if (me <= carry) { ++dropped; continue; }
      if (ms < carry) {
        if (me - carry < kMinMatch || carry > mfl) { ++dropped; continue; }
        ms = carry;
        ++trimmed;
      }
      if (first) {
        s.lstart = carry;
        first = false;
      }
      s.lit = ms - s.lstart;
      s.mlen = me - ms;
      const int mc = s.mlen - kMinMatch;
      o.push_back(uint8_t(((s.lit < 15 ? s.lit : 15) << 4) | (mc < 15 ? mc : 15)));
      if (s.lit >= 15) put_len(o, s.lit);
      o.insert(o.end(), src + s.lstart, src + s.lstart + s.lit);
      o.push_back(uint8_t(s.off));
      o.push_back(uint8_t(s.off >> 8));
      if (mc >= 15) put_len(o, mc);
      carry = me;
      ++nseq;
    }
  }
  const int last = n - carry;
  o.push_back(uint8_t((last < 15 ? last : 15) << 4));
  if (last >= 15) put_len(o, last);
  o.insert(o.end(), src + carry, src + n);
  if (stats) {
    stats[0] = nseq;
    stats[1] = nunits;
    stats[2] = long(o.size());
    stats[3] = dropped * 100000 + trimmed;
  }
  if (long(o.size()) > long(cap)) return 0;
  memcpy(dst, o.data(), o.size());
  return int(o.size());
}

// Whole LZ4F frame as the engine writes it: header 04 22 4D 18 60 40 82, 64 KiB blocks
// (size word, bit 31 = stored raw), end mark.
extern "C" long sim_lz4_units_frame(const uint8_t *src, long n, uint8_t *dst, int unit_windows) {
  static const uint8_t hdr[7] = {0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82};
  long op = 7;
  memcpy(dst, hdr, 7);
  std::vector<uint8_t> tmp(65536 + 64);
  for (long at = 0; at < n; at += 65536) {
    const int bn = int(n - at < 65536 ? n - at : 65536);
    const int cs = sim_lz4_units_block(src + at, bn, tmp.data(), bn - 1, unit_windows, nullptr);
    const uint32_t w = cs ? uint32_t(cs) : (uint32_t(bn) | 0x80000000u);
    memcpy(dst + op, &w, 4);
    op += 4;
    if (cs) memcpy(dst + op, tmp.data(), cs);
    else memcpy(dst + op, src + at, bn);
    op += cs ? cs : bn;
  }
  memset(dst + op, 0, 4);
  return op + 4;
}
