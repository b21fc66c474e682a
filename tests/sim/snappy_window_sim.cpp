// snappy_window_sim.cpp -- host model of the windowed exact snappy fragment compressor
// (librdkafka_amd/csrc/snappy.hip, sn_window_fragment()).
//
// TEST INFRASTRUCTURE.  The HIP kernel reproduces compress_fragment's greedy parse
// (snappy.c:957-1103) in windows of 64 consecutive positions, one per lane: every lane
// measures the match its table candidate would give, and the sequential loop's path over
// those per-lane results is an orbit over the lanes (the parallel walk), with a walk that
// takes one copy at a time for the windows outside the conditions under which that shortcut
// is exact.  This file is the same algorithm with the 64 lanes as arrays and the wave
// intrinsics as loops, so the parse logic (which positions are probed and inserted, the
// ip-1 insertion and the immediate re-test after a copy, the skip schedule's hand-over to
// the probe-by-probe search, window hand-over) can be checked against the oracle on a
// machine without a GPU.  tests/test_snappy_window_sim.py compares its output byte for byte
// with oracle/snappy_oracle.c on the same inputs.
//
// Build: g++ -O2 -shared -fPIC -o libsnappywindowsim.so snappy_window_sim.cpp
#include <cstdint>
#include <cstring>

namespace {

constexpr int kRegLen = 92;     // match bytes a lane measures itself
constexpr int kStride1 = 31;    // probes 0..31 of a search step by one byte (skip++ >> 5, :1019), so
                                // probe 32 is still the next position; the windows stop there
constexpr uint32_t kMul = 0x1e35a7bdu;

struct Frag {
  const uint8_t *src;
  int n, ip_limit;
  uint8_t *dst;
  uint16_t table[1 << 14];
  int shift;
  int ip, cnt, anchor, op;
  long windows, generic, inwin, longfwd, fastwin, trunc;
};

inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint32_t hashof(const Frag &b, uint32_t seq) { return (seq * kMul) >> b.shift; }

inline int count_fwd(const Frag &b, int a, int c, int limit) {  // equal bytes, at most limit
  int k = 0;
  while (k < limit && b.src[a + k] == b.src[c + k]) ++k;
  return k;
}

enum Mode { SEARCH = 0, POSTMATCH = 1, FORCED = 2 };
enum Status { CONTINUE = 0, LAST = 1 };

inline uint64_t below(int x) { return x >= 64 ? ~0ull : x <= 0 ? 0ull : ((1ull << x) - 1ull); }
inline uint64_t range(int a, int b) { return a >= b ? 0ull : (below(b) & ~below(a)); }  // [a, b)

// bytes_between_hash_lookups after probe k of a search (skip++ >> 5, skip from 32)
inline int step_of(int k) { return (32 + k) >> 5; }

// The sequential search loop (:1015-1031) from probe index b.cnt at position b.ip.
// true with (P, cand) when a probe verifies; false = the fragment's remainder follows.
bool generic_search(Frag &b, int &P, int &cand) {
  int fwd = b.ip, k = b.cnt;
  for (;;) {
    const int cur = fwd;
    const int nxt = cur + step_of(k);
    if (nxt > b.ip_limit) return false;
    const uint32_t seq = rd32(b.src + cur);
    const uint32_t h = hashof(b, seq);
    const int m = b.table[h];
    b.table[h] = uint16_t(cur);
    if (rd32(b.src + m) == seq) {
      P = cur;
      cand = m;
      return true;
    }
    fwd = nxt;
    ++k;
  }
}

int emit_literal(uint8_t *op, const uint8_t *lit, int len) {  // snappy.c:652-695
  int n = len - 1, o = 0;
  if (n < 60) {
    op[o++] = uint8_t(n << 2);
  } else {
    const int count = n < 0x100 ? 1 : n < 0x10000 ? 2 : 3;
    op[o++] = uint8_t((59 + count) << 2);
    for (int j = 0; j < count; ++j) op[o++] = uint8_t(n >> (8 * j));
  }
  memcpy(op + o, lit, size_t(len));
  return o + len;
}
int emit_copy64(uint8_t *op, int offset, int len) {  // snappy.c:697
  if (len < 12 && offset < 2048) {
    op[0] = uint8_t(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
    op[1] = uint8_t(offset);
    return 2;
  }
  op[0] = uint8_t(2 + ((len - 1) << 2));
  op[1] = uint8_t(offset);
  op[2] = uint8_t(offset >> 8);
  return 3;
}
int emit_copy(uint8_t *op, int offset, int len) {  // snappy.c:718
  int o = 0;
  while (len >= 68) { o += emit_copy64(op + o, offset, 64); len -= 64; }
  if (len > 64) { o += emit_copy64(op + o, offset, 60); len -= 60; }
  return o + emit_copy64(op + o, offset, len);
}

// One window of 64 positions starting at w0.
Status window(Frag &b, int w0, Mode mode, int forced_cand, Mode &next_mode) {
  b.windows++;
  // ---- per-lane precomputation (vector part of the kernel)
  bool act[64], tver[64], sat[64];
  uint32_t seq[64], h[64];
  int tc[64], len[64];
  uint64_t eq[64];
  for (int l = 0; l < 64; ++l) {
    const int i = w0 + l;
    act[l] = i < b.ip_limit;  // a probe here has next_ip <= ip_limit; a re-test here has ip < ip_limit
    seq[l] = 0; h[l] = 0; tc[l] = 0; len[l] = 0; tver[l] = false; sat[l] = false;
    if (!act[l]) continue;
    seq[l] = rd32(b.src + i);
    h[l] = hashof(b, seq[l]);
    tc[l] = (mode == FORCED && l == 0) ? forced_cand : int(b.table[h[l]]);
    tver[l] = rd32(b.src + tc[l]) == seq[l];
    int lim = b.n - i;  // find_match_length stops at the end of the input (:823)
    if (lim > kRegLen) lim = kRegLen;
    len[l] = 4 + count_fwd(b, i + 4, tc[l] + 4, lim - 4);
    sat[l] = tver[l] && len[l] == kRegLen && i + kRegLen < b.n;  // length not final
  }
  for (int l = 0; l < 64; ++l) {
    eq[l] = 0;
    for (int j = 0; j < 64; ++j)
      if (act[l] && act[j] && h[j] == h[l]) eq[l] |= 1ull << j;
  }
  uint64_t VT = 0, DUP = 0, ACT = 0;
  for (int l = 0; l < 64; ++l) {
    if (act[l]) ACT |= 1ull << l;
    if (tver[l]) VT |= 1ull << l;
    if (eq[l] & below(l)) DUP |= 1ull << l;
  }
  const int NA = ~ACT ? __builtin_ctzll(~ACT) : 64;  // first lane that may not be probed

  const int anchor_in = b.anchor;
  uint64_t INS = 0, chosen = 0;
  int L_cand[64], L_len[64];
  int anchor = b.anchor, cnt = b.cnt;
  int q = 0, x = 0, cand = 0, ipn = 0;
  bool inwin = false;
  Status st = CONTINUE;
  next_mode = SEARCH;

  auto lookup = [&](int lx, int &c, bool &iw) -> bool {  // candidate of lane lx given the inserts so far
    const uint64_t m = eq[lx] & INS & below(lx);
    if (m) {
      const int j = 63 - __builtin_clzll(m);
      c = w0 + j;
      iw = true;
      return seq[j] == seq[lx];
    }
    c = tc[lx];
    iw = false;
    return (VT >> lx) & 1;
  };

  // ---- parallel walk.  Copies hop from one verified lane to the next: f(m) = first verified
  // lane at or after m + len[m]; the chosen lanes are the orbit of f from the entry.  The
  // walk is cut at the first probe whose index in its search passes kStride1 (the skip
  // schedule leaves stride 1 there); what lies before the cut is exact if every candidate
  // used is the table's and every chosen length is final.
  bool fast_done = false;
  if (NA == 64) {
    auto first_vt = [&](int from) {
      return from >= 64 ? 64 : ((VT & ~below(from)) ? __builtin_ctzll(VT & ~below(from)) : 64);
    };
    const int e = mode == POSTMATCH ? 1 : 0;
    int Jd[4][65];
    for (int l = 0; l < 64; ++l) Jd[0][l] = first_vt(l + len[l]);
    Jd[0][64] = 64;
    for (int d = 1; d < 4; ++d) {
      for (int l = 0; l < 64; ++l) Jd[d][l] = Jd[d - 1][Jd[d - 1][l]];
      Jd[d][64] = 64;
    }
    uint64_t ch = 0;
    for (int k = 0; k < 16; ++k) {  // lane k: k-th copy
      int pos = first_vt(e);
      for (int d = 0; d < 4; ++d)
        if ((k >> d) & 1) pos = Jd[d][pos];
      if (pos < 64) ch |= 1ull << pos;
    }
    uint64_t Mv = 0, Tm = 0, Rm = 0;
    int pend_of[64];
    for (int l = 0; l < 64; ++l) {
      const int i = w0 + l;
      const uint64_t lowc = ch & below(l);
      const int pl = lowc ? 63 - __builtin_clzll(lowc) : -1;
      const int pend = pl >= 0 ? w0 + pl + len[pl] : 0;
      pend_of[l] = pl >= 0 ? pend : anchor_in;
      const bool interior = pl >= 0 && pend > i;
      if (l >= e && !interior) Mv |= 1ull << l;
      if (pl >= 0 && pend == i) Tm |= 1ull << l;
      if (pl >= 0 && pend == i + 1 && pend - w0 < 64) Rm |= 1ull << l;
    }
    if (mode == POSTMATCH) { Tm |= 2; Rm |= 1; }
    // probe index of every searched lane: distance from the last re-tested lane
    uint64_t over = 0;
    for (int l = 0; l < 64; ++l) {
      if (!((Mv >> l) & 1) || ((Tm >> l) & 1)) continue;
      if (mode == FORCED && l == 0) continue;  // found by the probe-by-probe search
      const uint64_t lt = Tm & below(l);
      const int idx = lt ? l - 1 - (63 - __builtin_clzll(lt)) : b.cnt + l;
      if (idx > kStride1) over |= 1ull << l;
    }
    const int Z = over ? __builtin_ctzll(over) : 64;
    ch &= below(Z);
    const uint64_t ins = (Mv | Rm) & below(Z);
    bool ok = true;
    for (int l = 0; l < Z; ++l) {
      const int i = w0 + l;
      if ((ch >> l) & 1) {
        if (sat[l]) ok = false;                      // length not final
        if (i + len[l] >= b.ip_limit) ok = false;    // the remainder follows (:1062)
      }
      if (((Mv >> l) & 1) && (eq[l] & ins & below(l))) ok = false;  // a window-local candidate
    }
    if (ok) {
      fast_done = true;
      b.fastwin++;
      INS = ins;
      chosen = ch;
      for (int l = 0; l < 64; ++l)
        if ((ch >> l) & 1) { L_cand[l] = tc[l]; L_len[l] = len[l]; }
      const int cl = ch ? 63 - __builtin_clzll(ch) : -1;
      const int end = cl >= 0 ? cl + len[cl] : -1;  // lane after the last copy
      if (cl >= 0) anchor = w0 + end;
      if (Z < 64) {
        b.trunc++;
        b.ip = w0 + Z;
        b.cnt = kStride1 + 1;
      } else if (cl >= 0 && end >= 64) {
        b.ip = w0 + end;
        next_mode = POSTMATCH;
      } else {
        b.ip = w0 + 64;
        const uint64_t tm = Tm;
        const int tl = tm ? 63 - __builtin_clzll(tm) : -1;  // last re-tested lane
        b.cnt = tl >= 0 ? 63 - tl : b.cnt + 64;
      }
    }
  }

  if (!fast_done) {
    enum { S_SEARCH = 0, S_FOUND = 1, S_POST = 2 };
    int state = S_SEARCH;
    if (mode == POSTMATCH) {
      ipn = w0 + 1;
      state = S_POST;
    } else if (mode == FORCED) {
      x = 0;
      cand = forced_cand;
      inwin = false;
      state = S_FOUND;
    }
    for (;;) {
      if (state == S_SEARCH) {
        const int xmax = q + (kStride1 - cnt);  // last lane whose probe index is <= kStride1
        int stop = NA < 64 ? NA : 64;
        int why = NA < 64 ? 1 : 0;  // 1: remainder, 0: window end
        if (xmax + 1 <= stop) { stop = xmax + 1; why = 2; }  // 2: strides above 1 from here
        const uint64_t cm = (VT | DUP) & range(q, stop);
        if (!cm) {
          INS |= range(q, stop);
          if (why == 1) {
            st = LAST;
          } else {
            b.ip = w0 + stop;
            b.cnt = cnt + (stop - q);
          }
          break;
        }
        x = __builtin_ctzll(cm);
        INS |= range(q, x);
        const bool ver = lookup(x, cand, inwin);
        INS |= 1ull << x;
        cnt += x + 1 - q;
        q = x + 1;
        if (ver) state = S_FOUND;
      } else if (state == S_FOUND) {
        const int P = w0 + x;
        int fl;
        if (inwin) {
          b.inwin++;
          fl = count_fwd(b, P + 4, cand + 4, b.n - (P + 4));
        } else {
          fl = len[x] - 4;
          if (sat[x]) {
            b.longfwd++;
            fl += count_fwd(b, P + kRegLen, cand + kRegLen, b.n - P - kRegLen);
          }
        }
        L_cand[x] = cand;
        L_len[x] = 4 + fl;
        chosen |= 1ull << x;
        ipn = P + 4 + fl;
        anchor = ipn;
        if (ipn >= b.ip_limit) { st = LAST; break; }  // :1062
        state = S_POST;
      } else {
        const int r = ipn - 1 - w0;
        if (r + 1 >= 64) {  // the re-test position lies beyond this window
          b.ip = ipn;
          next_mode = POSTMATCH;
          break;
        }
        INS |= 1ull << r;  // table[hash(ip-1)] = ip-1 (:1071)
        x = r + 1;
        const bool ver = lookup(x, cand, inwin);
        INS |= 1ull << x;
        if (ver) {
          state = S_FOUND;
        } else {
          q = x + 1;
          cnt = 0;
          state = S_SEARCH;
        }
      }
    }
  }
  // ---- table update: every inserted lane, the latest position per hash wins
  if (st != LAST)
    for (int l = 0; l < 64; ++l)
      if (((INS >> l) & 1) && !(eq[l] & INS & ~below(l + 1))) b.table[h[l]] = uint16_t(w0 + l);
  // ---- emission of the window's elements, in lane order
  {
    int prev = anchor_in, op = b.op;
    for (int l = 0; l < 64; ++l) {
      if (!((chosen >> l) & 1)) continue;
      const int P = w0 + l;
      if (P > prev) op += emit_literal(b.dst + op, b.src + prev, P - prev);
      op += emit_copy(b.dst + op, P - L_cand[l], L_len[l]);
      prev = P + L_len[l];
    }
    b.op = op;
  }
  b.anchor = anchor;
  return st;
}

}  // namespace

// compress_fragment over src[0, n) with a zeroed table of tsize entries; returns the size
extern "C" int sim_snappy_window_fragment(const uint8_t *src, int n, uint8_t *dst, int tsize,
                                          long *stats /* 6 counters, may be null */) {
  static thread_local Frag b;
  b.src = src;
  b.n = n;
  b.dst = dst;
  b.ip_limit = n - 15;
  int lg = 0;
  while ((2 << lg) <= tsize) lg++;
  b.shift = 32 - lg;
  b.ip = 1; b.cnt = 0; b.anchor = 0; b.op = 0;
  b.windows = b.generic = b.inwin = b.longfwd = b.fastwin = b.trunc = 0;
  memset(b.table, 0, sizeof b.table);
  if (n >= 15) {
    Mode mode = SEARCH;
    int forced = 0;
    for (;;) {
      int w0;
      if (mode == SEARCH && b.cnt > kStride1) {
        b.generic++;
        int P, cand;
        if (!generic_search(b, P, cand)) break;
        mode = FORCED;
        forced = cand;
        w0 = P;
      } else {
        w0 = mode == POSTMATCH ? b.ip - 1 : b.ip;
      }
      Mode nm;
      const Status st = window(b, w0, mode, forced, nm);
      if (st == LAST) break;
      mode = nm;
    }
  }
  if (b.anchor < n) b.op += emit_literal(dst + b.op, src + b.anchor, n - b.anchor);  // :1097
  if (stats) {
    stats[0] = b.windows; stats[1] = b.generic; stats[2] = b.inwin;
    stats[3] = b.longfwd; stats[4] = b.fastwin; stats[5] = b.trunc;
  }
  return b.op;
}
