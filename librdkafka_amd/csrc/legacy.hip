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
// One 512-thread workgroup per MessageSet finds the messages with the speculative parallel
// walk of specwalk.h (message p is [p, p + 12 + MessageSize)); each verified thread then
// computes the CRC-32 of its own messages from the LDS window (slicing-by-8).  A message
// larger than the window is computed by the whole workgroup from global memory
// (per-thread chunks combined with x^(8n) mod P shifts).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "common.h"
#include "specwalk.h"

namespace rdk {
namespace {

using namespace spec;

// MsgVersion 0/1 message format for spec::walk
struct V01 {
  // rdkafka_msgset_reader.c:566-600
  __device__ __forceinline__ uint32_t classify(const Win &W, uint32_t p, uint32_t &next) const {
    if (p == W.len) return kDone;
    const uint32_t R = W.len - p;
    if (R < 16u) return kPartial;                     // Offset, MessageSize, Crc :566-570
    if (p + 16u > W.end) return kCut;
    const int32_t s = int32_t(W.be32(p + 8u));
    if (s < 4) return kErr;  // (MessageSize - 4 wraps: rd_slice_narrow_copy asserts, rdbuf.c:1027)
    if (uint32_t(s) - 4u > R - 16u) return kPartial;  // narrow_copy / check_len :571-573
    if (R < 18u) return kPartial;                     // MagicByte, Attributes :575-576
    if (p + 18u > W.end) return kCut;
    uint32_t hdr = 6u;
    if (W.b(p + 16u) == 1u) {                         // MsgVersion 1: Timestamp :578-580
      if (R < 26u) return kPartial;
      hdr = 14u;
    }
    if (uint32_t(s) < hdr) return kErr;               // MessageSize < hdrsize :590-597
    if (p + 12u + uint32_t(s) > W.end) return kCut;   // not whole in the window
    next = p + 12u + uint32_t(s);
    return kOk;
  }
  // heuristic message-start test: never decides a result.  Branch-free in two rounds of
  // independent LDS loads (the candidate's fields, then the ones their values point at).
  __device__ __forceinline__ bool plausible(const Win &W, uint32_t q) const {
    const uint32_t len = W.len;
    if (q + 34u > W.end) return false;
    // first gather: Offset, MessageSize, MagicByte/Attributes, KeyLength (v0 at +18, v1 at +26)
    const uint32_t o1h = W.be32(q), o1l = W.be32(q + 4u), S = W.be32(q + 8u);
    const uint32_t h = W.be32(q + 16u), k0 = W.be32(q + 18u), k1 = W.be32(q + 26u);
    const uint32_t m = h >> 24, a = (h >> 16) & 0xffu, hdr = m ? 14u : 6u;
    bool ok = m <= 1u && !(a & 0xf0u) && (a & 7u) <= 4u && S >= hdr + 8u &&
              S <= len - q - 12u;
    const int32_t kl = int32_t(m ? k1 : k0);
    ok = ok && kl >= -1 && (kl <= 0 || uint32_t(kl) <= S - hdr - 8u);
    const uint32_t kb = kl > 0 ? uint32_t(kl) : 0u;
    const uint32_t r = q + 12u + S;
    const bool at_end = r == len;
    ok = ok && (at_end || r + 28u <= W.end);  // the next header must be staged too
    // second gather: ValueLength, the next message's Offset, MessageSize, MagicByte
    const uint32_t va = ok ? q + 16u + hdr + kb : q, ra = ok && !at_end ? r : q;
    const int32_t vl = int32_t(W.be32(va));
    const uint32_t o2h = W.be32(ra), o2l = W.be32(ra + 4u), S2 = W.be32(ra + 8u);
    const uint32_t m2 = W.b(ra + 16u);
    // Key and Value length fields fill the message exactly (:630-637)
    ok = ok && vl >= -1 && hdr + 8u + kb + (vl > 0 ? uint32_t(vl) : 0u) == S;
    if (at_end) return ok;
    const uint64_t o1 = (uint64_t(o1h) << 32) | o1l, o2 = (uint64_t(o2h) << 32) | o2l;
    return ok && m2 <= 1u && S2 >= (m2 ? 14u : 6u) && S2 <= len - r - 12u &&
           int64_t(o2 - o1) > 0 && o2 - o1 < (uint64_t(1) << 32);  // Offsets increase
  }
  // prefilter: bytes q, q+1 (Offset's top bytes: offsets < 2^48), q+8 (MessageSize's top
  // byte: < 16 MiB), q+16 (MagicByte <= 1) and q+17 (Attributes < 8) of candidates
  // i+4k..i+4k+3
  __device__ __forceinline__ uint32_t scan(const Win &W, uint32_t s0, uint32_t lim) const {
    auto pre = [](const uint32_t *D, int k) {
      return zb(D[k]) & zb(__builtin_amdgcn_alignbyte(D[k + 1], D[k], 1u)) & zb(D[k + 2]) &
             zb(D[k + 4] & 0xfefefefeu) &
             zb(__builtin_amdgcn_alignbyte(D[k + 5], D[k + 4], 1u) & 0xf8f8f8f8u);
    };
    return spec::scan(W, s0, lim, pre, [&](uint32_t q) { return plausible(W, q); });
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

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void v01_crc_kernel(
    uint8_t *__restrict__ sbase, const uint64_t *__restrict__ set_offs,
    const uint32_t *__restrict__ set_lens, const uint64_t *__restrict__ row_offs,
    const uint32_t *__restrict__ row_caps, uint32_t *__restrict__ msg_pos,
    uint32_t *__restrict__ msg_out, int32_t *__restrict__ count,
    const uint32_t *__restrict__ gtab, const uint32_t *__restrict__ x2n) {
  __shared__ Shared S;
  __shared__ uint32_t T_s[2048];
  __shared__ uint32_t red_s[kWaves];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  for (uint32_t i = t; i < 2048u; i += kThreads) T_s[i] = gtab[i];  // slicing tables 0..7
  const lds_w *T = (const lds_w *)T_s;
  const uint32_t si = blockIdx.x;
  uint8_t *set = sbase + set_offs[si];
  const uint64_t row0 = row_offs[si];
  const uint32_t cap = row_caps[si];
  auto out_row = [&](uint32_t r, uint32_t p, uint32_t crc, uint32_t stored) {
    msg_pos[row0 + r] = p;
    if (MODE == RDK_HIP_V2_CRC_VERIFY) {
      msg_out[row0 + r] = stored == crc ? 0u : 1u;  // :602-628
    } else {
      msg_out[row0 + r] = crc;
      if (MODE == RDK_HIP_V2_CRC_FINALIZE) put_be32(set + p + 12u, crc);  // :640-641
    }
  };
  // a verified thread's k messages from c: CRC-32 of [16, 12+MessageSize) from LDS
  auto emit = [&](const Win &W, uint32_t c, uint32_t k, uint32_t rb) -> uint32_t {
    uint32_t p = c;
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t Sz = W.be32(p + 8u);
      if (rb + i < cap)
        out_row(rb + i, p, ~crc_lds(W.w - W.base, p + 16u, p + 12u + Sz, 0xffffffffu, T),
                W.be32(p + 12u));
      p += 12u + Sz;
    }
    return kNone;
  };
  // a message larger than the window: per-thread chunks from global memory, virtual zero
  // bytes in front so all chunks have one length C, combined with x^(8n) mod P shifts
  auto big = [&](const Win &W, uint32_t base, uint32_t row, uint32_t &next) -> bool {
    const uint32_t Sz = W.be32(base + 8u);
    const uint8_t *p0 = set + base + 16u;
    const uint64_t L = uint64_t(Sz) - 4u;
    const uint64_t C = ((L + kThreads - 1) / kThreads + 3u) & ~uint64_t(3);
    const uint64_t pad = C * kThreads - L;
    const uint64_t vs = uint64_t(t) * C, ve = vs + C;
    uint32_t term = 0;
    if (ve > pad) {
      const uint64_t rs0 = vs > pad ? vs - pad : 0, re0 = ve - pad;
      const uint32_t r = crc_gbl(p0 + rs0, p0 + re0, rs0 == 0 ? 0xffffffffu : 0u, T);
      term = mulp(xpow8(uint64_t(kThreads - 1u - t) * C, x2n), r);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) term ^= __shfl_xor(term, d);
    if (lane == 0) red_s[wv] = term;
    __syncthreads();
    uint32_t acc = 0;
    for (uint32_t w = 0; w < uint32_t(kWaves); ++w) acc ^= red_s[w];
    __syncthreads();
    if (t == 0) out_row(row, base, ~acc, W.be32(base + 12u));
    next = base + 12u + Sz;
    return true;
  };
  const int32_t res = walk(set, set_lens[si], cap, S, V01(), emit, big);
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
  hipLaunchKernelGGL(v01_crc_kernel<M>, dim3(n), dim3(kThreads), 0, s, b, d_set_offs,   \
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
