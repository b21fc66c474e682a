// lz4_host.cpp -- drop-in rd_kafka_lz4_compress / rd_kafka_lz4_decompress
// drivers: stage host bytes -> device, run the LZ4F kernels, copy the frame
// or payload back into malloc() memory.  Host work is limited to the framing
// bookkeeping the reference also does outside the codec (HC fix-up for
// MsgVersion 0, rdkafka_lz4.c:50-155; sizing the output from the block table).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "common.h"
#include "lz4_engine.h"
#define RDK_HD
#include "lz4_frame.h"

namespace rdk {

int lz4hc_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, int level, hipStream_t s);
int lz4f_compress_device(Ctx *c, const uint8_t *d_in, const uint64_t *d_in_offs,
                         const uint32_t *d_in_lens, uint8_t *d_out, const uint64_t *d_out_offs,
                         uint32_t *d_out_lens, uint32_t n, int accel, hipStream_t s,
                         const FuseCrc *fuse);
int lz4f_decompress_device(Ctx *c, const uint8_t *d_in, const uint64_t *d_in_offs,
                           const uint32_t *d_in_lens, uint8_t *d_out,
                           const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                           uint32_t *d_out_lens, int32_t *d_status, uint32_t n, hipStream_t s);
size_t lz4f_compress_bound(size_t len);

namespace {
struct HostReader {
  const uint8_t *p;
  uint32_t operator()(uint64_t i) const { return p[i]; }
};

// XXH32 of up to ~20 header bytes (LZ4F header checksum input)
uint32_t xxh32_small(const uint8_t *p, size_t len) {
  const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                 P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  auto rd = [&](size_t i) {
    return uint32_t(p[i]) | (uint32_t(p[i + 1]) << 8) | (uint32_t(p[i + 2]) << 16) |
           (uint32_t(p[i + 3]) << 24);
  };
  size_t i = 0;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0u - P1;
    for (; i + 16 <= len; i += 16) {
      v1 = rotl(v1 + rd(i) * P2, 13) * P1;
      v2 = rotl(v2 + rd(i + 4) * P2, 13) * P1;
      v3 = rotl(v3 + rd(i + 8) * P2, 13) * P1;
      v4 = rotl(v4 + rd(i + 12) * P2, 13) * P1;
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  } else {
    h = P5;
  }
  h += uint32_t(len);
  for (; i + 4 <= len; i += 4) h = rotl(h + rd(i) * P3, 17) * P4;
  for (; i < len; ++i) h = rotl(h + p[i] * P5, 11) * P1;
  h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
  return h;
}

// header byte offset of HC, or 0 when the legacy fix-up cannot apply
size_t hc_offset(const uint8_t *b, size_t len) {
  static const uint8_t magic[4] = {0x04, 0x22, 0x4d, 0x18};
  if (len < 7 || std::memcmp(b, magic, 4)) return 0;
  size_t of = 6;
  if ((b[4] >> 3) & 1u) of += 8;
  return of < len ? of : 0;
}
}  // namespace

// rd_kafka_lz4_decompress_fixup_bad_framing (rdkafka_lz4.c:50-98): recompute HC in place
int lz4f_fix_hc_in(uint8_t *in, size_t inlen) {
  const size_t of = hc_offset(in, inlen);
  if (!of) return kErrBadCompression;
  in[of] = uint8_t((xxh32_small(in + 4, of - 4) >> 8) & 0xFFu);
  return 0;
}

// rd_kafka_lz4_compress_break_framing (rdkafka_lz4.c:108-155): the legacy (wrong) HC
int lz4f_break_hc_out(uint8_t *o, size_t flen) {
  const size_t of = hc_offset(o, flen);
  if (!of) return kErrBadCompression;
  o[of] = uint8_t((xxh32_small(o, of) >> 8) & 0xFFu);
  return 0;
}

// Output capacity for one frame in host memory, from a walk of its block headers.
// Two sizings: `tight` = what the blocks can yield at most (lz4f_block_most), `slots` =
// the in-place layout of independent blocks (block k at k * max_block).  The slot layout
// is used when it costs at most 4x the tight bound (+ 1 MiB): every frame the reference's
// writer makes.  A small frame of many short blocks of a large block class would
// otherwise ask for gigabytes of staging; it gets the tight size and the device decodes
// it in stream order.  Returns 0 or the frame's error.
int lz4f_frame_capacity(const uint8_t *in, size_t inlen, uint64_t *cap_out) {
  if (inlen > 0xFFFFFFFFull) return kErrBadCompression;
  FrameWalker<HostReader> wk{HostReader{in}, inlen};
  wk.header();
  BlockInfo b;
  uint64_t tight = 0, slots = 0, last_most = 0;
  uint32_t nb = 0;
  while (wk.next(b)) {
    last_most = lz4f_block_most(b, wk.fi.max_block);
    tight += last_most;
    ++nb;
  }
  if (nb) slots = uint64_t(nb - 1) * wk.fi.max_block + last_most;
  const uint64_t cap = (slots <= 4 * tight + (1u << 20)) ? (slots > tight ? slots : tight) : tight;
  if (wk.fi.status) return wk.fi.status;
  if (cap > 0xFFFFFFF0ull) return RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE;
  *cap_out = cap;
  return 0;
}

// frames whose bound is at most this come back in the same copy as their length
constexpr size_t kOneSyncBytes = 256u << 10;

int lz4f_compress_host(Ctx *c, size_t len, int proper_hc, int level, void **out, size_t *outlen) {
  if (len > 0xFFFFFFFFull) return kErrBadCompression;
  const size_t bound = lz4f_compress_bound(len);
  const size_t in_bytes = (len + 255) & ~size_t(255);
  int rc;
  if ((rc = ensure_dev(c, 0, in_bytes + bound + 64)) || (rc = ensure_desc(c, 64))) return rc;
  uint8_t *d_in = c->d_stage[0], *d_out = c->d_stage[0] + in_bytes;
  // descriptors: in_off, out_off (u64), in_len (u32), out_len (u32)
  uint64_t *hd = reinterpret_cast<uint64_t *>(c->h_desc);
  hd[0] = 0;
  hd[1] = 0;
  reinterpret_cast<uint32_t *>(hd + 2)[0] = uint32_t(len);
  uint64_t *dd = reinterpret_cast<uint64_t *>(c->d_desc);
  uint32_t *d_len = reinterpret_cast<uint32_t *>(dd + 2), *d_olen = d_len + 1;
  if (len) RDK_HIP_CHECK(hipMemcpyAsync(d_in, c->h_stage, len, hipMemcpyHostToDevice, c->stream));
  RDK_HIP_CHECK(hipMemcpyAsync(dd, hd, 24, hipMemcpyHostToDevice, c->stream));
  const int accel = level < 0 ? -level + 1 : 1;
  if (level >= 3) {  // LZ4F_selectCompression (lz4frame.c:797-805): LZ4HC hash chain
    if ((rc = lz4hc_compress_device(d_in, dd, d_len, d_out, dd + 1, d_olen, 1, level, c->stream)))
      return rc;
  } else if ((rc = lz4f_compress_device(c, d_in, dd, d_len, d_out, dd + 1, d_olen, 1, accel,
                                        c->stream, nullptr))) {
    return rc;
  }
  RDK_HIP_CHECK(hipMemcpyAsync(c->h_desc + 32, d_olen, 4, hipMemcpyDeviceToHost, c->stream));
  // A small frame comes back whole behind its length, one synchronisation for both (the
  // staging already has room: the caller sized it for the bound); a large one waits for
  // its length first and copies only that much.
  const bool whole = bound <= kOneSyncBytes && c->h_cap >= bound;
  if (whole) RDK_HIP_CHECK(hipMemcpyAsync(c->h_stage, d_out, bound, hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  uint32_t flen;
  std::memcpy(&flen, c->h_desc + 32, 4);
  if (flen > bound) return set_error(RDK_HIP_E_HIP, "lz4f compress: frame longer than its bound");
  if (!whole) {
    if ((rc = ensure_host(c, flen))) return rc;
    RDK_HIP_CHECK(hipMemcpyAsync(c->h_stage, d_out, flen, hipMemcpyDeviceToHost, c->stream));
    RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  }
  uint8_t *o = static_cast<uint8_t *>(std::malloc(flen));
  if (!o) return RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE;
  std::memcpy(o, c->h_stage, flen);
  if (!proper_hc && (rc = lz4f_break_hc_out(o, flen))) {
    std::free(o);
    return rc;
  }
  *out = o;
  *outlen = flen;
  return 0;
}

int lz4f_decompress_host(Ctx *c, int proper_hc, uint8_t *in, size_t inlen, void **out,
                         size_t *outlen) {
  int rc;
  if (!proper_hc && (rc = lz4f_fix_hc_in(in, inlen))) return rc;
  uint64_t cap = 0;
  if ((rc = lz4f_frame_capacity(in, inlen, &cap))) return rc;
  const size_t in_bytes = (inlen + 255) & ~size_t(255);
  if ((rc = ensure_host(c, inlen > cap ? inlen : cap)) ||
      (rc = ensure_dev(c, 0, in_bytes + cap + 64)) || (rc = ensure_desc(c, 128)))
    return rc;
  uint8_t *d_in = c->d_stage[0], *d_out = c->d_stage[0] + in_bytes;
  std::memcpy(c->h_stage, in, inlen);
  // descriptors: in_off, out_off (u64) | in_len, out_cap, out_len (u32) | status (i32)
  uint64_t *hd = reinterpret_cast<uint64_t *>(c->h_desc);
  hd[0] = 0;
  hd[1] = 0;
  uint32_t *hw = reinterpret_cast<uint32_t *>(hd + 2);
  hw[0] = uint32_t(inlen);
  hw[1] = uint32_t(cap);
  uint64_t *dd = reinterpret_cast<uint64_t *>(c->d_desc);
  uint32_t *dw = reinterpret_cast<uint32_t *>(dd + 2);
  if (inlen) RDK_HIP_CHECK(hipMemcpyAsync(d_in, c->h_stage, inlen, hipMemcpyHostToDevice, c->stream));
  RDK_HIP_CHECK(hipMemcpyAsync(dd, hd, 32, hipMemcpyHostToDevice, c->stream));
  if ((rc = lz4f_decompress_device(c, d_in, dd, dw, d_out, dd + 1, dw + 1, dw + 2,
                                   reinterpret_cast<int32_t *>(dw + 3), 1, c->stream)))
    return rc;
  RDK_HIP_CHECK(hipMemcpyAsync(c->h_desc + 64, dw + 2, 8, hipMemcpyDeviceToHost, c->stream));
  // a small payload comes back whole behind its length and status (one synchronisation)
  const bool whole = cap != 0 && cap <= kOneSyncBytes;
  if (whole) RDK_HIP_CHECK(hipMemcpyAsync(c->h_stage, d_out, cap, hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  uint32_t olen;
  int32_t status;
  std::memcpy(&olen, c->h_desc + 64, 4);
  std::memcpy(&status, c->h_desc + 68, 4);
  if (status == kErrDstSize) return set_error(RDK_HIP_E_HIP, "lz4f decompress: output sizing");
  if (status) return status;
  if (olen > cap) return set_error(RDK_HIP_E_HIP, "lz4f decompress: length beyond the capacity");
  if (olen && !whole) {  // the copy first: nothing is owned yet if it fails
    RDK_HIP_CHECK(hipMemcpyAsync(c->h_stage, d_out, olen, hipMemcpyDeviceToHost, c->stream));
    RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  }
  uint8_t *o = static_cast<uint8_t *>(std::malloc(olen ? olen : 1));
  if (!o) return RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE;
  if (olen) std::memcpy(o, c->h_stage, olen);
  *out = o;
  *outlen = olen;
  return 0;
}

}  // namespace rdk
