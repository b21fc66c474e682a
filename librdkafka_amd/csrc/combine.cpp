// combine.cpp -- see combine.h.  Host code only: the queue, the one-request path (a request
// served alone) and the batch path (several requests, one staging copy, one launch per batch
// kernel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "combine.h"
#include "crc32c_tables.h"
#include "lz4_engine.h"

namespace rdk {

int crc_device_buffer(Ctx *c, const uint8_t *d_buf, uint64_t len, uint32_t init,
                      uint32_t *d_scratch, hipStream_t s, int kind, uint32_t *d_final);
uint32_t crc_scratch_words(uint64_t len);
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
int lz4f_fix_hc_in(uint8_t *in, size_t inlen);
int lz4f_break_hc_out(uint8_t *o, size_t flen);
int lz4f_frame_capacity(const uint8_t *in, size_t inlen, uint64_t *cap_out);

namespace {

constexpr int kErrDstSizeStatus = RDK_HIP_LZ4F_E_DSTSIZE;
constexpr size_t kCrcPiece = 4096;  // a CRC request goes to the ranges kernel in pieces

std::atomic<uint64_t> g_host_crcs{0};
// [0] batches of two or more requests, [1] requests served in them, [2] the largest batch,
// [3] batches that fell back to one request at a time after a device error
std::atomic<uint64_t> g_stat[4];

struct HostCrc {
  uint32_t tab[2][256];
  uint32_t x2n[2][64];
  HostCrc() {
    std::vector<uint32_t> image(kCrcTableWords);
    for (int kind = 0; kind < 2; ++kind) {
      const uint32_t poly = kind == kCrcKind32 ? kCrc32Poly : kCrcPoly;
      crc_build_tables(image.data(), poly);  // table 0 is the plain byte table
      std::memcpy(tab[kind], image.data(), sizeof tab[kind]);
      crc_build_x2n(x2n[kind], poly);
    }
  }
};
const HostCrc &host_crc() {
  static const HostCrc h;
  return h;
}
uint32_t poly_of(int kind) { return kind == kCrcKind32 ? kCrc32Poly : kCrcPoly; }

// Byte-at-a-time CRC over host bytes.  Only the CRC symbols' last resort uses it.
uint32_t crc_host_bytes(const uint8_t *p, size_t len, uint32_t init, int kind) {
  const uint32_t *tab = host_crc().tab[kind];
  uint32_t c = ~init;
  for (size_t i = 0; i < len; ++i) c = tab[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return ~c;
}

uint32_t crc_host_segs(const Req &r, int kind) {
  uint32_t crc = r.init;
  for (size_t i = 0; i < r.nseg; ++i) crc = crc_host_bytes(r.segs[i].p, r.segs[i].n, crc, kind);
  return crc;
}

void count_host_crc(const char *who, const char *why) {
  if (!g_host_crcs.fetch_add(1))
    fprintf(stderr, "librdkafka_hip: %s: %s (%s); this call's checksum is computed on the host "
                    "(counted in rdk_hip_dropin_host_crcs)\n", who, why, last_error());
  (void)hipGetLastError();
}

void gather(uint8_t *dst, const Req &r) {
  for (size_t i = 0; i < r.nseg; ++i) {
    if (r.segs[i].n) std::memcpy(dst, r.segs[i].p, r.segs[i].n);
    dst += r.segs[i].n;
  }
}

// ------------------------------------------------------------------ one request
// CRC32C (kind kCrcKind32C) or CRC-32 (kCrcKind32) of `len` bytes gathered in c->h_stage
int crc_staged(Ctx *c, size_t len, uint32_t init, uint32_t *out, int kind) {
  const uint32_t words = crc_scratch_words(len);
  int rc;
  if ((rc = ensure_desc(c, size_t(words) * 4))) return rc;
  if (c->dh_stage && c->dh_desc) {
    // the kernels read the mapped staging in place (one pass over PCIe, no copy command to
    // wait for) and leave the CRC in the mapped result word: launch, synchronise, done
    if ((rc = crc_device_buffer(c, c->dh_stage, len, init, reinterpret_cast<uint32_t *>(c->d_desc),
                                c->stream, kind, reinterpret_cast<uint32_t *>(c->dh_desc))))
      return rc;
    RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
    std::memcpy(out, c->h_desc, 4);
    return 0;
  }
  if ((rc = ensure_dev(c, 0, len + 64))) return rc;
  if (len) RDK_HIP_CHECK(hipMemcpyAsync(c->d_stage[0], c->h_stage, len, hipMemcpyHostToDevice, c->stream));
  if ((rc = crc_device_buffer(c, c->d_stage[0], len, init,
                              reinterpret_cast<uint32_t *>(c->d_desc), c->stream, kind, nullptr)))
    return rc;
  RDK_HIP_CHECK(hipMemcpyAsync(c->h_desc, c->d_desc + size_t(words - 1) * 4, 4,
                               hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  std::memcpy(out, c->h_desc, 4);
  return 0;
}

// The CRC symbols return the checksum itself, so they have no way to report a device
// error: a failed attempt is retried once after draining the device (a transient
// allocation or launch failure).  If that fails too, or the pinned staging cannot be had,
// the checksum of THIS call is finished on the host from the caller's bytes -- reported
// on stderr the first time and counted (rdk_hip_dropin_host_crcs) -- because neither a
// wrong CRC nor taking the producer down is acceptable for a per-call device error.  A
// process with no usable gfx950 device never gets here: the symbols stop it first.
void serve_crc(Ctx *c, Req &r) {
  const int kind = r.kind == kReqCrc32 ? kCrcKind32 : kCrcKind32C;
  if (r.total == 0) {  // pre/post inversions cancel (crc32c.c:102,133)
    r.crc = r.init;
    return;
  }
  if (ensure_host(c, r.total)) {
    count_host_crc(r.who, "no pinned staging");
    r.crc = crc_host_segs(r, kind);
    return;
  }
  gather(c->h_stage, r);
  if (crc_staged(c, r.total, r.init, &r.crc, kind) == 0) return;
  fprintf(stderr, "librdkafka_hip: %s: %s; retrying\n", r.who, last_error());
  (void)hipDeviceSynchronize();
  (void)hipGetLastError();
  if (crc_staged(c, r.total, r.init, &r.crc, kind) == 0) return;
  count_host_crc(r.who, "device path failed twice");
  r.crc = crc_host_segs(r, kind);
}

// staging for a compress request served alone: the input, and the whole bound when that is
// small enough for lz4f_compress_host to fetch the frame together with its length
size_t compress_staging(size_t total) {
  const size_t bound = lz4f_compress_bound(total);
  return bound <= (size_t(256) << 10) ? bound : (total ? total : 1);
}

void keep_error(Req &r) {
  if (r.rc) snprintf(r.err, sizeof r.err, "%s", last_error());
}

void serve_one(Ctx *c, Req &r) {
  switch (r.kind) {
    case kReqCrc32c:
    case kReqCrc32:
      serve_crc(c, r);
      return;
    case kReqLz4Compress:
      // (room for a small frame's bound: it comes back in one copy with its length)
      if ((r.rc = ensure_host(c, compress_staging(r.total))) == 0) {
        gather(c->h_stage, r);  // the rdkafka_lz4.c:390 loop, gathered
        r.rc = lz4f_compress_host(c, r.total, r.proper_hc, r.level, &r.out, &r.outlen);
      }
      keep_error(r);
      return;
    default:  // one contiguous frame; the legacy HC fix-up was done by the owner
      r.rc = lz4f_decompress_host(c, 1, const_cast<uint8_t *>(r.segs[0].p), r.segs[0].n, &r.out,
                                  &r.outlen);
      keep_error(r);
      return;
  }
}

// ------------------------------------------------------------------ several requests
inline size_t up(size_t v, size_t a) { return (v + a - 1) & ~(a - 1); }

struct Item {
  Req *r;
  size_t in_off = 0;       // from the device base
  size_t out_off = 0;
  uint64_t out_cap = 0;
  uint32_t first = 0;      // CRC kinds: first piece; LZ4 kinds: row in the kind's arrays
  uint32_t pieces = 0;
  bool on_device = false;  // false: finished (or failed) in the planning pass
};

int level_key(const Req &r) {  // requests that one launch can serve share a key
  if (r.kind != kReqLz4Compress) return 0;
  return r.level < 0 ? r.level : (r.level < 3 ? 0 : r.level);
}

// One staging copy, one launch of each batch kernel that the batch needs, one copy back.
// Returns non-zero when a device step failed before any result was handed out: the caller
// then serves the requests one at a time (which retries and reports per request).
int serve_many(Ctx *c, std::vector<Req *> &batch) {
  std::stable_sort(batch.begin(), batch.end(), [](const Req *a, const Req *b) {
    return a->kind != b->kind ? a->kind < b->kind : level_key(*a) < level_key(*b);
  });
  std::vector<Item> items(batch.size());
  uint32_t npiece[2] = {0, 0}, nlz = 0, ndz = 0;
  size_t in_bytes = 0, out_bytes = 0;
  for (size_t i = 0; i < batch.size(); ++i) {
    Item &it = items[i];
    Req &r = *batch[i];
    it.r = &r;
    switch (r.kind) {
      case kReqCrc32c:
      case kReqCrc32:
        if (r.total == 0) {
          r.crc = r.init;
          break;
        }
        if (r.total > 0xFFFFFFFFull) return set_error(RDK_HIP_E_INVAL, "crc request too large for a batch");
        it.on_device = true;
        it.pieces = uint32_t((r.total + kCrcPiece - 1) / kCrcPiece);
        it.first = npiece[r.kind];
        npiece[r.kind] += it.pieces;
        break;
      case kReqLz4Compress:
        if (r.total > 0xFFFFFFFFull) {
          r.rc = RDK_HIP_RESP_ERR__BAD_COMPRESSION;
          break;
        }
        it.on_device = true;
        it.out_cap = lz4f_compress_bound(r.total);
        it.first = nlz++;
        break;
      default:
        if ((r.rc = lz4f_frame_capacity(r.segs[0].p, r.segs[0].n, &it.out_cap))) {
          keep_error(r);
          break;
        }
        it.on_device = true;
        it.first = ndz++;
        break;
    }
    if (!it.on_device) continue;
    in_bytes += up(r.total + 64, 256);
    out_bytes += up(size_t(it.out_cap) + 64, 256);
  }
  const uint32_t npieces = npiece[0] + npiece[1];
  if (!npieces && !nlz && !ndz) return 0;
  // descriptor block, in front of the inputs (one copy takes both to the device):
  //   u64 piece_off[npieces] lz_in[nlz] lz_out[nlz] dz_in[ndz] dz_out[ndz]
  //   u32 piece_len[npieces] lz_len[nlz] dz_len[ndz] dz_cap[ndz]
  //   u32 results: piece_crc[npieces] lz_out_len[nlz] dz_out_len[ndz] dz_status[ndz]
  const size_t n64 = size_t(npieces) + 2 * size_t(nlz) + 2 * size_t(ndz);
  const size_t n32 = size_t(npieces) + nlz + 2 * size_t(ndz);
  const size_t nres = size_t(npieces) + nlz + 2 * size_t(ndz);
  const size_t res_at = n64 * 8 + n32 * 4;
  const size_t desc_bytes = up(res_at + nres * 4, 256);
  // a small output region comes back whole in the same round trip as the result words; a
  // large one is fetched frame by frame, at its real length, once the lengths are known
  const bool whole = out_bytes != 0 && out_bytes <= (size_t(512) << 10);
  int rc;
  if ((rc = ensure_host(c, desc_bytes + in_bytes + (whole ? out_bytes : 0))) ||
      (rc = ensure_dev(c, 0, desc_bytes + in_bytes + out_bytes + 64)))
    return rc;
  // A batch of CRC requests alone never leaves the mapped staging: the ranges kernel reads
  // descriptors and bytes in place and writes the pieces' CRCs into the result words.
  const bool in_place = !nlz && !ndz && c->dh_stage != nullptr;
  uint8_t *h = c->h_stage, *d = in_place ? c->dh_stage : c->d_stage[0];
  uint64_t *h_piece_off = reinterpret_cast<uint64_t *>(h);
  uint64_t *h_lz_in = h_piece_off + npieces, *h_lz_out = h_lz_in + nlz;
  uint64_t *h_dz_in = h_lz_out + nlz, *h_dz_out = h_dz_in + ndz;
  uint32_t *h_piece_len = reinterpret_cast<uint32_t *>(h + n64 * 8);
  uint32_t *h_lz_len = h_piece_len + npieces, *h_dz_len = h_lz_len + nlz, *h_dz_cap = h_dz_len + ndz;
  size_t in_at = desc_bytes, out_at = desc_bytes + in_bytes;
  for (Item &it : items) {
    if (!it.on_device) continue;
    Req &r = *it.r;
    it.in_off = in_at;
    it.out_off = out_at;
    gather(h + in_at, r);
    if (r.kind <= kReqCrc32) {
      const uint32_t base = (r.kind == kReqCrc32 ? npiece[0] : 0u) + it.first;
      for (uint32_t k = 0; k < it.pieces; ++k) {
        const size_t at = size_t(k) * kCrcPiece;
        h_piece_off[base + k] = in_at + at;
        h_piece_len[base + k] = uint32_t(std::min(kCrcPiece, r.total - at));
      }
    } else if (r.kind == kReqLz4Compress) {
      h_lz_in[it.first] = in_at;
      h_lz_out[it.first] = out_at;
      h_lz_len[it.first] = uint32_t(r.total);
    } else {
      h_dz_in[it.first] = in_at;
      h_dz_out[it.first] = out_at;
      h_dz_len[it.first] = uint32_t(r.total);
      h_dz_cap[it.first] = uint32_t(it.out_cap);
    }
    in_at += up(r.total + 64, 256);
    out_at += up(size_t(it.out_cap) + 64, 256);
  }
  hipStream_t s = c->stream;
  if (!in_place) RDK_HIP_CHECK(hipMemcpyAsync(d, h, desc_bytes + in_bytes, hipMemcpyHostToDevice, s));
  const uint64_t *d_piece_off = reinterpret_cast<const uint64_t *>(d);
  const uint64_t *d_lz_in = d_piece_off + npieces, *d_lz_out = d_lz_in + nlz;
  const uint64_t *d_dz_in = d_lz_out + nlz, *d_dz_out = d_dz_in + ndz;
  const uint32_t *d_piece_len = reinterpret_cast<const uint32_t *>(d + n64 * 8);
  const uint32_t *d_lz_len = d_piece_len + npieces, *d_dz_len = d_lz_len + nlz, *d_dz_cap = d_dz_len + ndz;
  uint32_t *d_res = reinterpret_cast<uint32_t *>(d + res_at);
  uint32_t *d_piece_crc = d_res, *d_lz_olen = d_res + npieces, *d_dz_olen = d_lz_olen + nlz;
  int32_t *d_dz_status = reinterpret_cast<int32_t *>(d_dz_olen + ndz);
  if (npiece[0] &&
      (rc = rdk_hip_crc32c_ranges(d, d_piece_off, d_piece_len, nullptr, d_piece_crc, npiece[0], s)))
    return rc;
  if (npiece[1] && (rc = rdk_hip_crc32_ranges(d, d_piece_off + npiece[0], d_piece_len + npiece[0],
                                              nullptr, d_piece_crc + npiece[0], npiece[1], s)))
    return rc;
  // compress requests are sorted by level key: one launch per run of equal keys
  for (size_t i = 0; i < items.size();) {
    if (!items[i].on_device || items[i].r->kind != kReqLz4Compress) {
      ++i;
      continue;
    }
    size_t j = i;
    uint32_t rows = 0;
    const int key = level_key(*items[i].r);
    for (; j < items.size() && items[j].r->kind == kReqLz4Compress && level_key(*items[j].r) == key; ++j)
      if (items[j].on_device) ++rows;
    uint32_t row0 = ~0u;
    for (size_t k = i; k < j; ++k)
      if (items[k].on_device && items[k].first < row0) row0 = items[k].first;
    if (rows) {
      const int level = items[i].r->level;
      if (level >= 3)  // LZ4F_selectCompression (lz4frame.c:797-805): LZ4HC
        rc = lz4hc_compress_device(d, d_lz_in + row0, d_lz_len + row0, d, d_lz_out + row0,
                                   d_lz_olen + row0, rows, level, s);
      else
        rc = lz4f_compress_device(c, d, d_lz_in + row0, d_lz_len + row0, d, d_lz_out + row0,
                                  d_lz_olen + row0, rows, level < 0 ? -level + 1 : 1, s, nullptr);
      if (rc) return rc;
    }
    i = j;
  }
  if (ndz && (rc = lz4f_decompress_device(c, d, d_dz_in, d_dz_len, d, d_dz_out, d_dz_cap, d_dz_olen,
                                          d_dz_status, ndz, s)))
    return rc;
  std::vector<uint32_t> res(nres);
  if (!in_place) RDK_HIP_CHECK(hipMemcpyAsync(h + res_at, d_res, nres * 4, hipMemcpyDeviceToHost, s));
  if (whole)
    RDK_HIP_CHECK(hipMemcpyAsync(h + desc_bytes + in_bytes, d + desc_bytes + in_bytes, out_bytes,
                                 hipMemcpyDeviceToHost, s));
  RDK_HIP_CHECK(hipStreamSynchronize(s));
  std::memcpy(res.data(), h + res_at, nres * 4);
  const uint32_t *lz_olen = res.data() + npieces, *dz_olen = lz_olen + nlz;
  const int32_t *dz_status = reinterpret_cast<const int32_t *>(dz_olen + ndz);
  // the frames / payloads come back packed; the staging may be re-made for them (the
  // inputs in it are no longer needed)
  size_t back = 0;
  for (Item &it : items) {
    if (!it.on_device || it.r->kind <= kReqCrc32) continue;
    Req &r = *it.r;
    if (r.kind == kReqLz4Compress) {
      r.outlen = lz_olen[it.first];
      if (r.outlen > it.out_cap) return set_error(RDK_HIP_E_HIP, "lz4f compress: frame longer than its bound");
    } else if (dz_status[it.first] == kErrDstSizeStatus) {
      return set_error(RDK_HIP_E_HIP, "lz4f decompress: output sizing");
    } else if (dz_status[it.first] != 0) {
      r.outlen = 0;  // the frame's own verdict: nothing to copy back
    } else {
      r.outlen = dz_olen[it.first];
      if (r.outlen > it.out_cap) return set_error(RDK_HIP_E_HIP, "lz4f decompress: length beyond the capacity");
    }
    back += up(r.outlen, 64);
  }
  if (back && !whole) {
    if ((rc = ensure_host(c, back))) return rc;
    h = c->h_stage;
    size_t at = 0;
    for (Item &it : items) {
      if (!it.on_device || it.r->kind <= kReqCrc32) continue;
      if (it.r->outlen)
        RDK_HIP_CHECK(hipMemcpyAsync(h + at, d + it.out_off, it.r->outlen, hipMemcpyDeviceToHost, s));
      at += up(it.r->outlen, 64);
    }
    RDK_HIP_CHECK(hipStreamSynchronize(s));
  }
  // from here on nothing can fail for the batch as a whole: hand the results out
  const HostCrc &hc = host_crc();
  size_t at = 0;
  for (Item &it : items) {
    if (!it.on_device) continue;
    Req &r = *it.r;
    if (r.kind <= kReqCrc32) {
      const int kind = r.kind == kReqCrc32 ? kCrcKind32 : kCrcKind32C;
      const uint32_t poly = poly_of(kind);
      const uint32_t *pc = res.data() + (r.kind == kReqCrc32 ? npiece[0] : 0u) + it.first;
      const uint32_t whole = crc_x_pow_bytes(hc.x2n[kind], kCrcPiece, poly);
      uint32_t acc = 0;
      for (uint32_t k = 0; k < it.pieces; ++k) {
        const size_t len = std::min(kCrcPiece, r.total - size_t(k) * kCrcPiece);
        const uint32_t xp = len == kCrcPiece ? whole : crc_x_pow_bytes(hc.x2n[kind], len, poly);
        acc = crc_multmodp(acc, xp, poly) ^ pc[k];
      }
      if (r.init) acc ^= crc_multmodp(r.init, crc_x_pow_bytes(hc.x2n[kind], r.total, poly), poly);
      r.crc = acc;
      continue;
    }
    const size_t here = whole ? it.out_off : at;  // whole: the device layout, mirrored
    at += up(r.outlen, 64);
    if (r.kind == kReqLz4Decompress && dz_status[it.first] != 0) {
      r.rc = dz_status[it.first];
      r.outlen = 0;
      snprintf(r.err, sizeof r.err, "lz4f decompress: frame status %d", r.rc);
      continue;
    }
    uint8_t *o = static_cast<uint8_t *>(std::malloc(r.outlen ? r.outlen : 1));
    if (!o) {
      r.rc = RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE;
      r.outlen = 0;
      continue;
    }
    if (r.outlen) std::memcpy(o, h + here, r.outlen);
    if (r.kind == kReqLz4Compress && !r.proper_hc && (r.rc = lz4f_break_hc_out(o, r.outlen))) {
      std::free(o);
      r.outlen = 0;
      continue;
    }
    r.out = o;
  }
  return 0;
}

void serve(Ctx *c, std::vector<Req *> &batch) {
  if (batch.size() == 1) {
    serve_one(c, *batch[0]);
    return;
  }
  g_stat[0]++;
  g_stat[1] += batch.size();
  uint64_t m = g_stat[2].load();
  while (batch.size() > m && !g_stat[2].compare_exchange_weak(m, batch.size())) {
  }
  if (serve_many(c, batch) == 0) return;
  // a device step failed: drain, then every request on its own (each retries and reports
  // by its own rules)
  g_stat[3]++;
  (void)hipDeviceSynchronize();
  (void)hipGetLastError();
  for (Req *r : batch) {
    r->rc = 0;
    r->out = nullptr;
    r->outlen = 0;
    serve_one(c, *r);
  }
}

// ------------------------------------------------------------------ the queue
std::mutex g_mu;
std::condition_variable g_cv;
std::vector<Req *> g_pending;      // under g_mu
bool g_leader = false;             // under g_mu: a batch is being served
size_t g_expect = 1;               // under g_mu: size of the last batch
std::atomic<size_t> g_npending{0};

// RDK_HIP_COMBINE=0: every call goes to the device on its own, on its thread's stream.
bool combine_enabled() {
  static const bool on = [] {
    const char *e = getenv("RDK_HIP_COMBINE");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// The rendezvous bound in microseconds (RDK_HIP_COMBINE_WAIT_US, default 50, far below
// linger.ms = 0.5 ms, rdkafka_conf.c:1095): a thread about to serve fewer requests than the
// previous batch held waits at most this long for the rest to arrive.  A lone caller
// follows a batch of one and never waits.
unsigned wait_us() {
  static const unsigned us = [] {
    const char *e = getenv("RDK_HIP_COMBINE_WAIT_US");
    return e ? unsigned(strtoul(e, nullptr, 10)) : 50u;
  }();
  return us;
}

}  // namespace

uint64_t combine_host_crcs() { return g_host_crcs.load(); }

// A large CRC or decompress request is mostly host copies (gather, result) and PCIe time:
// those run in parallel on the callers' own threads and streams, but one after the other
// in a batch.  Measured with 8 threads at 1 MiB: 27 us (own streams) against 57 us
// (batched) per crc32c call, 212 against 445 us per decompress; at 64 KiB and below the
// batch wins.  Compress requests gain at every size (the block kernel's latency dominates).
constexpr size_t kCombineMaxBytes = 128u << 10;

void combine_submit(Ctx *c, Req *r) {
  if (!combine_enabled() || (r->kind != kReqLz4Compress && r->total > kCombineMaxBytes)) {
    serve_one(c, *r);
    return;
  }
  std::vector<Req *> batch;
  std::unique_lock<std::mutex> lk(g_mu);
  g_pending.push_back(r);
  g_npending.store(g_pending.size(), std::memory_order_release);
  while (!r->done) {
    if (g_leader) {
      g_cv.wait(lk);
      continue;
    }
    g_leader = true;  // r is still queued: whoever took it would have finished it
    if (g_pending.size() < g_expect && wait_us()) {
      const size_t want = g_expect;
      lk.unlock();
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(wait_us());
      while (g_npending.load(std::memory_order_acquire) < want &&
             std::chrono::steady_clock::now() < until)
        __builtin_ia32_pause();
      lk.lock();
    }
    batch.clear();
    batch.swap(g_pending);
    g_npending.store(0, std::memory_order_release);
    g_expect = batch.size();
    lk.unlock();
    serve(c, batch);
    lk.lock();
    for (Req *b : batch) b->done = true;
    g_leader = false;
    g_cv.notify_all();
  }
}

}  // namespace rdk

// [0] batches of two or more requests, [1] requests served in them, [2] the largest batch,
// [3] batches that fell back to one request at a time after a device error
RDK_API void rdk_hip_dropin_combined(uint64_t out[4]) {
  for (int i = 0; i < 4; ++i) out[i] = rdk::g_stat[i].load();
}
