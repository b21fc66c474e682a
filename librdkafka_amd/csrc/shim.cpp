// shim.cpp -- the drop-in symbols (see include/librdkafka_hip.h).
//
// Each call gathers its input (an rd_slice_t segment list or a contiguous
// buffer) into the calling thread's pinned staging buffer, copies it to the
// device, runs the gfx950 kernels on the thread's own stream and copies the
// result back into malloc() memory owned by the caller -- the ownership
// contract of rdkafka_lz4.c (rd_free == free, rd.h:104-119).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"
#include "crc32c_tables.h"
#include "lz4_engine.h"
#include "rdbuf_abi.h"

namespace rdk {
int crc_device_buffer(Ctx *c, const uint8_t *d_buf, uint64_t len, uint32_t init,
                      uint32_t *d_scratch, hipStream_t s, int kind);
uint32_t crc_scratch_words(uint64_t len);

// CRC32C (kind kCrcKind32C) or CRC-32 (kCrcKind32) of `len` bytes already gathered in
// c->h_stage.
static int crc_staged(Ctx *c, size_t len, uint32_t init, uint32_t *out, int kind) {
  const uint32_t words = crc_scratch_words(len);
  int rc;
  if ((rc = ensure_dev(c, 0, len + 64)) || (rc = ensure_desc(c, size_t(words) * 4))) return rc;
  if (len) RDK_HIP_CHECK(hipMemcpyAsync(c->d_stage[0], c->h_stage, len, hipMemcpyHostToDevice, c->stream));
  if ((rc = crc_device_buffer(c, c->d_stage[0], len, init,
                              reinterpret_cast<uint32_t *>(c->d_desc), c->stream, kind)))
    return rc;
  RDK_HIP_CHECK(hipMemcpyAsync(c->h_desc, c->d_desc + size_t(words - 1) * 4, 4,
                               hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  std::memcpy(out, c->h_desc, 4);
  return 0;
}

// how often each drop-in symbol was entered (rdk_hip_dropin_calls), and how often a CRC
// symbol had to finish on the host after the device failed twice (rdk_hip_dropin_host_crcs)
static std::atomic<uint64_t> g_calls[5];
static std::atomic<uint64_t> g_host_crcs{0};
enum { CALL_CRC32C = 0, CALL_SLICE_CRC32C, CALL_SLICE_CRC32, CALL_LZ4C, CALL_LZ4D };

// RDK_HIP_REPORT=1: one line on stderr at process exit with the call counts, so a preload
// run of an unmodified program shows that its call sites reached the engine
__attribute__((destructor)) static void report_calls() {
  const char *e = getenv("RDK_HIP_REPORT");
  if (!e || !atoi(e)) return;
  fprintf(stderr, "librdkafka_hip: calls crc32c=%llu rd_slice_crc32c=%llu rd_slice_crc32=%llu "
                  "rd_kafka_lz4_compress=%llu rd_kafka_lz4_decompress=%llu host_crcs=%llu\n",
          (unsigned long long)g_calls[0].load(), (unsigned long long)g_calls[1].load(),
          (unsigned long long)g_calls[2].load(), (unsigned long long)g_calls[3].load(),
          (unsigned long long)g_calls[4].load(), (unsigned long long)g_host_crcs.load());
}

static Ctx *ctx_or_die(const char *who) {
  Ctx *c = ctx();
  if (!c) fatal(who);
  return c;
}

// Byte-at-a-time CRC over host bytes with the table the device images are built from
// (crc_build_tables: table 0 is the plain byte table of the polynomial).  Only the CRC
// symbols' last resort below uses it.
static uint32_t crc_host_bytes(const uint8_t *p, size_t len, uint32_t init, int kind) {
  static uint32_t tab[2][256];
  static std::once_flag once[2];
  std::call_once(once[kind], [kind] {
    std::vector<uint32_t> image(kCrcTableWords);
    crc_build_tables(image.data(), kind == kCrcKind32 ? kCrc32Poly : kCrcPoly);
    std::memcpy(tab[kind], image.data(), sizeof tab[kind]);
  });
  uint32_t c = ~init;
  for (size_t i = 0; i < len; ++i) c = tab[kind][(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return ~c;
}

// Stage `len` bytes already gathered in `bytes` (c->h_stage when the pinned staging could be
// had) and CRC them.  The CRC symbols return the checksum itself, so they have no way to
// report a device error: a failed attempt is retried once after draining the device (a
// transient allocation or launch failure).  If that fails too the checksum of THIS call is
// finished on the host from the staged bytes -- reported on stderr the first time and
// counted (rdk_hip_dropin_host_crcs) -- because neither a wrong CRC nor taking the
// producer down is acceptable for a per-call device error.  A process with no usable
// gfx950 device never gets here: ctx_or_die() stops it.
static uint32_t crc_or_host(Ctx *c, const uint8_t *bytes, size_t len, uint32_t init, int kind,
                            const char *who) {
  uint32_t out = 0;
  if (bytes == c->h_stage && c->h_stage) {
    if (crc_staged(c, len, init, &out, kind) == 0) return out;
    fprintf(stderr, "librdkafka_hip: %s: %s; retrying\n", who, last_error());
    (void)hipDeviceSynchronize();
    (void)hipGetLastError();
    if (crc_staged(c, len, init, &out, kind) == 0) return out;
  }
  if (!g_host_crcs.fetch_add(1))
    fprintf(stderr, "librdkafka_hip: %s: device path failed twice (%s); this call's checksum is "
                    "computed on the host (counted in rdk_hip_dropin_host_crcs)\n", who, last_error());
  (void)hipGetLastError();
  return crc_host_bytes(bytes, len, init, kind);
}

// The LZ4 symbols do have an error channel (rdkafka_lz4.c returns
// rd_kafka_resp_err_t): a device failure becomes __CRIT_SYS_RESOURCE (no device, out
// of memory) or __BAD_COMPRESSION (anything else), never an abort.  The writer then
// sends the MessageSet uncompressed (rdkafka_msgset_writer.c:1175-1176) and the reader
// raises a consumer error for the batch (rdkafka_msgset_reader.c:517-526).  The first
// failure of each kind is reported on stderr.
static std::atomic<int> g_reported{0};
static rd_kafka_resp_err_t lz4_err(int rc, const char *who) {
  if (rc <= -100) return rc;  // already an rd_kafka_resp_err_t
  const int bit = (rc == RDK_HIP_E_NODEV) ? 1 : (rc == RDK_HIP_E_NOMEM) ? 2 : 4;
  if (!(g_reported.fetch_or(bit) & bit))
    fprintf(stderr, "librdkafka_hip: %s failed on the device: %s\n", who, last_error());
  return (rc == RDK_HIP_E_NODEV || rc == RDK_HIP_E_NOMEM) ? RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE
                                                            : RDK_HIP_RESP_ERR__BAD_COMPRESSION;
}

static void slice_drain(rd_slice_t *slice) {  // leave the slice consumed, as the reference does
  const void *skip;
  while (slice_reader(slice, &skip)) {
  }
}

}  // namespace rdk

using namespace rdk;

RDK_API void crc32c_global_init(void) { (void)ctx_or_die("crc32c_global_init"); }

RDK_API void rdk_hip_dropin_calls(uint64_t out[5]) {
  for (int i = 0; i < 5; ++i) out[i] = g_calls[i].load();
}

RDK_API uint64_t rdk_hip_dropin_host_crcs(void) { return g_host_crcs.load(); }

RDK_API uint32_t crc32c(uint32_t crc, const void *buf, size_t len) {
  g_calls[CALL_CRC32C]++;
  Ctx *c = ctx_or_die("crc32c");
  if (len == 0) return crc;  // pre/post inversions cancel (crc32c.c:102,133)
  if (ensure_host(c, len))  // no pinned staging: nothing to copy from, finish on the host
    return crc_or_host(c, static_cast<const uint8_t *>(buf), len, crc, kCrcKind32C, "crc32c");
  std::memcpy(c->h_stage, buf, len);
  return crc_or_host(c, c->h_stage, len, crc, kCrcKind32C, "crc32c");
}

// iovec gather (the rdbuf.c:1099-1101 / :1118-1119 loops) into the pinned staging buffer;
// chaining the CRC over segments == one CRC over their concatenation
static uint32_t slice_crc(rd_slice_t *slice, int kind, const char *who) {
  Ctx *c = ctx_or_die(who);
  const size_t total = slice_remains(slice);
  size_t of = 0, rlen;
  const void *p;
  if (ensure_host(c, total ? total : 1)) {
    // no pinned staging: chain the segments on the host, as rdbuf.c:1118-1119 does
    if (!g_host_crcs.fetch_add(1))
      fprintf(stderr, "librdkafka_hip: %s: %s; this call's checksum is computed on the host "
                      "(counted in rdk_hip_dropin_host_crcs)\n", who, last_error());
    uint32_t crc = 0;
    while ((rlen = slice_reader(slice, &p)))
      crc = crc_host_bytes(static_cast<const uint8_t *>(p), rlen, crc, kind);
    return crc;
  }
  while ((rlen = slice_reader(slice, &p))) {
    std::memcpy(c->h_stage + of, p, rlen);
    of += rlen;
  }
  return crc_or_host(c, c->h_stage, of, 0u, kind, who);
}

RDK_API uint32_t rd_slice_crc32c(rd_slice_t *slice) {
  g_calls[CALL_SLICE_CRC32C]++;
  return slice_crc(slice, kCrcKind32C, "rd_slice_crc32c");
}

// rdbuf.c:1093-1104: rd_crc32_init/update/finalize, i.e. zlib crc32(0, ...) over the slice
// (rdcrc32.h:93-131, WITH_ZLIB) -- the MsgVersion 0/1 check.crcs site
// (rdkafka_msgset_reader.c:606)
RDK_API uint32_t rd_slice_crc32(rd_slice_t *slice) {
  g_calls[CALL_SLICE_CRC32]++;
  return slice_crc(slice, kCrcKind32, "rd_slice_crc32");
}

// ------------------------------------------------------------------- LZ4F
RDK_API rd_kafka_resp_err_t rd_kafka_lz4_compress(rd_kafka_broker_t *rkb, int proper_hc,
                                                  int comp_level, rd_slice_t *slice,
                                                  void **outbuf, size_t *outlenp) {
  (void)rkb;
  g_calls[CALL_LZ4C]++;
  *outbuf = nullptr;
  Ctx *c = ctx();
  if (!c) {
    slice_drain(slice);
    return lz4_err(RDK_HIP_E_NODEV, "rd_kafka_lz4_compress");
  }
  const size_t total = slice_remains(slice);
  int rc = ensure_host(c, total ? total : 1);
  if (rc) {
    slice_drain(slice);
    return lz4_err(rc, "rd_kafka_lz4_compress");
  }
  size_t of = 0, rlen;
  const void *p;
  while ((rlen = slice_reader(slice, &p))) {  // rdkafka_lz4.c:390 loop, gathered
    std::memcpy(c->h_stage + of, p, rlen);
    of += rlen;
  }
  rc = lz4f_compress_host(c, of, proper_hc, comp_level, outbuf, outlenp);
  return rc ? lz4_err(rc, "rd_kafka_lz4_compress") : RDK_HIP_RESP_ERR_NO_ERROR;
}

RDK_API rd_kafka_resp_err_t rd_kafka_lz4_decompress(rd_kafka_broker_t *rkb, int proper_hc,
                                                    int64_t Offset, char *inbuf, size_t inlen,
                                                    void **outbuf, size_t *outlenp) {
  (void)rkb;
  (void)Offset;
  g_calls[CALL_LZ4D]++;
  *outbuf = nullptr;
  Ctx *c = ctx();
  if (!c) return lz4_err(RDK_HIP_E_NODEV, "rd_kafka_lz4_decompress");
  int rc = lz4f_decompress_host(c, proper_hc, reinterpret_cast<uint8_t *>(inbuf), inlen, outbuf,
                                outlenp);
  return rc ? lz4_err(rc, "rd_kafka_lz4_decompress") : RDK_HIP_RESP_ERR_NO_ERROR;
}
