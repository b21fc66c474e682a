// shim.cpp -- the drop-in symbols (see include/librdkafka_hip.h).
//
// Each call becomes a request over the caller's bytes (an rd_slice_t segment list or a
// contiguous buffer).  Whoever serves it (combine.h: the calling thread itself, or another
// broker thread that is taking a batch of requests to the device) gathers the bytes into
// pinned staging, copies them to the device, runs the gfx950 kernels and copies the result
// back into malloc() memory owned by the caller -- the ownership contract of rdkafka_lz4.c
// (rd_free == free, rd.h:104-119).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "combine.h"
#include "common.h"
#include "lz4_engine.h"
#include "rdbuf_abi.h"

namespace rdk {
int lz4f_fix_hc_in(uint8_t *in, size_t inlen);

// how often each drop-in symbol was entered (rdk_hip_dropin_calls)
static std::atomic<uint64_t> g_calls[5];
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
          (unsigned long long)g_calls[4].load(), (unsigned long long)combine_host_crcs());
}

static Ctx *ctx_or_die(const char *who) {
  Ctx *c = ctx();
  if (!c) fatal(who);
  return c;
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

// The slice's remaining runs (the rdbuf.c:1099-1101 / :1118-1119 / rdkafka_lz4.c:390 loops),
// leaving the slice consumed as the reference does.  The bytes stay where they are: whoever
// serves the request gathers them into its pinned staging.
static size_t slice_segments(rd_slice_t *slice, std::vector<Seg> &segs) {
  size_t total = 0, rlen;
  const void *p;
  while ((rlen = slice_reader(slice, &p))) {
    segs.push_back(Seg{static_cast<const uint8_t *>(p), rlen});
    total += rlen;
  }
  return total;
}

// the result's error detail belongs to the thread that served it: make it this thread's
static int owner_rc(const Req &r) {
  if (r.rc && r.err[0]) return set_error(r.rc, "%s", r.err);
  return r.rc;
}

}  // namespace rdk

using namespace rdk;

RDK_API void crc32c_global_init(void) { (void)ctx_or_die("crc32c_global_init"); }

RDK_API void rdk_hip_dropin_calls(uint64_t out[5]) {
  for (int i = 0; i < 5; ++i) out[i] = g_calls[i].load();
}

RDK_API uint64_t rdk_hip_dropin_host_crcs(void) { return combine_host_crcs(); }

RDK_API uint32_t crc32c(uint32_t crc, const void *buf, size_t len) {
  g_calls[CALL_CRC32C]++;
  Ctx *c = ctx_or_die("crc32c");
  if (len == 0) return crc;  // pre/post inversions cancel (crc32c.c:102,133)
  const Seg seg{static_cast<const uint8_t *>(buf), len};
  Req r;
  r.kind = kReqCrc32c;
  r.segs = &seg;
  r.nseg = 1;
  r.total = len;
  r.init = crc;
  r.who = "crc32c";
  combine_submit(c, &r);
  return r.crc;
}

// chaining the CRC over segments == one CRC over their concatenation
static uint32_t slice_crc(rd_slice_t *slice, int kind, const char *who) {
  Ctx *c = ctx_or_die(who);
  std::vector<Seg> segs;
  segs.reserve(8);
  Req r;
  r.kind = kind;
  r.total = slice_segments(slice, segs);
  r.segs = segs.data();
  r.nseg = segs.size();
  r.who = who;
  if (r.total == 0) return 0;
  combine_submit(c, &r);
  return r.crc;
}

RDK_API uint32_t rd_slice_crc32c(rd_slice_t *slice) {
  g_calls[CALL_SLICE_CRC32C]++;
  return slice_crc(slice, kReqCrc32c, "rd_slice_crc32c");
}

// rdbuf.c:1093-1104: rd_crc32_init/update/finalize, i.e. zlib crc32(0, ...) over the slice
// (rdcrc32.h:93-131, WITH_ZLIB) -- the MsgVersion 0/1 check.crcs site
// (rdkafka_msgset_reader.c:606)
RDK_API uint32_t rd_slice_crc32(rd_slice_t *slice) {
  g_calls[CALL_SLICE_CRC32]++;
  return slice_crc(slice, kReqCrc32, "rd_slice_crc32");
}

// ------------------------------------------------------------------- LZ4F
RDK_API rd_kafka_resp_err_t rd_kafka_lz4_compress(rd_kafka_broker_t *rkb, int proper_hc,
                                                  int comp_level, rd_slice_t *slice,
                                                  void **outbuf, size_t *outlenp) {
  (void)rkb;
  g_calls[CALL_LZ4C]++;
  *outbuf = nullptr;
  std::vector<Seg> segs;
  segs.reserve(8);
  Req r;
  r.kind = kReqLz4Compress;
  r.total = slice_segments(slice, segs);  // consumed on every path, as the reference does
  r.segs = segs.data();
  r.nseg = segs.size();
  r.proper_hc = proper_hc;
  r.level = comp_level;
  r.who = "rd_kafka_lz4_compress";
  Ctx *c = ctx();
  if (!c) return lz4_err(RDK_HIP_E_NODEV, r.who);
  combine_submit(c, &r);
  if (r.rc) return lz4_err(owner_rc(r), r.who);
  *outbuf = r.out;
  *outlenp = r.outlen;
  return RDK_HIP_RESP_ERR_NO_ERROR;
}

RDK_API rd_kafka_resp_err_t rd_kafka_lz4_decompress(rd_kafka_broker_t *rkb, int proper_hc,
                                                    int64_t Offset, char *inbuf, size_t inlen,
                                                    void **outbuf, size_t *outlenp) {
  (void)rkb;
  (void)Offset;
  g_calls[CALL_LZ4D]++;
  *outbuf = nullptr;
  const char *who = "rd_kafka_lz4_decompress";
  Ctx *c = ctx();
  if (!c) return lz4_err(RDK_HIP_E_NODEV, who);
  int rc;  // rd_kafka_lz4_decompress_fixup_bad_framing (rdkafka_lz4.c:50-98), on the caller's bytes
  if (!proper_hc && (rc = lz4f_fix_hc_in(reinterpret_cast<uint8_t *>(inbuf), inlen)))
    return lz4_err(rc, who);
  const Seg seg{reinterpret_cast<const uint8_t *>(inbuf), inlen};
  Req r;
  r.kind = kReqLz4Decompress;
  r.segs = &seg;
  r.nseg = 1;
  r.total = inlen;
  r.who = who;
  combine_submit(c, &r);
  if (r.rc) return lz4_err(owner_rc(r), who);
  *outbuf = r.out;
  *outlenp = r.outlen;
  return RDK_HIP_RESP_ERR_NO_ERROR;
}
