// combine.h -- concurrent drop-in calls go to the device together.
//
// librdkafka calls crc32c / rd_slice_crc32c / rd_kafka_lz4_compress / rd_kafka_lz4_decompress
// from every broker thread at once (rdkafka_broker.c:5082), one MessageSet per call
// (rdkafka_msgset_writer.c:1095, :1242; rdkafka_msgset_reader.c:395, :993).  A call of its
// own is one PCIe round trip and one stream synchronisation for one frame.  Here every
// call is queued as a request; the first thread that finds no batch in flight serves
// everything queued so far -- its own request and those of the threads that arrived while
// the previous batch was on the device -- as ONE staging copy and ONE launch of each batch
// kernel, then wakes the owners.  A lone caller finds the queue empty and no batch in
// flight and goes straight to the device.
#pragma once

#include <cstddef>
#include <cstdint>

#include "common.h"

namespace rdk {

struct Seg {
  const uint8_t *p;
  size_t n;
};

enum { kReqCrc32c = 0, kReqCrc32 = 1, kReqLz4Compress = 2, kReqLz4Decompress = 3 };

struct Req {
  int kind = 0;
  const Seg *segs = nullptr;  // the caller's bytes: valid until the request is served
  size_t nseg = 0;
  size_t total = 0;
  uint32_t init = 0;          // CRC kinds: the previous CRC
  int proper_hc = 1;          // LZ4 kinds
  int level = 0;              // compress: compression.level
  const char *who = "";
  // results
  uint32_t crc = 0;
  int rc = 0;                 // LZ4 kinds: 0, an rd_kafka_resp_err_t or an RDK_HIP_E_* code
  void *out = nullptr;        // LZ4 kinds: malloc()ed
  size_t outlen = 0;
  char err[160] = {0};        // LZ4 kinds: detail of rc for the owner's last_error()
  bool done = false;          // written and read under the combiner's mutex only
};

// Serves *r (on the calling thread's context c, or on another caller's, as part of its
// batch) and returns when its results are in place.
void combine_submit(Ctx *c, Req *r);

// How often the CRC symbols finished on the host (see shim.cpp).
uint64_t combine_host_crcs();

}  // namespace rdk
