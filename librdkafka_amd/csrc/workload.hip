// workload.hip -- deterministic synthetic inputs (bench + tests).  Not on the
// product path; kept in the engine so bench.py can build multi-GB device
// workloads without a host round trip.
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.h"

namespace rdk {

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Every 8-byte word w of the buffer = splitmix64(seed + w).
__global__ void fill_random_kernel(uint64_t *__restrict__ p, uint64_t nwords, uint64_t seed) {
  for (uint64_t w = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; w < nwords;
       w += uint64_t(gridDim.x) * blockDim.x)
    p[w] = splitmix64(seed + w);
}

__device__ inline void put_be32(uint8_t *p, uint32_t v) {
  p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}
__device__ inline void put_be64(uint8_t *p, uint64_t v) {
  put_be32(p, uint32_t(v >> 32));
  put_be32(p + 4, uint32_t(v));
}
__device__ inline void put_be16(uint8_t *p, uint16_t v) { p[0] = uint8_t(v >> 8); p[1] = uint8_t(v); }

// MsgVersion 2 header (rdkafka_msgset_writer.c:352-403; offsets in
// rdkafka_proto.h:540-550): big-endian fields, CRC left 0.
__global__ void v2_headers_kernel(uint8_t *__restrict__ base, uint32_t n, uint32_t batch_size) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < n; b += gridDim.x * blockDim.x) {
    uint8_t *h = base + uint64_t(b) * batch_size;
    const uint32_t records = (batch_size - 61u) / 100u + 1u;
    put_be64(h + 0, uint64_t(b) * records);        // BaseOffset
    put_be32(h + 8, batch_size - 12u);             // Length
    put_be32(h + 12, 0);                           // PartitionLeaderEpoch
    h[16] = 2;                                     // Magic
    put_be32(h + 17, 0);                           // CRC (filled by FINALIZE)
    put_be16(h + 21, 0);                           // Attributes
    put_be32(h + 23, records - 1u);                // LastOffsetDelta
    put_be64(h + 27, 1600000000000ull + b);        // BaseTimestamp
    put_be64(h + 35, 1600000000000ull + b + 1);    // MaxTimestamp
    put_be64(h + 43, ~0ull);                       // ProducerId -1
    put_be16(h + 51, 0xffff);                      // ProducerEpoch -1
    put_be32(h + 53, 0xffffffffu);                 // BaseSequence -1
    put_be32(h + 57, records);                     // RecordCount
  }
}

}  // namespace rdk

using namespace rdk;

RDK_API int rdk_hip_gen_v2_batches(void *d_base, uint32_t n, uint32_t batch_size, uint64_t seed,
                                   void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (batch_size < 61 || (batch_size & 7)) return set_error(RDK_HIP_E_INVAL, "batch_size");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t nwords = uint64_t(n) * batch_size / 8;
  hipLaunchKernelGGL(fill_random_kernel, dim3(4096), dim3(256), 0, s,
                     static_cast<uint64_t *>(d_base), nwords, seed);
  hipLaunchKernelGGL(v2_headers_kernel, dim3((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096),
                     dim3(256), 0, s, static_cast<uint8_t *>(d_base), n, batch_size);
  RDK_HIP_CHECK(hipGetLastError());
  return RDK_HIP_OK;
}

// JSON-like record stream; byte-identical to
// librdkafka_amd.workload.gen_json().
RDK_API void rdk_hip_gen_json(uint8_t *dst, size_t len, uint32_t seed) {
  static const char *const kEvents[4] = {"click", "view", "purchase", "scroll"};
  uint32_t s = seed;
  auto draw = [&s]() {
    s = s * 1103515245u + 12345u;
    return s >> 8;
  };
  size_t of = 0;
  char rec[192];
  for (uint64_t id = 0; of < len; ++id) {
    const uint32_t user = draw() % 100000u;
    const uint32_t ts = 1600000000u + draw() % 86400u;
    const char *ev = kEvents[draw() & 3u];
    const uint32_t v = draw() % 10000u;
    const uint32_t f = draw() % 100u;
    int n = snprintf(rec, sizeof rec,
                     "{\"id\":%llu,\"user\":\"u%05u\",\"ts\":%u,\"event\":\"%s\",\"value\":%u.%02u}\n",
                     static_cast<unsigned long long>(id), user, ts, ev, v, f);
    size_t take = size_t(n) < len - of ? size_t(n) : len - of;
    std::memcpy(dst + of, rec, take);
    of += take;
  }
}
