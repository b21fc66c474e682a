// hip_stub.cpp -- TEST INFRASTRUCTURE: a host-only stand-in for the HIP runtime and for the
// engine's device entry points, so that the library's host files (shim.cpp, combine.cpp,
// engine.cpp, lz4_host.cpp) can be built with -fsanitize=thread and run without a GPU.
//
// "Device" memory is malloc() memory, copies are memcpy at the call, streams and events are
// tokens.  The CRC entry points compute the right answer (byte table); the LZ4F entry
// points write / read valid frames of stored blocks (lz4frame.c:739-761 stores a block raw
// when it does not shrink), so round trips work and the host-side bookkeeping -- staging
// layout, descriptors, result hand-out, error paths -- is what runs under the sanitizer.
// STUB_FAIL_EVERY=N makes every Nth device entry point call fail, STUB_FAIL_ALLOC=1 makes
// pinned allocations fail: the retry, one-at-a-time fallback and host-CRC paths.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "crc32c_tables.h"
#include "lz4_engine.h"

static std::atomic<uint64_t> g_entry{0};
static int fail_every() {
  static const int n = [] {
    const char *e = getenv("STUB_FAIL_EVERY");
    return e ? atoi(e) : 0;
  }();
  return n;
}
static bool entry_fails() {
  const int n = fail_every();
  return n > 0 && (g_entry.fetch_add(1) + 1) % uint64_t(n) == 0;
}

extern "C" {
hipError_t hipGetDeviceCount(int *n) { *n = 1; return hipSuccess; }
hipError_t hipGetDeviceProperties(hipDeviceProp_t *p, int) {
  std::memset(p, 0, sizeof *p);
  std::strcpy(p->gcnArchName, "gfx950:stub");
  return hipSuccess;
}
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
hipError_t hipMalloc(void **p, size_t n) { *p = std::malloc(n ? n : 1); return *p ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipFree(void *p) { std::free(p); return hipSuccess; }
hipError_t hipHostMalloc(void **p, size_t n, unsigned) {
  const char *e = getenv("STUB_FAIL_ALLOC");
  if (e && atoi(e)) { *p = nullptr; return hipErrorOutOfMemory; }
  *p = std::malloc(n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void *p) { std::free(p); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void **d, void *h, unsigned) {
  const char *e = getenv("STUB_NO_MAPPED");  // the copy path instead of the in-place one
  if (e && atoi(e)) return hipErrorInvalidValue;
  *d = h;
  return hipSuccess;
}
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { std::memcpy(d, s, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind, hipStream_t) {
  std::memcpy(d, s, n);
  return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) {
  *s = reinterpret_cast<hipStream_t>(std::malloc(8));
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) { std::free(s); return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) {
  *e = reinterpret_cast<hipEvent_t>(std::malloc(8));
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) { std::free(e); return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
const char *hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "stub error"; }
}

namespace rdk {

int lz4f_noalloc_setup(int) { return 0; }

static uint32_t crc_bytes(const uint8_t *p, size_t len, uint32_t init, int kind) {
  static uint32_t tab[2][256];
  static std::atomic<int> ready{0};
  static std::atomic_flag busy = ATOMIC_FLAG_INIT;
  while (!ready.load(std::memory_order_acquire)) {
    if (!busy.test_and_set()) {
      for (int k = 0; k < 2; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
          uint32_t r = b;
          for (int i = 0; i < 8; ++i) r = (r >> 1) ^ ((r & 1u) ? (k ? kCrc32Poly : kCrcPoly) : 0u);
          tab[k][b] = r;
        }
      ready.store(1, std::memory_order_release);
    }
  }
  uint32_t c = ~init;
  for (size_t i = 0; i < len; ++i) c = tab[kind][(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return ~c;
}

uint32_t crc_scratch_words(uint64_t) { return 2; }

int crc_device_buffer(Ctx *, const uint8_t *d_buf, uint64_t len, uint32_t init, uint32_t *d_scratch,
                      hipStream_t, int kind, uint32_t *d_final) {
  if (entry_fails()) return set_error(RDK_HIP_E_HIP, "stub: crc_device_buffer fails");
  *(d_final ? d_final : d_scratch + 1) = crc_bytes(d_buf, len, init, kind);
  return 0;
}

static int ranges(const void *base, const uint64_t *offs, const uint32_t *lens, const uint32_t *init,
                  uint32_t *out, uint32_t n, int kind) {
  if (entry_fails()) return set_error(RDK_HIP_E_HIP, "stub: crc ranges fails");
  for (uint32_t i = 0; i < n; ++i)
    out[i] = crc_bytes(static_cast<const uint8_t *>(base) + offs[i], lens[i], init ? init[i] : 0u, kind);
  return 0;
}

size_t lz4f_compress_bound(size_t len) { return 7 + len + 4 * ((len + 65535) / 65536) + 4 + 64; }

static const uint8_t kHdr[7] = {0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82};

static int compress(const uint8_t *d_in, const uint64_t *in_offs, const uint32_t *in_lens, uint8_t *d_out,
                    const uint64_t *out_offs, uint32_t *out_lens, uint32_t n) {
  if (entry_fails()) return set_error(RDK_HIP_E_HIP, "stub: compress fails");
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *src = d_in + in_offs[i];
    uint8_t *o = d_out + out_offs[i];
    size_t op = 7;
    std::memcpy(o, kHdr, 7);
    for (size_t at = 0; at < in_lens[i]; at += 65536) {
      const uint32_t bn = uint32_t(in_lens[i] - at < 65536 ? in_lens[i] - at : 65536);
      const uint32_t w = bn | 0x80000000u;
      std::memcpy(o + op, &w, 4);
      std::memcpy(o + op + 4, src + at, bn);
      op += 4 + bn;
    }
    std::memset(o + op, 0, 4);
    out_lens[i] = uint32_t(op + 4);
  }
  return 0;
}

int lz4f_compress_device(Ctx *, const uint8_t *d_in, const uint64_t *in_offs, const uint32_t *in_lens,
                         uint8_t *d_out, const uint64_t *out_offs, uint32_t *out_lens, uint32_t n, int,
                         hipStream_t, const FuseCrc *) {
  return compress(d_in, in_offs, in_lens, d_out, out_offs, out_lens, n);
}

int lz4hc_compress_device(const uint8_t *d_in, const uint64_t *in_offs, const uint32_t *in_lens,
                          uint8_t *d_out, const uint64_t *out_offs, uint32_t *out_lens, uint32_t n, int,
                          hipStream_t) {
  return compress(d_in, in_offs, in_lens, d_out, out_offs, out_lens, n);
}

int lz4f_decompress_device(Ctx *, const uint8_t *d_in, const uint64_t *in_offs, const uint32_t *in_lens,
                           uint8_t *d_out, const uint64_t *out_offs, const uint32_t *out_caps,
                           uint32_t *out_lens, int32_t *status, uint32_t n, hipStream_t) {
  if (entry_fails()) return set_error(RDK_HIP_E_HIP, "stub: decompress fails");
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *in = d_in + in_offs[i];
    uint8_t *o = d_out + out_offs[i];
    size_t ip = 7, op = 0;
    status[i] = 0;
    out_lens[i] = 0;
    if (in_lens[i] < 11 || std::memcmp(in, kHdr, 4)) {
      status[i] = -198;
      continue;
    }
    for (;;) {
      uint32_t w;
      if (ip + 4 > in_lens[i]) { status[i] = -198; break; }
      std::memcpy(&w, in + ip, 4);
      ip += 4;
      if (!w) break;
      const uint32_t bn = w & 0x7FFFFFFFu;
      if (!(w & 0x80000000u) || ip + bn > in_lens[i] || op + bn > out_caps[i]) { status[i] = -198; break; }
      std::memcpy(o + op, in + ip, bn);
      ip += bn;
      op += bn;
    }
    if (!status[i]) out_lens[i] = uint32_t(op);
  }
  return 0;
}

}  // namespace rdk

extern "C" int rdk_hip_crc32c_ranges(const void *b, const uint64_t *o, const uint32_t *l, const uint32_t *i,
                                     uint32_t *out, uint32_t n, void *) {
  return rdk::ranges(b, o, l, i, out, n, rdk::kCrcKind32C);
}
extern "C" int rdk_hip_crc32_ranges(const void *b, const uint64_t *o, const uint32_t *l, const uint32_t *i,
                                    uint32_t *out, uint32_t n, void *) {
  return rdk::ranges(b, o, l, i, out, n, rdk::kCrcKind32);
}
