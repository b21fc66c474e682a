// engine.cpp -- device/context management for librdkafka_hip.
//
// One context per calling thread (librdkafka calls the drop-in symbols from
// every broker thread concurrently, rdkafka_broker.c:5082): own HIP stream,
// own pinned staging and device scratch, released when the thread exits.
// Concurrent drop-in calls are queued and served in batches on the context of
// whichever caller takes the batch (combine.cpp).  CRC tables are uploaded once
// per device.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "common.h"
#include "crc32c_tables.h"

namespace rdk {

int lz4f_noalloc_setup(int dev);  // lz4_decode.hip: per-device address of its static scratch

static thread_local char tl_err[512];
static thread_local Ctx *tl_ctx = nullptr;

// Releases everything a thread's context holds: its stream, pinned staging and device
// scratch.  librdkafka creates and destroys broker threads as brokers come and go
// (rdkafka_broker.c:5082), so a context must not outlive its thread.
static void ctx_destroy(Ctx *c) {
  if (!c) return;
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
  }
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  for (int i = 0; i < kScratchRegions; ++i) {
    if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
    if (c->d_done[i]) (void)hipEventDestroy(c->d_done[i]);
  }
  for (int i = 0; i < c->crc_streams; ++i)
    if (c->crc_buf[i]) (void)hipFree(c->crc_buf[i]);
  if (c->d_desc) (void)hipFree(c->d_desc);
  if (c->h_desc) (void)hipHostFree(c->h_desc);
  (void)hipGetLastError();
  delete c;
}

// Owner of the calling thread's context: its destructor runs when the thread exits (for
// the main thread: before the static destructors, so before the HIP runtime unloads).
static std::atomic<uint64_t> g_ctx_created{0}, g_ctx_destroyed{0};
struct CtxOwner {
  ~CtxOwner() {
    if (tl_ctx) {
      ctx_destroy(tl_ctx);
      tl_ctx = nullptr;
      g_ctx_destroyed++;
    }
  }
};
static thread_local CtxOwner tl_owner;

int set_error(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(tl_err, sizeof tl_err, fmt, ap);
  va_end(ap);
  if (getenv("RDK_HIP_DEBUG")) fprintf(stderr, "librdkafka_hip: %s\n", tl_err);
  return code;
}

const char *last_error() { return tl_err; }

[[noreturn]] void fatal(const char *what) {
  fprintf(stderr, "librdkafka_hip: FATAL: %s: %s\n", what, tl_err[0] ? tl_err : "(no detail)");
  fflush(stderr);
  abort();
}

namespace {
constexpr int kMaxDev = 64;
std::mutex g_mu;
// [kind][device]: kind 0 = CRC-32C (MsgVersion 2), 1 = CRC-32 (MsgVersion 0/1)
uint32_t *g_tables[2][kMaxDev];
uint32_t *g_tables_v3[2][kMaxDev];
uint32_t *g_tables_v4[2][kMaxDev];
uint32_t *g_x2n[2][kMaxDev];

int default_device() {
  const char *e = getenv("RDK_HIP_DEVICE");
  return e ? atoi(e) : 0;
}

template <size_t N>
int upload(uint32_t **dst, const uint32_t (&host)[N]) {
  RDK_HIP_CHECK(hipMalloc(dst, sizeof host));
  RDK_HIP_CHECK(hipMemcpy(*dst, host, sizeof host, hipMemcpyHostToDevice));
  return 0;
}

int upload_tables(int dev) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_tables[1][dev]) return 0;
  static uint32_t host_tab[kCrcTableWords];
  static uint32_t host_tab2[kCrcV3Words];
  static uint32_t host_tab4[kCrcV4Words];
  static uint32_t host_x2n[kX2nDevWords];
  for (int kind = 0; kind < 2; ++kind) {
    const uint32_t poly = kind ? kCrc32Poly : kCrcPoly;
    crc_build_tables(host_tab, poly);
    crc_build_tables_v4(host_tab4, poly);
    crc_build_tables_v3(host_tab2, poly);
    crc_build_x2n_dev(host_x2n, poly);
    int rc;
    if ((rc = upload(&g_tables_v4[kind][dev], host_tab4)) ||
        (rc = upload(&g_tables[kind][dev], host_tab)) ||
        (rc = upload(&g_tables_v3[kind][dev], host_tab2)) ||
        (rc = upload(&g_x2n[kind][dev], host_x2n)))
      return rc;
  }
  return 0;
}

int bind(int dev) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_error(RDK_HIP_E_NODEV, "no HIP device visible");
  if (dev < 0 || dev >= ndev || dev >= kMaxDev)
    return set_error(RDK_HIP_E_INVAL, "device %d out of range (%d visible)", dev, ndev);
  hipDeviceProp_t prop;
  RDK_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_error(RDK_HIP_E_NODEV, "device %d is %s, engine is built for gfx950 only", dev,
                     prop.gcnArchName);
  RDK_HIP_CHECK(hipSetDevice(dev));
  int rc = upload_tables(dev);
  if (rc) return rc;
  if ((rc = lz4f_noalloc_setup(dev))) return rc;
  if (!tl_ctx) {
    (void)&tl_owner;  // odr-use: registers the thread-exit destructor
    tl_ctx = new Ctx();
    g_ctx_created++;
  }
  if (tl_ctx->device != dev) {
    if (tl_ctx->stream) (void)hipStreamDestroy(tl_ctx->stream);
    tl_ctx->stream = nullptr;
    RDK_HIP_CHECK(hipStreamCreateWithFlags(&tl_ctx->stream, hipStreamNonBlocking));
    tl_ctx->device = dev;
    // device scratch belongs to the old device: drop it
    for (int i = 0; i < kScratchRegions; ++i) {
      if (tl_ctx->d_stage[i]) (void)hipFree(tl_ctx->d_stage[i]);
      tl_ctx->d_stage[i] = nullptr;
      tl_ctx->d_cap[i] = 0;
      tl_ctx->d_used[i] = false;
      if (tl_ctx->d_done[i]) (void)hipEventDestroy(tl_ctx->d_done[i]);
      tl_ctx->d_done[i] = nullptr;
    }
    for (int i = 0; i < tl_ctx->crc_streams; ++i) (void)hipFree(tl_ctx->crc_buf[i]);
    tl_ctx->crc_streams = 0;
    if (tl_ctx->d_desc) (void)hipFree(tl_ctx->d_desc);
    tl_ctx->d_desc = nullptr;
    tl_ctx->d_desc_cap = 0;
  }
  return 0;
}
}  // namespace

Ctx *ctx() {
  if (tl_ctx && tl_ctx->device >= 0) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == tl_ctx->device) return tl_ctx;
    (void)hipSetDevice(tl_ctx->device);
    return tl_ctx;
  }
  if (bind(default_device())) return nullptr;
  return tl_ctx;
}

static size_t grow(size_t have, size_t want) {
  size_t n = have ? have : (size_t(1) << 20);
  while (n < want) n *= 2;
  return n;
}

// Upper bound on any one device scratch region, from $RDK_HIP_MAX_SCRATCH_BYTES
// (0 / unset = no bound): lets a deployment cap the engine's footprint and lets the
// tests force the allocation-failure paths.
static size_t scratch_limit() {
  const char *e = getenv("RDK_HIP_MAX_SCRATCH_BYTES");
  return e ? size_t(strtoull(e, nullptr, 10)) : 0;
}

int ensure_host(Ctx *c, size_t bytes) {
  if (c->h_cap >= bytes) return 0;
  // grow-only; the old contents are NOT kept: callers size the staging before they fill it
  size_t n = grow(c->h_cap, bytes);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  c->h_stage = nullptr;
  c->dh_stage = nullptr;
  c->h_cap = 0;  // a failed allocation must not leave a capacity behind a null pointer
  const size_t lim = scratch_limit();
  if (lim && n > lim)
    return set_error(RDK_HIP_E_NOMEM, "pinned staging of %zu bytes exceeds RDK_HIP_MAX_SCRATCH_BYTES=%zu",
                     n, lim);
  RDK_HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&c->h_stage), n,
                              hipHostMallocMapped | hipHostMallocCoherent));
  c->h_cap = n;
  // the device's view of the staging: kernels that pass over their input once (the CRCs)
  // read it in place instead of waiting for a copy
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&c->dh_stage), c->h_stage, 0) != hipSuccess) {
    c->dh_stage = nullptr;
    (void)hipGetLastError();
  }
  return 0;
}

static int dev_alloc(uint8_t **p, size_t n) {
  const size_t lim = scratch_limit();
  if (lim && n > lim)
    return set_error(RDK_HIP_E_NOMEM, "device scratch of %zu bytes exceeds RDK_HIP_MAX_SCRATCH_BYTES=%zu",
                     n, lim);
  RDK_HIP_CHECK(hipMalloc(reinterpret_cast<void **>(p), n));
  return 0;
}

// kScratchStage only: used on c->stream alone, and every drop-in call returns with
// that stream idle, so growing needs no wait.
int ensure_dev(Ctx *c, int which, size_t bytes) {
  if (c->d_cap[which] >= bytes) return 0;
  if (c->d_stage[which]) (void)hipFree(c->d_stage[which]);
  c->d_stage[which] = nullptr;
  c->d_cap[which] = 0;
  size_t n = grow(c->d_cap[which], bytes);
  int rc = dev_alloc(&c->d_stage[which], n);
  if (rc) return rc;
  c->d_cap[which] = n;
  return 0;
}

int scratch_acquire(Ctx *c, int which, size_t bytes, hipStream_t s) {
  if (!c->d_done[which])
    RDK_HIP_CHECK(hipEventCreateWithFlags(&c->d_done[which], hipEventDisableTiming));
  if (c->d_cap[which] < bytes) {
    // the previous user may still be running on another stream: wait for it alone
    if (c->d_used[which]) RDK_HIP_CHECK(hipEventSynchronize(c->d_done[which]));
    if (c->d_stage[which]) (void)hipFree(c->d_stage[which]);
    c->d_stage[which] = nullptr;
    c->d_cap[which] = 0;
    c->d_used[which] = false;
    size_t n = grow(0, bytes);
    int rc = dev_alloc(&c->d_stage[which], n);
    if (rc) return rc;
    c->d_cap[which] = n;
  } else if (c->d_used[which] && c->d_last[which] != s) {
    RDK_HIP_CHECK(hipStreamWaitEvent(s, c->d_done[which], 0));
  }
  return 0;
}

int scratch_release(Ctx *c, int which, hipStream_t s) {
  RDK_HIP_CHECK(hipEventRecord(c->d_done[which], s));
  c->d_last[which] = s;
  c->d_used[which] = true;
  return 0;
}

uint32_t *crc_scratch(Ctx *c, hipStream_t s, size_t bytes) {
  if (bytes < 65536) bytes = 65536;
  int slot = -1;
  for (int i = 0; i < c->crc_streams; ++i)
    if (c->crc_stream[i] == s) slot = i;
  if (slot < 0) {
    if (c->crc_streams < Ctx::kCrcStreams) {
      slot = c->crc_streams++;
      c->crc_buf[slot] = nullptr;
      c->crc_cap[slot] = 0;
    } else {  // more streams than slots: recycle the oldest once its stream has drained
      slot = 0;
      if (hipStreamSynchronize(c->crc_stream[0]) != hipSuccess) (void)hipGetLastError();
    }
    c->crc_stream[slot] = s;
  }
  if (c->crc_cap[slot] < bytes) {
    if (c->crc_buf[slot]) {  // kernels of earlier calls on this stream may still use it
      if (hipStreamSynchronize(s) != hipSuccess) (void)hipGetLastError();
      (void)hipFree(c->crc_buf[slot]);
      c->crc_buf[slot] = nullptr;
      c->crc_cap[slot] = 0;
    }
    uint8_t *p = nullptr;
    const size_t n = grow(0, bytes);
    if (dev_alloc(&p, n)) return nullptr;
    c->crc_buf[slot] = reinterpret_cast<uint32_t *>(p);
    c->crc_cap[slot] = n;
  }
  return c->crc_buf[slot];
}

// drop-in symbols only (c->stream, idle between calls)
int ensure_desc(Ctx *c, size_t bytes) {
  if (c->d_desc_cap >= bytes) return 0;
  if (c->d_desc) {
    (void)hipFree(c->d_desc);
    (void)hipHostFree(c->h_desc);
  }
  c->d_desc = nullptr;
  c->h_desc = nullptr;
  c->dh_desc = nullptr;
  c->d_desc_cap = 0;
  size_t n = grow(0, bytes);
  int rc = dev_alloc(&c->d_desc, n);
  if (rc) return rc;
  RDK_HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&c->h_desc), n,
                              hipHostMallocMapped | hipHostMallocCoherent));
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&c->dh_desc), c->h_desc, 0) != hipSuccess) {
    c->dh_desc = nullptr;
    (void)hipGetLastError();
  }
  c->d_desc_cap = n;
  return 0;
}

const uint32_t *crc_tables_dev(int device, int kind) { return g_tables[kind][device]; }
const uint32_t *crc_tables_v3_dev(int device, int kind) { return g_tables_v3[kind][device]; }
const uint32_t *crc_tables_v4_dev(int device, int kind) { return g_tables_v4[kind][device]; }
const uint32_t *crc_x2n_dev(int device, int kind) { return g_x2n[kind][device]; }

}  // namespace rdk

RDK_API int rdk_hip_init(int device) {
  if (device < 0) device = rdk::default_device();
  return rdk::bind(device);
}

// contexts created / destroyed so far (one per calling thread; destroyed at thread exit)
RDK_API void rdk_hip_ctx_counts(uint64_t out[2]) {
  out[0] = rdk::g_ctx_created.load();
  out[1] = rdk::g_ctx_destroyed.load();
}

RDK_API const char *rdk_hip_last_error(void) { return rdk::last_error(); }

RDK_API const char *rdk_hip_version(void) {
  return "librdkafka_hip 0.6 gfx950 crc32c:group16-bytetab-lds lz4c:window64-exact+round64-fast+wave-finish+seq-queue+units-lds lz4hc:3-12-lds-build lz4d:seg64-parallel snappy:window64-exact+fragment-decode dropin:combined-callers";
}
