// common.h -- shared definitions for the librdkafka_hip engine (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include "librdkafka_hip.h"

#include <cstddef>
#include <cstdint>

#define RDK_API extern "C" __attribute__((visibility("default")))

namespace rdk {

constexpr int kWave = 64;  // CDNA wavefront width; never 32.

// Records the last error (thread-local) and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
const char *last_error();

// Per-thread engine context: device, stream, staging memory.
struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  // pinned host staging (grow-only)
  uint8_t *h_stage = nullptr;
  uint8_t *dh_stage = nullptr;  // h_stage as the device sees it (nullptr: not mapped)
  size_t h_cap = 0;
  // device scratch (grow-only), independent regions: kScratchStage is the drop-in
  // symbols' staging (only ever used on `stream`, which every drop-in call leaves
  // idle); kScratchDecode / kScratchHc hold the batch API's descriptors and the
  // LZ4HC tables and follow the caller's streams (scratch_acquire / _release)
  uint8_t *d_stage[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t d_cap[4] = {0, 0, 0, 0};
  hipStream_t d_last[4] = {nullptr, nullptr, nullptr, nullptr};  // stream of the last user
  hipEvent_t d_done[4] = {nullptr, nullptr, nullptr, nullptr};  // recorded after the last use
  bool d_used[4] = {false, false, false, false};
  // CRC partial registers (the split CRC's chunks, the compress epilogue's block
  // registers), one grow-only buffer per caller stream: calls on different streams never
  // meet, so no event or allocation orders them
  static constexpr int kCrcStreams = 32;
  hipStream_t crc_stream[kCrcStreams] = {};
  uint32_t *crc_buf[kCrcStreams] = {};
  size_t crc_cap[kCrcStreams] = {};
  int crc_streams = 0;
  // small device descriptor buffer
  uint8_t *d_desc = nullptr;
  size_t d_desc_cap = 0;
  uint8_t *h_desc = nullptr;  // pinned mirror
  uint8_t *dh_desc = nullptr; // h_desc as the device sees it (nullptr: not mapped)
};

// Returns the calling thread's context bound to a device, creating it on
// first use.  nullptr (with last_error set) when no gfx950 device exists.
Ctx *ctx();
int ensure_host(Ctx *c, size_t bytes);
int ensure_dev(Ctx *c, int which, size_t bytes);
int ensure_desc(Ctx *c, size_t bytes);
constexpr int kScratchStage = 0, kScratchDecode = 1, kScratchHc = 2, kScratchCrc = 3;
constexpr int kScratchRegions = 4;
// Stream-ordered reuse of one scratch region by kernels on any stream: acquire makes
// stream `s` wait for the region's previous user (an event, no host wait unless the
// region has to grow), release marks the end of this use on `s`.
int scratch_acquire(Ctx *c, int which, size_t bytes, hipStream_t s);
int scratch_release(Ctx *c, int which, hipStream_t s);
// `bytes` (at least 64 KiB) of device words private to (this thread, stream s); nullptr
// with the error set
uint32_t *crc_scratch(Ctx *c, hipStream_t s, size_t bytes = 65536);

// Device-resident CRC tables for `device` (uploaded once per device).  kind selects the
// polynomial: kCrcKind32C (CRC-32C, crc32c.c) or kCrcKind32 (CRC-32/zlib, rdcrc32.h).
constexpr int kCrcKind32C = 0, kCrcKind32 = 1;
const uint32_t *crc_tables_dev(int device, int kind = kCrcKind32C);     // v1: slicing-by-16 image
const uint32_t *crc_tables_v3_dev(int device, int kind = kCrcKind32C);  // v3: rotated-nibble image
const uint32_t *crc_tables_v4_dev(int device, int kind = kCrcKind32C);  // v4: 16-lane-group image
// x^(2^k) mod P table (k = 0..63) for arbitrary-length shifts.
const uint32_t *crc_x2n_dev(int device, int kind = kCrcKind32C);

// Aborts the process with a message: only for the drop-in CRC symbols, whose
// signatures have no error channel, after a retry.
[[noreturn]] void fatal(const char *what);

}  // namespace rdk

#define RDK_HIP_CHECK(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess)                                                     \
      return ::rdk::set_error(_e == hipErrorOutOfMemory ? RDK_HIP_E_NOMEM     \
                                                        : RDK_HIP_E_HIP,      \
                              "%s failed: %s (%s:%d)", #expr,                 \
                              hipGetErrorString(_e), __FILE__, __LINE__);     \
  } while (0)
