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
  size_t h_cap = 0;
  // device scratch (grow-only), two independent regions
  uint8_t *d_stage[2] = {nullptr, nullptr};
  size_t d_cap[2] = {0, 0};
  // small device descriptor buffer
  uint8_t *d_desc = nullptr;
  size_t d_desc_cap = 0;
  uint8_t *h_desc = nullptr;  // pinned mirror
};

// Returns the calling thread's context bound to a device, creating it on
// first use.  nullptr (with last_error set) when no gfx950 device exists.
Ctx *ctx();
int ensure_host(Ctx *c, size_t bytes);
int ensure_dev(Ctx *c, int which, size_t bytes);
int ensure_desc(Ctx *c, size_t bytes);

// Device-resident CRC tables for `device` (uploaded once per device).  kind selects the
// polynomial: kCrcKind32C (CRC-32C, crc32c.c) or kCrcKind32 (CRC-32/zlib, rdcrc32.h).
constexpr int kCrcKind32C = 0, kCrcKind32 = 1;
const uint32_t *crc_tables_dev(int device, int kind = kCrcKind32C);     // v1: slicing-by-16 image
const uint32_t *crc_tables_v3_dev(int device, int kind = kCrcKind32C);  // v3: rotated-nibble image
const uint32_t *crc_tables_v4_dev(int device, int kind = kCrcKind32C);  // v4: 16-lane-group image
// x^(2^k) mod P table (k = 0..63) for arbitrary-length shifts.
const uint32_t *crc_x2n_dev(int device, int kind = kCrcKind32C);

// Aborts the process with a message (drop-in symbols have no error channel).
[[noreturn]] void fatal(const char *what);

}  // namespace rdk

#define RDK_HIP_CHECK(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess)                                                     \
      return ::rdk::set_error(-2, "%s failed: %s (%s:%d)", #expr,             \
                              hipGetErrorString(_e), __FILE__, __LINE__);     \
  } while (0)
