// lz4_engine.h -- host entry points of the LZ4F engine used by the shim.
#pragma once

#include <cstddef>
#include <cstdint>

#include "common.h"

namespace rdk {

// Compress the `len` bytes staged in c->h_stage as one LZ4F frame with the
// reference's prefs (rdkafka_lz4.c:343-347).  *out is malloc()ed.
// Returns 0, an rd_kafka_resp_err_t (< -100), or an RDK_HIP_E_* code.
int lz4f_compress_host(Ctx *c, size_t len, int proper_hc, int level, void **out, size_t *outlen);

// Decompress one LZ4F frame from host memory (rdkafka_lz4.c:167-317
// semantics).  *out is malloc()ed.  Same return convention.
int lz4f_decompress_host(Ctx *c, int proper_hc, uint8_t *in, size_t inlen, void **out,
                         size_t *outlen);

}  // namespace rdk
