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

// The compress epilogue's CRC (crc_wave.h): when block_crc is set, the block kernels store
// the raw CRC32C register of every block in stream form (LE32 size word || payload) at
// block_crc[frame * 64 + block] (blocks 0..63), and the frame assembler turns a frame that
// sits 61 bytes into a MsgVersion 2 batch slot into the finished batch: header copied from
// in front of the records with Length and the LZ4 codec bits set (or the records kept
// plain when the frame is larger, rdkafka_msgset_writer.c:1179), CRC32C combined from the
// header, the block registers and the end mark, stored at offset 17.
struct FuseCrc {
  uint32_t *block_crc = nullptr;   // n * 64 words of device scratch
  const uint32_t *t0 = nullptr;    // byte table (256 words, device)
  const uint32_t *x2n = nullptr;   // x^(2^k) mod P, k = 0..63 (device)
  uint32_t *batch_lens = nullptr;  // out: 61 + payload bytes
  uint32_t *crcs = nullptr;        // out: the stored CRC
  // Set by an engine whose block kernel finishes the batches of single-block frames itself
  // (lz4_finish_wave.h); the assembler then passes over them.
  bool single_done = false;
  // One spare device word (optional): with thousands of frames the block kernels first find
  // the largest block count of any frame there, so that their slot-major item loop does not
  // visit 64 block slots of frames that have one.
  uint32_t *max_nb = nullptr;
};

// Largest block count of any of the n frames -> *d_max_nb (one small launch).
void lz4f_max_blocks_launch(const uint32_t *d_in_lens, uint32_t n, uint32_t *d_max_nb, void *stream);
// Above this many frames the launch above pays (fewer: the empty slots are a few loop turns).
constexpr uint32_t kMaxNbFrames = 4096;

}  // namespace rdk
