// lz4_finish_wave.h -- what a block kernel's wavefront does behind a block when the batch's
// CRC is fused into the compressor (FuseCrc, lz4_engine.h).
//
//   * A frame of ONE block (record batches up to 64 KiB) is finished by the wave that has
//     compressed it, with no second kernel: LZ4F header and end mark (lz4frame.c:671-701,
//     :984-1018), the writer's codec choice (rdkafka_msgset_writer.c:1179-1187),
//     finalize_MessageSet_v2_header (:1251-1295) and calc_crc_v2 (:1229-1246).  The block
//     sits where the frame wants it (slot 0 starts 7 bytes into the frame), so header,
//     frame and end mark are one contiguous range written by this wave, and the CRC is one
//     pass over it.
//   * A block of a longer frame leaves its raw CRC32C register in stream form (LE32 size
//     word || payload) for the frame assembler to combine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "crc_wave.h"
#include "lz4_device.h"
#include "lz4_engine.h"
#include "lz4_wave.h"

namespace rdk {

constexpr uint32_t kFinHdr = 61;  // RD_KAFKAP_MSGSET_V2_SIZE (rdkafka_proto.h:540)

// ob: the frame's place (61 bytes into the batch slot); ib: the records (the header the
// writer left is the 61 bytes in front of them); len: record bytes; w: the block's size
// word as stored at ob + 7.  t4: the four byte tables in LDS.
__device__ __forceinline__ void wave_finish_single(uintptr_t ob, uintptr_t ib, uint32_t len, uint32_t w,
                                                   uint32_t f, uint32_t *__restrict__ out_lens,
                                                   const FuseCrc &fuse, const crcw_lds_u32 *t4,
                                                   int lane) {
  const uint32_t sz = w & 0x7FFFFFFFu;
  const uint32_t flen = 7u + 4u + sz + 4u;
  const bool compressed = flen <= len;  // (a stored block never is: its frame is len + 15 bytes)
  const uint32_t payload = compressed ? flen : len;
  const uintptr_t bo = ob - kFinHdr, hdr = ib - kFinHdr;
  if (compressed) {
    // magic, FLG 0x60 (v01, independent), BD 0x40 (64 KB), HC 0x82; end mark
    if (lane < 7) stb(ob + uint32_t(lane), uint32_t(0x00824060184D2204ull >> (8 * lane)) & 0xFFu);
    if (lane >= 8 && lane < 12) stb(ob + 11u + sz + uint32_t(lane - 8), 0u);
  } else {
    asm_slide<64, false>(ob, ib, len, lane);  // keep the records plain
  }
  if (uint32_t(lane) < kFinHdr) {
    uint32_t v = ldb(hdr + uint32_t(lane));
    const uint32_t length = kFinHdr + payload - 12u;
    if (lane >= 8 && lane < 12) v = (length >> (8u * (3u - (uint32_t(lane) - 8u)))) & 0xFFu;
    if (lane == 22 && compressed) v |= 3u;  // Attributes |= RD_KAFKA_COMPRESSION_LZ4
    if (lane >= 17 && lane < 21) v = 0;
    stb(bo + uint32_t(lane), v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the range below is this wave's own stores
  const uint32_t crc = ~wave_crc_range(bo + 21u, kFinHdr - 21u + payload, true, t4, fuse.x2n, lane);
  if (lane == 0) {
    stb(bo + 17, crc >> 24); stb(bo + 18, (crc >> 16) & 0xFFu);
    stb(bo + 19, (crc >> 8) & 0xFFu); stb(bo + 20, crc & 0xFFu);
    fuse.batch_lens[f] = kFinHdr + payload;
    fuse.crcs[f] = crc;
    out_lens[f] = flen;
  }
}

// Raw register of block k of a longer frame: size word || payload.  A compressed block is
// contiguous in its slot; a stored one has its payload in the input.
__device__ __forceinline__ uint32_t wave_block_register(uint32_t w, uintptr_t slot, uintptr_t src,
                                                        const FuseCrc &fuse, const crcw_lds_u32 *t4,
                                                        int lane) {
  const uint32_t sz = w & 0x7FFFFFFFu;
  if (!(w >> 31)) return wave_crc_range(slot, 4u + sz, false, t4, fuse.x2n, lane);
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) r = t4[(r ^ (w >> (8 * j))) & 0xFFu] ^ (r >> 8);
  return crcw_shift_lut(r, sz, fuse.x2n) ^ wave_crc_range(src, sz, false, t4, fuse.x2n, lane);
}

// Behind block k of frame f (size word w stored at `slot`, the wave's stores retired by the
// caller): finish the batch or leave the block's register.  `lds`: at least 4 KiB, dead.
__device__ __forceinline__ void wave_block_epilogue(uint32_t w, uintptr_t slot, uintptr_t src, uint32_t k,
                                                    uint32_t nb, uint32_t f, uintptr_t ob, uintptr_t ib,
                                                    uint32_t len, uint32_t *__restrict__ out_lens,
                                                    const FuseCrc &fuse, crcw_lds_u32 *lds, int lane) {
  crcw_load_t4(lds, fuse.t0, lane);
  if (fuse.single_done && nb == 1u)
    wave_finish_single(ob, ib, len, w, f, out_lens, fuse, lds, lane);
  else
    fuse.block_crc[size_t(f) * 64u + k] = wave_block_register(w, slot, src, fuse, lds, lane);
  asm volatile("" ::: "memory");
}

}  // namespace rdk
