// lz4_frame.h -- LZ4F frame walking shared by host bookkeeping and kernels.
//
// Semantics follow rd_kafka_lz4_decompress (rdkafka_lz4.c:167-317) driving
// LZ4F_getFrameInfo / LZ4F_decompress (lz4frame.c:1109-1198, 1371-1840) over
// one contiguous input: header errors -> __BAD_COMPRESSION; a frame that runs
// out of input is a success holding the blocks completed so far (a truncated
// raw block contributes the bytes present); bytes after a complete frame ->
// __BAD_MSG; skippable frames yield no output.
#pragma once

#include <cstdint>

#ifndef RDK_HD
#define RDK_HD __host__ __device__
#endif

namespace rdk {

enum : uint32_t {
  F_LINKED = 1u,           // blockMode == linked
  F_BCHK = 2u,             // block checksums
  F_CCHK = 4u,             // content checksum flag
  F_CSIZE = 8u,            // content size present (non-zero)
  F_SEQ = 16u,             // decode sequentially in one wave (linked / many blocks)
  F_COMPLETE = 32u,        // frame fully consumed (end mark + checksum if any)
  F_ENDMARK = 64u,         // end mark reached (content size is checked)
  F_CCHK_PRESENT = 128u,   // stored content checksum available
  F_TRAILING = 256u,       // bytes follow a complete frame -> __BAD_MSG
  F_SKIPPABLE = 512u,
};

enum : uint32_t { B_RAW = 1u, B_TRUNC = 2u, B_XXH = 4u };

constexpr int32_t kErrBadMsg = -199;
constexpr int32_t kErrBadCompression = -198;
constexpr int32_t kErrDstSize = -1000;

struct FrameInfo {
  int32_t status;       // 0 or an rd_kafka_resp_err_t decided by the walk
  uint32_t nblocks;     // block descriptors produced
  uint32_t max_block;   // bytes
  uint32_t flags;
  uint64_t content_size;
  uint32_t content_xxh;
  uint32_t total_blocks;  // blocks in the frame (may exceed descriptor capacity)
};

struct BlockInfo {
  uint32_t src_off;  // offset of the block payload in the frame
  uint32_t csize;    // payload bytes (raw: bytes present)
  uint32_t flags;
  uint32_t xxh;      // stored block checksum (B_XXH)
};

// The most bytes a block can decode to: a stored block yields its own bytes; a compressed
// block of c bytes at most 255 * c (each 255-run byte of a match length adds 255 bytes of
// output), and never more than the frame's block size.
RDK_HD inline uint64_t lz4f_block_most(const BlockInfo &b, uint32_t max_block) {
  const uint64_t most = (b.flags & B_RAW) ? uint64_t(b.csize) : uint64_t(b.csize) * 255u;
  return most < max_block ? most : max_block;
}

template <typename Rd>
struct FrameWalker {
  Rd rd;            // byte reader: rd(i) -> byte i of the frame
  uint64_t inlen;
  uint64_t pos = 0;
  FrameInfo fi{};
  bool done = false;

  RDK_HD uint32_t le32(uint64_t i) {
    return uint32_t(rd(i)) | (uint32_t(rd(i + 1)) << 8) | (uint32_t(rd(i + 2)) << 16) |
           (uint32_t(rd(i + 3)) << 24);
  }

  // XXH32 of header bytes [4, n) (only 2..14 bytes; cheap on any side)
  RDK_HD uint32_t hdr_xxh(uint32_t n) {
    const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                   P5 = 374761393u;
    uint32_t len = n - 4, h = P5 + len;
    uint64_t p = 4;
    while (p + 4 <= n) { h += le32(p) * P3; h = ((h << 17) | (h >> 15)) * P4; p += 4; }
    while (p < n) { h += uint32_t(rd(p)) * P5; h = ((h << 11) | (h >> 21)) * P1; p++; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
  }

  // LZ4F_headerSize + LZ4F_decodeHeader (lz4frame.c:1109-1198, 1206-1228)
  RDK_HD void header() {
    fi.status = 0;
    if (inlen < 5) { fi.status = kErrBadCompression; done = true; return; }
    const uint32_t magic = le32(0);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      fi.flags |= F_SKIPPABLE;
      if (inlen < 8) { fi.status = kErrBadCompression; done = true; return; }
      const uint64_t end = 8ull + le32(4);
      if (end < inlen) fi.status = kErrBadMsg;
      done = true;
      return;
    }
    if (magic != 0x184D2204u) { fi.status = kErrBadCompression; done = true; return; }
    const uint32_t FLG = rd(4);
    const uint32_t hsize = 7u + ((FLG >> 3) & 1u ? 8u : 0u) + ((FLG & 1u) ? 4u : 0u);
    if (inlen < hsize || ((FLG >> 1) & 1u) || ((FLG >> 6) & 3u) != 1u) {
      fi.status = kErrBadCompression; done = true; return;
    }
    const uint32_t BD = rd(5), bsid = (BD >> 4) & 7u;
    if ((BD >> 7) || bsid < 4 || (BD & 15u) ||
        ((hdr_xxh(hsize - 1) >> 8) & 0xFFu) != uint32_t(rd(hsize - 1))) {
      fi.status = kErrBadCompression; done = true; return;
    }
    fi.max_block = (64u * 1024u) << (2u * (bsid - 4u));
    if (!((FLG >> 5) & 1u)) fi.flags |= F_LINKED;
    if ((FLG >> 4) & 1u) fi.flags |= F_BCHK;
    if ((FLG >> 2) & 1u) fi.flags |= F_CCHK;
    if ((FLG >> 3) & 1u) {
      fi.content_size = uint64_t(le32(6)) | (uint64_t(le32(10)) << 32);
      if (fi.content_size) fi.flags |= F_CSIZE;
    }
    pos = hsize;
  }

  // Next block in stream order; false when the frame ends (complete,
  // truncated or failed -- see fi.status / fi.flags).
  RDK_HD bool next(BlockInfo &b) {
    if (done) return false;
    if (pos >= inlen || inlen - pos < 4) { done = true; return false; }  // truncated
    const uint32_t bh = le32(pos);
    const uint32_t bsz = bh & 0x7FFFFFFFu;
    pos += 4;
    if (bsz == 0) {  // end mark -> dstage_getSuffix
      fi.flags |= F_ENDMARK;
      if (fi.flags & F_CCHK) {
        if (inlen - pos < 4) { done = true; return false; }
        fi.content_xxh = le32(pos);
        fi.flags |= F_CCHK_PRESENT;
        pos += 4;
      }
      fi.flags |= F_COMPLETE;
      if (pos < inlen) fi.flags |= F_TRAILING;
      done = true;
      return false;
    }
    if (bsz > fi.max_block) { fi.status = kErrBadCompression; done = true; return false; }
    b.flags = 0;
    b.xxh = 0;
    b.src_off = uint32_t(pos);
    const bool bchk = fi.flags & F_BCHK;
    if (bh & 0x80000000u) {  // dstage_copyDirect
      const uint64_t avail = inlen - pos;
      const uint32_t n = avail < bsz ? uint32_t(avail) : bsz;
      b.csize = n;
      b.flags = B_RAW;
      pos += n;
      if (n < bsz) { b.flags |= B_TRUNC; done = true; }
      else if (bchk) {
        if (inlen - pos < 4) { done = true; }
        else { b.xxh = le32(pos); b.flags |= B_XXH; pos += 4; }
      }
      fi.total_blocks++;
      return true;
    }
    const uint64_t need = uint64_t(bsz) + (bchk ? 4u : 0u);
    if (inlen - pos < need) { done = true; return false; }  // dstage_storeCBlock
    b.csize = bsz;
    if (bchk) { b.xxh = le32(pos + bsz); b.flags |= B_XXH; }
    pos += need;
    fi.total_blocks++;
    return true;
  }
};

}  // namespace rdk
