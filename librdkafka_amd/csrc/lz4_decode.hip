// lz4_decode.hip -- LZ4F frame decompression on gfx950.
//
// Replaces rd_kafka_lz4_decompress (src/rdkafka_lz4.c:167-317) ->
// LZ4F_decompress (lz4frame.c:1371) -> LZ4_decompress_safe_usingDict
// (lz4.c:2307 -> LZ4_decompress_generic lz4.c:1654-2068).
//
// Pipeline per batch of frames:
//   1. walk kernel   : one lane per frame parses the header and block table
//                      (FrameWalker, lz4_frame.h) into descriptors;
//   2. block kernel  : one wavefront per independent block decodes straight
//                      into out + k*maxBlockSize (zero-copy for regular frames);
//                      linked frames / frames with more than kMaxDesc blocks
//                      are decoded whole by one wavefront, in stream order;
//   3. finish kernel : one wavefront per frame applies the frame-level checks
//                      (content size / checksum, trailing bytes) in the
//                      reference's order and compacts irregular frames.
//
// The block decoder is a wave-uniform restatement of LZ4_decompress_generic
// including its fast loop (lz4.c:1707-1824) and the safe-loop shortcut
// (lz4.c:1846-1889): every bounds check is kept so malformed blocks are
// accepted or rejected exactly as the reference does.  Control is scalar
// (token parsing from a 512-byte register window via v_readlane); literal and
// match bytes are moved by all 64 lanes.
#include <hip/hip_runtime.h>

#include "common.h"
#include "lz4_device.h"
#include "lz4_frame.h"

namespace rdk {

constexpr int kMaxDesc = 64;          // descriptors per frame (4 MiB of 64 KiB blocks)
constexpr int kFastloopSafeDistance = 64;

struct BlockDesc {
  BlockInfo b;
  int32_t result;   // decoded bytes, or <0
  uint32_t pad;
};

struct FrameState {
  FrameInfo fi;
  int32_t seq_result;  // F_SEQ frames: total bytes or <0
  uint32_t pad;
};

// ----------------------------------------------------------- input window
struct InWin {
  uintptr_t base;  // 4-aligned address held by lane 0 of `cur`
  uintptr_t lim;   // first address past the last readable dword
  uint32_t cur, nxt;
};

__device__ __forceinline__ uint32_t ld_dw(uintptr_t a, uintptr_t lim) {
  return a < lim ? *(g_cu32 *)a : 0u;
}

__device__ __forceinline__ void win_load(InWin &w, uintptr_t base, int lane) {
  w.base = base;
  w.cur = ld_dw(base + 4u * lane, w.lim);
  w.nxt = ld_dw(base + 256u + 4u * lane, w.lim);
}

__device__ __forceinline__ uint32_t win_byte(InWin &w, uintptr_t p, int lane) {
  if (p < w.base || p >= w.base + 512u) {
    win_load(w, p & ~uintptr_t(3), lane);
  } else if (p >= w.base + 256u) {
    w.base += 256u;
    w.cur = w.nxt;
    w.nxt = ld_dw(w.base + 256u + 4u * lane, w.lim);
  }
  const uint32_t off = uint32_t(p - w.base);
  // uniform branch: only touch nxt (possibly still in flight) when needed
  uint32_t dw;
  if (off < 256u) dw = __builtin_amdgcn_readlane(w.cur, int(off >> 2));
  else dw = __builtin_amdgcn_readlane(w.nxt, int((off & 255u) >> 2));
  return (dw >> (8u * uint32_t(p & 3u))) & 0xFFu;
}

// ---------------------------------------------------------- byte movers
__device__ __forceinline__ void copy_fwd(uintptr_t d, uintptr_t s, uint32_t len, int lane) {
  asm volatile("" ::: "memory");
  // up to 3 bytes bring the destination to a dword boundary; then a dword per lane and step
  // (four steps' loads in flight), each made of the two aligned source dwords it lies in,
  // read through a range-checked resource (nothing is touched past the source's end); the
  // last 0..3 bytes by lanes again
  uint32_t head = uint32_t((4u - uint32_t(d & 3u)) & 3u);
  head = head < len ? head : len;
  if (uint32_t(lane) < head) stb(d + uint32_t(lane), ldb(s + uint32_t(lane)));
  const uintptr_t d4 = d + head, s4 = s + head;
  const uint32_t n4 = (len - head) >> 2;
  const uint32_t sh = uint32_t(s4 & 3u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void *>(s4 - sh), 0, int((sh + (len - head) + 3u) & ~3u), 0x00020000);
  for (uint32_t base = 0; base < n4; base += 256u) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + uint32_t(lane) + 64u * uint32_t(j);
      lo[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * i, 0, 0);  // (past the end: 0)
      hi[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * i + 4u, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + uint32_t(lane) + 64u * uint32_t(j);
      if (i < n4) *(g_u32 *)(d4 + 4u * i) = __builtin_amdgcn_alignbyte(hi[j], lo[j], sh);
    }
  }
  const uint32_t done = head + 4u * n4;
  if (uint32_t(lane) < len - done) stb(d + done + uint32_t(lane), ldb(s + done + uint32_t(lane)));
  asm volatile("" ::: "memory");
}

// ------------------------------------------------------ output history ring
// Each wavefront decodes into an 8 KiB LDS ring holding the newest output
// bytes and streams it to HBM in 4 KiB pieces with 16-byte stores.  Matches
// reaching <= kRingReach back (the common case) are served from LDS; longer
// ones, and linked-block matches into the previous blocks, read the
// already-flushed output from global memory.  Literals come from the input
// register window (cross-lane ds_bpermute), so in the steady state a sequence
// touches HBM only through the window prefetch and the ring flush.
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4v lds_u32x4;
typedef __attribute__((address_space(1))) u32x4v g_u32x4;
#ifndef RDK_DEC_RING
#define RDK_DEC_RING 4096
#endif
constexpr uint32_t kRing = RDK_DEC_RING;        // LDS history per wavefront (>= 4096, see
                                                // lz4_decode_fast.h far-history note)
static_assert(kRing >= 4096 && (kRing & (kRing - 1)) == 0, "ring size");
constexpr uint32_t kRingMask = kRing - 1u;
constexpr uint32_t kFlush = kRing / 2 < 4096 ? kRing / 2 : 4096;  // bytes per streamed piece
constexpr uint32_t kRingReach = kRing - 256u;   // max offset served from LDS
constexpr int kDecWaves = 4;                    // wavefronts per workgroup

struct OutRing {
  uintptr_t dst;      // block output in global memory
  lds_u8 *ring;
  uint32_t flushed;   // bytes [0, flushed) are in global memory
};

// copy output bytes [from, to) from the ring to global memory
__device__ __forceinline__ void ring_store(const OutRing &o, uint32_t from, uint32_t to, int lane) {
  uint32_t x = from;
  if (((o.dst + from) & 15u) == 0) {
    const uint32_t vend = from + ((to - from) & ~15u);
    for (uint32_t y = from + uint32_t(lane) * 16u; y < vend; y += 1024u)
      *(g_u32x4 *)(o.dst + y) = *(const lds_u32x4 *)(o.ring + (y & kRingMask));
    x = vend;
  }
  for (uint32_t y = x + uint32_t(lane); y < to; y += 64u) stb(o.dst + y, o.ring[y & kRingMask]);
}

// after output reached `op`: stream every complete 4 KiB piece
__device__ __forceinline__ void ring_advance(OutRing &o, uint32_t op, int lane) {
  while (op - o.flushed >= kFlush) {
    ring_store(o, o.flushed, o.flushed + kFlush, lane);
    o.flushed += kFlush;
  }
}

__device__ __forceinline__ void ring_finish(OutRing &o, uint32_t op, int lane) {
  ring_advance(o, op, lane);
  if (op > o.flushed) ring_store(o, o.flushed, op, lane);
  o.flushed = op;
}

// window bytes rel0 + lane (rel0 wave-uniform, rel0 + 64 <= 512): cross-lane
// gather of the dword holding each; nxt (possibly still in flight) is only
// touched when the range reaches it
__device__ __forceinline__ uint32_t win_gather(uint32_t rel0, uint32_t cur, uint32_t nxt, int lane) {
  const uint32_t rel = rel0 + uint32_t(lane);
  const uint32_t dw = rel >> 2;
  const int addr = int((dw & 63u) << 2);
  uint32_t v;
  if (rel0 + 63u < 256u) {
    v = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(cur)));
  } else if (rel0 >= 256u) {
    v = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(nxt)));
  } else {
    const uint32_t a = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(cur)));
    const uint32_t b = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(nxt)));
    v = dw < 64u ? a : b;
  }
  return (v >> (8u * (rel & 3u))) & 0xFFu;
}

// make the window cover input bytes [p, p+64) (p wave-uniform)
__device__ __forceinline__ void win_cover(InWin &w, uintptr_t p, int lane) {
  if (p >= w.base && p + 64u <= w.base + 512u) return;
  if (p >= w.base + 256u && p < w.base + 512u) {  // slide by 256, prefetching the next half
    w.base += 256u;
    w.cur = w.nxt;
    w.nxt = ld_dw(w.base + 256u + 4u * lane, w.lim);
  } else {
    win_load(w, p & ~uintptr_t(3), lane);
  }
}

// literal run: input [p, p+n) -> output [op, op+n) through the ring
__device__ __forceinline__ void ring_literals(OutRing &o, InWin &w, uintptr_t p, uint32_t op,
                                              uint32_t n, int lane) {
  for (uint32_t base = 0; base < n; base += 64u) {
    const uintptr_t q = p + base;
    win_cover(w, q, lane);
    const uint32_t v = win_gather(uint32_t(q - w.base), w.cur, w.nxt, lane);
    if (base + uint32_t(lane) < n) o.ring[(op + base + uint32_t(lane)) & kRingMask] = uint8_t(v);
    ring_advance(o, op + (n - base < 64u ? n : base + 64u), lane);
  }
}

// match: out[op+i] = out[op-off+i], i < len, with LZ77 overlap semantics
// (offset 0 writes zeros like the reference, lz4.c:2026).  GLOBAL: some
// source bytes are older than the ring (far offsets, or linked-block history
// in front of dst) and come from global memory; the LDS-only instantiation
// never waits on vector memory.
template <bool GLOBAL>
__device__ __forceinline__ void ring_match_t(OutRing &o, uint32_t op, uint32_t off, uint32_t len,
                                             int lane) {
  const bool far = GLOBAL && off > kRingReach;
  const long back = long(op) - long(off);
  auto rd = [&](long q) -> uint32_t {
    if (GLOBAL && (far || q < 0)) return ldb(o.dst + q);
    return uint32_t(o.ring[uint32_t(q) & kRingMask]);
  };
  if (off == 0) {
    for (uint32_t base = 0; base < len; base += 64u) {
      if (base + uint32_t(lane) < len) o.ring[(op + base + uint32_t(lane)) & kRingMask] = 0;
      ring_advance(o, op + (len - base < 64u ? len : base + 64u), lane);
    }
  } else if (off < 64u) {  // small period: each 64-byte step reads the off bytes before it
    const uint32_t lm = uint32_t(lane) % off;
    for (uint32_t base = 0; base < len; base += 64u) {
      const uint32_t v = rd(back + long(base) + long(lm));
      if (base + uint32_t(lane) < len) o.ring[(op + base + uint32_t(lane)) & kRingMask] = uint8_t(v);
      ring_advance(o, op + (len - base < 64u ? len : base + 64u), lane);
    }
  } else {  // steps of min(off, 256) never read bytes written in the same step
    const uint32_t step = off >= 256u ? 256u : 64u;
    for (uint32_t base = 0; base < len; base += step) {
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = base + uint32_t(lane) + 64u * j;
        v[j] = (64u * j < step && i < len) ? rd(back + long(i)) : 0u;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = base + uint32_t(lane) + 64u * j;
        if (64u * j < step && i < len) o.ring[(op + i) & kRingMask] = uint8_t(v[j]);
      }
      ring_advance(o, op + (len - base < step ? len : base + step), lane);
    }
  }
}

__device__ __forceinline__ void ring_match(OutRing &o, uint32_t op, uint32_t off, uint32_t len,
                                           int lane) {
  if (off <= kRingReach && off <= op) {
    ring_match_t<false>(o, op, off, len, lane);
  } else {
    // flushed / previous-block output is read back by this same wavefront: a
    // workgroup-scope fence (wait for its stores) suffices -- __threadfence()
    // would write back the whole L2 for cross-XCD coherence
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    ring_match_t<true>(o, op, off, len, lane);
  }
}

// ---------------------------------------------------------- block decoder
// Returns decoded size, -1 for a block the reference rejects, -2 when the
// caller's buffer (realcap) is too small.  `hist` = bytes of frame history
// directly in front of dst (linked frames), selecting noDict /
// withSmallPrefix / withPrefix64k exactly like LZ4_decompress_safe_usingDict.
__device__ int decode_block(uintptr_t src, int csize, OutRing &o, int vcap, int realcap,
                            int hist, int lane) {
  const int iend = csize, oend = vcap;
  const bool prefix64k = hist >= 65535;
  const long lowPrefix = hist <= 0 ? 0L : (prefix64k ? -65536L : -long(hist));
  InWin w;
  w.lim = (src + uintptr_t(csize) + 3u) & ~uintptr_t(3);
  win_load(w, src & ~uintptr_t(3), lane);
#define RDK_B(i) win_byte(w, src + uintptr_t(i), lane)
  int ip = 0, op = 0, cpy = 0;
  uint32_t token, length;
  long match, offset;

  if (oend == 0) return (csize == 1 && RDK_B(0) == 0) ? 0 : -1;
  if (csize == 0) return -1;

  // read_variable_length (lz4.c:1625): -1 initial error, -2 loop error
  auto rvl = [&](int lencheck, bool initial_check, uint32_t &len) -> int {
    uint32_t acc = 0, b;
    if (initial_check && ip >= lencheck) { len = 0; return -1; }
    do {
      b = RDK_B(ip);
      ip++;
      acc += b;
      if (ip >= lencheck) { len = acc; return -2; }
    } while (b == 255u);
    len = acc;
    return 0;
  };
  auto lit = [&](uint32_t n) -> bool {
    if (op + int(n) > realcap) return false;
    ring_literals(o, w, src + uintptr_t(ip), uint32_t(op), n, lane);
    return true;
  };
  auto mat = [&](uint32_t n) -> bool {
    if (op + int(n) > realcap) return false;
    ring_match(o, uint32_t(op), uint32_t(offset), n, lane);
    return true;
  };

  if (oend - op < kFastloopSafeDistance) goto safe_decode;
  for (;;) {  // fast loop (lz4.c:1712-1824)
    token = RDK_B(ip);
    ip++;
    length = token >> 4;
    if (length == 15u) {
      uint32_t add;
      if (rvl(iend - 15, true, add) == -1) return -1;
      length += add;
      cpy = op + int(length);
      if (cpy > oend - 32 || ip + int(length) > iend - 32) goto safe_literal_copy;
      if (!lit(length)) return -2;
      ip += int(length);
      op = cpy;
    } else {
      cpy = op + int(length);
      if (ip > iend - (16 + 1)) goto safe_literal_copy;
      if (!lit(length)) return -2;
      ip += int(length);
      op = cpy;
    }
    offset = long(RDK_B(ip)) | (long(RDK_B(ip + 1)) << 8);
    ip += 2;
    match = op - offset;
    length = token & 15u;
    if (length == 15u) {
      uint32_t add;
      if (match < lowPrefix) return -1;
      if (rvl(iend - kLz4LastLiterals + 1, false, add) != 0) return -1;
      length += add + kLz4MinMatch;
      if (op + int(length) >= oend - kFastloopSafeDistance) goto safe_match_copy;
    } else {
      length += kLz4MinMatch;
      if (op + int(length) >= oend - kFastloopSafeDistance) goto safe_match_copy;
      if ((prefix64k || match >= lowPrefix) && offset >= 8) {
        if (!mat(length)) return -2;
        op += int(length);
        continue;
      }
    }
    if (match < lowPrefix) return -1;
    if (!mat(length)) return -2;
    op += int(length);
  }

safe_decode:
  for (;;) {  // safe loop (lz4.c:1827-2053)
    token = RDK_B(ip);
    ip++;
    length = token >> 4;
    if (length != 15u && ip < iend - 16 && op <= oend - 32) {  // shortcut
      if (!lit(length)) return -2;
      op += int(length);
      ip += int(length);
      length = token & 15u;
      offset = long(RDK_B(ip)) | (long(RDK_B(ip + 1)) << 8);
      ip += 2;
      match = op - offset;
      if (length != 15u && offset >= 8 && (prefix64k || match >= lowPrefix)) {
        if (!mat(length + kLz4MinMatch)) return -2;
        op += int(length) + kLz4MinMatch;
        continue;
      }
      goto copy_match_len;
    }
    if (length == 15u) {
      uint32_t add;
      if (rvl(iend - 15, true, add) == -1) return -1;
      length += add;
    }
    cpy = op + int(length);
  safe_literal_copy:
    if (cpy > oend - kLz4MFLimit || ip + int(length) > iend - (2 + 1 + kLz4LastLiterals)) {
      if (ip + int(length) != iend || cpy > oend) return -1;
      if (!lit(length)) return -2;
      ip += int(length);
      op += int(length);
      break;
    }
    if (!lit(length)) return -2;
    ip += int(length);
    op = cpy;
    offset = long(RDK_B(ip)) | (long(RDK_B(ip + 1)) << 8);
    ip += 2;
    match = op - offset;
    length = token & 15u;
  copy_match_len:
    if (length == 15u) {
      uint32_t add;
      if (rvl(iend - kLz4LastLiterals + 1, false, add) != 0) return -1;
      length += add;
    }
    length += kLz4MinMatch;
  safe_match_copy:
    if (match < lowPrefix) return -1;
    cpy = op + int(length);
    if (cpy > oend - kLz4LastLiterals) return -1;
    if (!mat(length)) return -2;
    op = cpy;
  }
#undef RDK_B
  ring_finish(o, uint32_t(op), lane);
  return op;
}

#include "lz4_decode_fast.h"

// ------------------------------------------------------------ kernels
struct DevReader {
  uintptr_t p;
  __device__ uint32_t operator()(uint64_t i) const { return ldb(p + i); }
};

// Also appends the (frame, block) items of every regular frame to a compact
// work list, so the block kernel's wavefronts only ever see real blocks.
__global__ void lz4f_walk_kernel(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
                                 const uint32_t *__restrict__ in_lens,
                                 const uint32_t *__restrict__ out_caps, uint32_t n,
                                 FrameState *__restrict__ fs, BlockDesc *__restrict__ bd,
                                 uint32_t *__restrict__ work_count, uint32_t *__restrict__ work) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  FrameWalker<DevReader> wk{DevReader{reinterpret_cast<uintptr_t>(in) + in_offs[f]}, in_lens[f]};
  wk.header();
  BlockInfo b;
  uint32_t k = 0;
  uint64_t last_most = 0;
  while (wk.next(b)) {
    if (k < uint32_t(kMaxDesc)) {
      bd[size_t(f) * kMaxDesc + k].b = b;
      bd[size_t(f) * kMaxDesc + k].result = 0;
    }
    last_most = lz4f_block_most(b, wk.fi.max_block);
    ++k;
  }
  wk.fi.nblocks = k < uint32_t(kMaxDesc) ? k : uint32_t(kMaxDesc);
  if ((wk.fi.flags & F_LINKED) || k > uint32_t(kMaxDesc)) wk.fi.flags |= F_SEQ;
  // Independent blocks decode in place at k * max_block, each within what is left of the
  // capacity from there (a frame of full blocks fits a capacity equal to its decoded size).
  // A capacity that ends before the last block's place -- a caller that sized the output
  // from what the blocks can yield, for a frame of many short blocks -- cannot hold that
  // layout: such a frame is decoded in stream order by one wavefront instead.
  (void)last_most;
  if (k && uint64_t(k - 1) * wk.fi.max_block >= out_caps[f]) wk.fi.flags |= F_SEQ;
  fs[f].fi = wk.fi;
  fs[f].seq_result = 0;
  if (wk.fi.status == 0 && !(wk.fi.flags & (F_SKIPPABLE | F_SEQ)) && wk.fi.nblocks) {
    const uint32_t at = atomicAdd(work_count, wk.fi.nblocks);
    for (uint32_t j = 0; j < wk.fi.nblocks; ++j) work[at + j] = f * uint32_t(kMaxDesc) + j;
  }
}

// one block: raw copy or LZ4 decode, with the block checksum check first
// (dstage_getCBlock verifies XXH32 before decoding, lz4frame.c:1596-1608)
__device__ int run_block(const BlockInfo &b, uintptr_t frame, uintptr_t dst, uint32_t max_block,
                         int realcap, int hist, lds_u8 *ring, lds_u8 *map, int lane) {
  const uintptr_t src = frame + b.src_off;
  if (b.flags & B_RAW) {
    if (int(b.csize) > realcap) return -2;
    copy_fwd(dst, src, b.csize, lane);
    if (b.flags & B_XXH) {
      uint32_t h = lane == 0 ? xxh32_lane(src, b.csize, 0) : 0u;
      if (uni(h) != b.xxh) return -1;
    }
    return int(b.csize);
  }
  if (b.flags & B_XXH) {
    uint32_t h = lane == 0 ? xxh32_lane(src, b.csize, 0) : 0u;
    if (uni(h) != b.xxh) return -1;
  }
  if (hist == 0 && !(b.flags & B_TRUNC) && realcap >= 0) {
    const int r =
        decode_block_fast(src, b.csize, dst, max_block, uint32_t(realcap), ring, map, lane);
    if (r != kFastFallback) return r;
#ifdef RDK_DEC_DEBUG
    if (lane == 0) printf("fallback src_off %u csize %u\n", b.src_off, b.csize);
#endif
  }
  OutRing o{dst, ring, 0u};
  return decode_block(src, int(b.csize), o, int(max_block), realcap, hist, lane);
}

__device__ __forceinline__ int realcap_at(uint64_t cap, uint64_t at, uint32_t limit) {
  if (cap <= at) return 0;
  const uint64_t r = cap - at;
  return int(r < limit ? r : limit);
}

// independent blocks of regular frames: one wavefront per (frame, block)
__global__ __launch_bounds__(64 * kDecWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void
lz4f_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs, uint8_t *out,
    const uint64_t *__restrict__ out_offs, const uint32_t *__restrict__ out_caps, uint32_t n,
    const FrameState *__restrict__ fs, BlockDesc *__restrict__ bd,
    const uint32_t *__restrict__ work_count, const uint32_t *__restrict__ work) {
  __shared__ __attribute__((aligned(kRing))) uint8_t rings[kDecWaves][kRing];  // (ring_at)
  __shared__ __attribute__((aligned(16))) uint8_t maps[kDecWaves][128];
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  lds_u8 *ring = (lds_u8 *)rings[uni(threadIdx.x >> 6)];
  lds_u8 *map = (lds_u8 *)maps[uni(threadIdx.x >> 6)];
  const uint32_t gw = blockIdx.x * wpb + uni(threadIdx.x >> 6);
  const uint32_t items = uni(*work_count);
  (void)n;
  for (uint32_t it = gw; it < items; it += gridDim.x * wpb) {
    const uint32_t wi = uni(work[it]);
    const uint32_t f = wi / uint32_t(kMaxDesc), k = wi % uint32_t(kMaxDesc);
    const uint32_t mb = uni(fs[f].fi.max_block);
    const uintptr_t frame = reinterpret_cast<uintptr_t>(in) + in_offs[f];
    const uintptr_t obase = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    BlockInfo b = bd[size_t(f) * kMaxDesc + k].b;
    b.src_off = uni(b.src_off); b.csize = uni(b.csize); b.flags = uni(b.flags); b.xxh = uni(b.xxh);
    const uint64_t slot = uint64_t(k) * mb;
    const int r = run_block(b, frame, obase + slot, mb, realcap_at(out_caps[f], slot, mb), 0, ring,
                            map, lane);
    if (lane == 0) bd[size_t(f) * kMaxDesc + k].result = r;
  }
}

// linked frames and frames with more than kMaxDesc blocks: one wavefront
// decodes the whole frame in stream order into contiguous output
__global__ __launch_bounds__(64 * kDecWaves) void lz4f_seq_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *out, const uint64_t *__restrict__ out_offs,
    const uint32_t *__restrict__ out_caps, uint32_t n, FrameState *__restrict__ fs) {
  __shared__ __attribute__((aligned(kRing))) uint8_t rings[kDecWaves][kRing];  // (ring_at)
  __shared__ __attribute__((aligned(16))) uint8_t maps[kDecWaves][128];
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  lds_u8 *ring = (lds_u8 *)rings[uni(threadIdx.x >> 6)];
  lds_u8 *map = (lds_u8 *)maps[uni(threadIdx.x >> 6)];
  const uint32_t gw = blockIdx.x * wpb + uni(threadIdx.x >> 6);
  for (uint32_t f = gw; f < n; f += gridDim.x * wpb) {
    const uint32_t status = uni(uint32_t(fs[f].fi.status));
    const uint32_t flags = uni(fs[f].fi.flags);
    if (status != 0 || (flags & F_SKIPPABLE) || !(flags & F_SEQ)) continue;
    const uintptr_t frame = reinterpret_cast<uintptr_t>(in) + in_offs[f];
    const uintptr_t obase = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    const uint64_t cap = out_caps[f];
    FrameWalker<DevReader> wk{DevReader{frame}, in_lens[f]};
    wk.header();
    const uint32_t mb = uni(wk.fi.max_block);
    const bool linked = flags & F_LINKED;
    uint64_t produced = 0;
    int32_t res = 0;
    BlockInfo b;
    while (wk.next(b)) {
      b.src_off = uni(b.src_off); b.csize = uni(b.csize); b.flags = uni(b.flags); b.xxh = uni(b.xxh);
      const int hist = linked ? int(produced < 65536u ? produced : 65536u) : 0;
      const int r = run_block(b, frame, obase + produced, mb, realcap_at(cap, produced, mb), hist,
                              ring, map, lane);
      if (r < 0) { res = r; break; }
      produced += uint64_t(r);
    }
    if (lane == 0) fs[f].seq_result = res < 0 ? res : int32_t(produced);
  }
}

// frame-level verdict + compaction of irregular frames, one wavefront per frame
__global__ __launch_bounds__(256) void lz4f_finish_kernel(
    uint8_t *out, const uint64_t *__restrict__ out_offs, uint32_t n,
    const FrameState *__restrict__ fs, const BlockDesc *__restrict__ bd,
    uint32_t *__restrict__ out_lens, int32_t *__restrict__ st) {
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + uni(threadIdx.x >> 6);
  for (uint32_t f = gw; f < n; f += gridDim.x * wpb) {
    const FrameInfo fi = fs[f].fi;
    int32_t status = int32_t(uni(uint32_t(fi.status)));
    const uint32_t flags = uni(fi.flags);
    uint64_t total = 0;
    const uintptr_t obase = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    if (status == 0 && !(flags & F_SKIPPABLE)) {
      if (flags & F_SEQ) {
        const int32_t r = int32_t(uni(uint32_t(fs[f].seq_result)));
        if (r < 0) status = (r == -2) ? kErrDstSize : kErrBadCompression;
        else total = uint32_t(r);
      } else {
        const uint32_t nb = uni(fi.nblocks), mb = uni(fi.max_block);
        bool regular = true;
        for (uint32_t k = 0; k < nb && status == 0; ++k) {
          const int32_t r = int32_t(uni(uint32_t(bd[size_t(f) * kMaxDesc + k].result)));
          if (r < 0) { status = (r == -2) ? kErrDstSize : kErrBadCompression; break; }
          if (k + 1 < nb && uint32_t(r) != mb) regular = false;
          total += uint32_t(r);
        }
        if (status == 0 && !regular) {  // memmove blocks down into stream order
          uint64_t at = 0;
          for (uint32_t k = 0; k < nb; ++k) {
            const uint32_t r = uni(uint32_t(bd[size_t(f) * kMaxDesc + k].result));
            const uint64_t from = uint64_t(k) * mb;
            if (from != at) {
              for (uint32_t base = 0; base < r; base += 256u) {
                uint32_t v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  const uint32_t i = base + lane + 64u * j;
                  v[j] = i < r ? ldb(obase + from + i) : 0u;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  const uint32_t i = base + lane + 64u * j;
                  if (i < r) stb(obase + at + i, v[j]);
                }
                asm volatile("" ::: "memory");
              }
            }
            at += r;
          }
        }
      }
      if (status == 0 && (flags & F_ENDMARK)) {  // dstage_getSuffix (lz4frame.c:1694-1731)
        if ((flags & F_CSIZE) && total != fi.content_size) status = kErrBadCompression;
        else if (flags & F_CCHK_PRESENT) {
          asm volatile("" ::: "memory");
          uint32_t h = lane == 0 ? xxh32_lane(obase, total, 0) : 0u;
          if (uni(h) != fi.content_xxh) status = kErrBadCompression;
        }
      }
      if (status == 0 && (flags & F_TRAILING)) status = kErrBadMsg;  // rdkafka_lz4.c:291
    }
    if (lane == 0) {
      out_lens[f] = status == 0 ? uint32_t(total) : 0u;
      st[f] = status;
    }
  }
}

// ------------------------------------------------------------ host side
static unsigned grid_waves(uint64_t waves, uint32_t wpb) {
  uint64_t b = (waves + wpb - 1) / wpb;
  if (b > 8192u) b = 8192u;
  return b ? unsigned(b) : 1u;
}

void launch_decode(uint8_t *scratch, const uint8_t *d_in, const uint64_t *d_in_offs,
                   const uint32_t *d_in_lens, uint8_t *d_out, const uint64_t *d_out_offs,
                   const uint32_t *d_out_caps, uint32_t *d_out_lens, int32_t *d_status,
                   uint32_t n, hipStream_t s);

int lz4f_decompress_device(Ctx *c, const uint8_t *d_in, const uint64_t *d_in_offs,
                           const uint32_t *d_in_lens, uint8_t *d_out,
                           const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                           uint32_t *d_out_lens, int32_t *d_status, uint32_t n, hipStream_t s) {
  if (!n) return 0;
  const size_t fs_bytes = (size_t(n) * sizeof(FrameState) + 255) & ~size_t(255);
  const size_t bd_bytes = size_t(n) * kMaxDesc * sizeof(BlockDesc);
  const size_t wk_bytes = 256 + size_t(n) * kMaxDesc * sizeof(uint32_t);
  int rc = scratch_acquire(c, kScratchDecode, fs_bytes + bd_bytes + wk_bytes, s);
  if (rc) return rc;
  uint8_t *scratch = c->d_stage[kScratchDecode];
  RDK_HIP_CHECK(hipMemsetAsync(scratch + fs_bytes + bd_bytes, 0, sizeof(uint32_t), s));
  launch_decode(scratch, d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_caps, d_out_lens,
                d_status, n, s);
  RDK_HIP_CHECK(hipGetLastError());
  return scratch_release(c, kScratchDecode, s);
}

// The four kernels of one batch decode on stream s.  `scratch` holds the FrameState
// array, the BlockDesc table and the work list, laid out as decode_scratch_bytes(n)
// says; its work counter (the word after the BlockDesc table) must be zero.
size_t decode_scratch_bytes(uint32_t n) {
  const size_t fs_bytes = (size_t(n) * sizeof(FrameState) + 255) & ~size_t(255);
  const size_t bd_bytes = size_t(n) * kMaxDesc * sizeof(BlockDesc);
  return fs_bytes + bd_bytes + 256 + size_t(n) * kMaxDesc * sizeof(uint32_t);
}

void launch_decode(uint8_t *scratch, const uint8_t *d_in, const uint64_t *d_in_offs,
                   const uint32_t *d_in_lens, uint8_t *d_out, const uint64_t *d_out_offs,
                   const uint32_t *d_out_caps, uint32_t *d_out_lens, int32_t *d_status,
                   uint32_t n, hipStream_t s) {
  const size_t fs_bytes = (size_t(n) * sizeof(FrameState) + 255) & ~size_t(255);
  const size_t bd_bytes = size_t(n) * kMaxDesc * sizeof(BlockDesc);
  FrameState *fs = reinterpret_cast<FrameState *>(scratch);
  BlockDesc *bd = reinterpret_cast<BlockDesc *>(scratch + fs_bytes);
  uint32_t *work_count = reinterpret_cast<uint32_t *>(scratch + fs_bytes + bd_bytes);
  uint32_t *work = work_count + 64;
  hipLaunchKernelGGL(lz4f_walk_kernel, dim3((n + 63) / 64), dim3(64), 0, s, d_in, d_in_offs,
                     d_in_lens, d_out_caps, n, fs, bd, work_count, work);
  // persistent grid: as many workgroups per CU as the LDS rings and the 32 wave slots allow
  constexpr unsigned kWgPerCu = (160u * 1024u) / (kDecWaves * (kRing + 128u)) < 32u / kDecWaves
                                    ? (160u * 1024u) / (kDecWaves * (kRing + 128u))
                                    : 32u / kDecWaves;
  const uint64_t want = (uint64_t(n) * kMaxDesc + kDecWaves - 1) / kDecWaves;
  const unsigned cap = 256u * kWgPerCu;
  const unsigned bgrid = unsigned(want < cap ? (want ? want : 1u) : cap);
  hipLaunchKernelGGL(lz4f_blocks_kernel, dim3(bgrid), dim3(64 * kDecWaves), 0, s, d_in,
                     d_in_offs, d_out, d_out_offs, d_out_caps, n, fs, bd, work_count, work);
  hipLaunchKernelGGL(lz4f_seq_kernel, dim3(grid_waves(n, 4)), dim3(256), 0, s, d_in, d_in_offs,
                     d_in_lens, d_out, d_out_offs, d_out_caps, n, fs);
  hipLaunchKernelGGL(lz4f_finish_kernel, dim3(grid_waves(n, 4)), dim3(256), 0, s, d_out,
                     d_out_offs, n, fs, bd, d_out_lens, d_status);
}

// ------------------------------------------------ allocation-free variant
// The same four kernels on a scratch buffer that is part of the code object, for callers
// that cannot allocate (HIP graph capture, tight serving loops).  One array per GPU, held
// until the process ends; every call on a GPU shares it, so calls that overlap on one GPU
// race.  The host never passes the array's name to a kernel: its per-device address is
// looked up once, at rdk_hip_init(), and that pointer is what the launches use.
constexpr size_t noalloc_scratch_bytes(uint32_t n) {
  return ((size_t(n) * sizeof(FrameState) + 255) & ~size_t(255)) +
         size_t(n) * kMaxDesc * sizeof(BlockDesc) + 256 + size_t(n) * kMaxDesc * sizeof(uint32_t);
}
constexpr size_t kNoAllocBytes = noalloc_scratch_bytes(RDK_HIP_LZ4F_NOALLOC_MAX_FRAMES);
static_assert(kNoAllocBytes <= (4u << 20), "the static scratch is meant to stay modest");
static __device__ __align__(256) uint8_t scratch[kNoAllocBytes];

namespace {
constexpr int kNoAllocMaxDev = 64;
uint8_t *g_noalloc_ptr[kNoAllocMaxDev];  // per device: that GPU's copy of `scratch`
}  // namespace

// Called by rdk_hip_init() with `dev` current.
int lz4f_noalloc_setup(int dev) {
  if (dev < 0 || dev >= kNoAllocMaxDev) return set_error(RDK_HIP_E_INVAL, "device %d", dev);
  if (__atomic_load_n(&g_noalloc_ptr[dev], __ATOMIC_ACQUIRE)) return 0;
  uint8_t *ptr = nullptr;
  RDK_HIP_CHECK(hipGetSymbolAddress(reinterpret_cast<void **>(&ptr), HIP_SYMBOL(scratch)));
  if (!ptr) return set_error(RDK_HIP_E_HIP, "hipGetSymbolAddress(scratch) returned null");
  __atomic_store_n(&g_noalloc_ptr[dev], ptr, __ATOMIC_RELEASE);
  return 0;
}

// a kernel, not hipMemsetAsync: the call may be recorded into a HIP graph
__global__ void lz4f_zero_word_kernel(uint32_t *p) { *p = 0u; }

}  // namespace rdk

using namespace rdk;

RDK_API int rdk_hip_lz4f_decompress_noalloc(const void *d_in, const uint64_t *d_in_offs,
                                            const uint32_t *d_in_lens, void *d_out,
                                            const uint64_t *d_out_offs,
                                            const uint32_t *d_out_caps, uint32_t *d_out_lens,
                                            int32_t *d_status, uint32_t n, void *stream) {
  if (!n) return RDK_HIP_OK;
  if (n > RDK_HIP_LZ4F_NOALLOC_MAX_FRAMES)
    return set_error(RDK_HIP_E_INVAL, "%u frames exceed RDK_HIP_LZ4F_NOALLOC_MAX_FRAMES (%u)", n,
                     unsigned(RDK_HIP_LZ4F_NOALLOC_MAX_FRAMES));
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_caps || !d_out_lens ||
      !d_status)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  int dev = -1;
  RDK_HIP_CHECK(hipGetDevice(&dev));
  uint8_t *ptr = (dev >= 0 && dev < kNoAllocMaxDev)
                     ? __atomic_load_n(&g_noalloc_ptr[dev], __ATOMIC_ACQUIRE) : nullptr;
  if (!ptr)
    return set_error(RDK_HIP_E_INVAL, "rdk_hip_init(%d) has not run: no scratch address for this device", dev);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // the work counter sits behind the FrameState and BlockDesc tables of THIS call's n
  const size_t counter_at = noalloc_scratch_bytes(n) - 256 - size_t(n) * kMaxDesc * sizeof(uint32_t);
  hipLaunchKernelGGL(lz4f_zero_word_kernel, dim3(1), dim3(1), 0, s,
                     reinterpret_cast<uint32_t *>(ptr + counter_at));
  launch_decode(ptr, static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                static_cast<uint8_t *>(d_out), d_out_offs, d_out_caps, d_out_lens, d_status, n, s);
  RDK_HIP_CHECK(hipGetLastError());
  return RDK_HIP_OK;
}

RDK_API int rdk_hip_lz4f_decompress(const void *d_in, const uint64_t *d_in_offs,
                                    const uint32_t *d_in_lens, void *d_out,
                                    const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                                    uint32_t *d_out_lens, int32_t *d_status, uint32_t n,
                                    void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_caps || !d_out_lens ||
      !d_status)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  return lz4f_decompress_device(c, static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                static_cast<uint8_t *>(d_out), d_out_offs, d_out_caps, d_out_lens,
                                d_status, n, s);
}
