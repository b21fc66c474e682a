// lz4_encode.hip -- LZ4F frame compression on gfx950.
//
// Replaces rd_kafka_lz4_compress (src/rdkafka_lz4.c:329-442) ->
// LZ4F_compressUpdate/End (lz4frame.c:823-1018) -> LZ4F_makeBlock (:739) ->
// LZ4_compress_fast_extState_fastReset (lz4.c:1211) -> LZ4_compress_generic
// (lz4.c:789-1177, byU16 table, limitedOutput, dstCapacity = srcSize-1).
//
// One wavefront (one 64-thread workgroup) per independent 64 KiB block with
// its own 8192-entry u16 hash table in LDS (16 KiB -> 10 blocks per CU).  The
// greedy parse is emulated EXACTLY, so frames are byte-identical to the
// reference's:
//   * the match search evaluates 64 consecutive probe positions at once
//     (the skip schedule step = searchMatchNb++ >> 6 is reproduced by a lane
//     prefix-sum); each lane's candidate is the latest earlier probe with the
//     same hash (13 ballots, one per hash bit) or else the table entry; the
//     first verifying lane wins and only probes up to it update the table,
//     last-writer-per-hash, as the sequential loop would;
//   * catch-up, LZ4_count and literal copies compare / move 64 bytes per step;
//   * the limitedOutput checks of lz4.c:961-1160 are applied verbatim, so a
//     block that does not fit in srcSize-1 bytes is stored raw (bit 31) like
//     LZ4F_makeBlock does.
// Blocks are written into worst-case slots of the caller's frame buffer;
// lz4f_assemble_kernel then writes the frame header / size words / end mark
// and slides the blocks down into stream order.
#include <hip/hip_runtime.h>

#include "common.h"
#include "lz4_device.h"

namespace rdk {

constexpr int kEncMaxItems = 64;           // block slots per frame per pass
constexpr uint32_t kSlot = kLz4Block + 4;  // worst-case bytes per block in a frame
constexpr uint32_t kHashLog = 13;          // LZ4_HASHLOG+1 for byU16 (lz4.c:633)

typedef __attribute__((address_space(3))) uint16_t lds_u16;

__device__ __forceinline__ uint32_t lz4_hash(uint32_t seq) {  // LZ4_hash4, lz4.c:631
  return (seq * 2654435761u) >> (32 - kHashLog);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d);
    if (lane >= d) v += t;
  }
  return v;
}

// number of equal bytes a[i]==b[i] for i in [0, limit), 64 per step
__device__ __forceinline__ int wave_count(uintptr_t a, uintptr_t b, int limit, int lane) {
  int cnt = 0;
  while (cnt < limit) {
    const int l = cnt + lane;
    const bool ok = l < limit && ldb(a + l) == ldb(b + l);
    const uint64_t m = ballot(ok);
    const int run = m == ~0ull ? 64 : __builtin_ctzll(~m);
    cnt += run;
    if (run < 64) break;
  }
  return cnt;
}

// catch-up: equal bytes walking backwards from a-1 / b-1, at most limit
__device__ __forceinline__ int wave_count_back(uintptr_t a, uintptr_t b, int limit, int lane) {
  int cnt = 0;
  while (cnt < limit) {
    const int l = cnt + lane;
    const bool ok = l < limit && ldb(a - 1 - l) == ldb(b - 1 - l);
    const uint64_t m = ballot(ok);
    const int run = m == ~0ull ? 64 : __builtin_ctzll(~m);
    cnt += run;
    if (run < 64) break;
  }
  return cnt;
}

__device__ __forceinline__ void wave_copy(uintptr_t d, uintptr_t s, uint32_t len, int lane) {
  for (uint32_t base = 0; base < len; base += 256u) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + lane + 64u * j;
      v[j] = i < len ? ldb(s + i) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + lane + 64u * j;
      if (i < len) stb(d + i, v[j]);
    }
  }
}

// n bytes of 255 followed by one `rest` byte at d (length extension bytes)
__device__ __forceinline__ void put_run(uintptr_t d, uint32_t n255, uint32_t rest, int lane) {
  for (uint32_t i = lane; i < n255; i += 64u) stb(d + i, 255u);
  if (lane == 0) stb(d + n255, rest);
}

// LZ4_compress_generic(byU16, limitedOutput, noDict, noDictIssue), table
// already zeroed.  Returns compressed size, or 0 if it does not fit in n-1.
__device__ int compress_block(uintptr_t src, int n, uintptr_t dst, int accel, lds_u16 *table,
                              int lane) {
  const int mflimitPlusOne = n - kLz4MFLimit + 1;  // lz4.c:821
  const int matchlimit = n - kLz4LastLiterals;     // lz4.c:822
  const int olimit = n - 1;                        // LZ4F_makeBlock dstCapacity
  const uint32_t A64 = uint32_t(accel) << 6;       // searchMatchNb start
  int ip = 1, anchor = 0, op = 0, match = 0;

  // position 0 hashes to the zero entry it already holds (lz4.c:879)
  for (;;) {
    // ------------------------------------------------ find a match (lz4.c:909-957)
    {
      int fwd = ip;
      uint32_t cbase = 0;
      for (;;) {
        const uint32_t c = cbase + uint32_t(lane);
        const uint32_t s = (c == 0) ? 1u : ((A64 + c - 1u) >> 6);
        const uint32_t incl = wave_incl_scan(s, lane);
        const int P = fwd + int(incl - s);
        const int Pn = fwd + int(incl);
        const bool valid = Pn <= mflimitPlusOne;
        const uint64_t vmask = ballot(valid);
        const uint32_t seq = valid ? ld32u(src + uint32_t(P)) : 0u;
        const uint32_t h = lz4_hash(seq);
        uint64_t eq = vmask;
#pragma unroll
        for (uint32_t bit = 0; bit < kHashLog; ++bit) {
          const bool hb = (h >> bit) & 1u;
          const uint64_t bm = ballot(hb);
          eq &= hb ? bm : ~bm;
        }
        const uint64_t lower = eq & ((1ull << lane) - 1ull);
        const int pred = lower ? 63 - __builtin_clzll(lower) : 0;
        const int predP = __shfl(P, pred);
        int cand = lower ? predP : int(table[h]);
        const bool m = valid && ld32u(src + uint32_t(cand)) == seq;
        const uint64_t mm = ballot(m);
        const int f = ffs64(mm);
        const int e = ffs64(~vmask);
        if (f < e) {
          const uint64_t upto = (2ull << f) - 1ull;
          const uint64_t later = eq & ~((2ull << lane) - 1ull) & upto;
          if (lane <= f && !later) table[h] = uint16_t(P);
          ip = __builtin_amdgcn_readlane(P, f);
          match = __builtin_amdgcn_readlane(cand, f);
          break;
        }
        if (e < 64) goto last_literals;  // forwardIp > mflimitPlusOne
        {
          const uint64_t later = eq & ~((2ull << lane) - 1ull);
          if (!later) table[h] = uint16_t(P);
        }
        fwd = __builtin_amdgcn_readlane(Pn, 63);
        cbase += 64u;
      }
    }
    // ------------------------------------------------ catch up (lz4.c:958-959)
    {
      const int lim = (ip - anchor) < match ? (ip - anchor) : match;
      const int back = wave_count_back(src + uint32_t(ip), src + uint32_t(match), lim, lane);
      ip -= back;
      match -= back;
    }
    uint32_t token_at, token;
    // ------------------------------------------------ literals (lz4.c:961-988)
    {
      const uint32_t litLength = uint32_t(ip - anchor);
      token_at = uint32_t(op++);
      if (op + int(litLength) + (2 + 1 + kLz4LastLiterals) + int(litLength / 255u) > olimit)
        return 0;
      if (litLength >= 15u) {
        const uint32_t len = litLength - 15u;
        put_run(dst + uint32_t(op), len / 255u, len % 255u, lane);
        op += int(len / 255u) + 1;
        token = 15u << 4;
      } else {
        token = litLength << 4;
      }
      wave_copy(dst + uint32_t(op), src + uint32_t(anchor), litLength, lane);
      op += int(litLength);
    }
    for (;;) {  // _next_match (lz4.c:990-1135)
      const uint32_t offset = uint32_t(ip - match);
      if (lane == 0) {
        stb(dst + uint32_t(op), offset & 0xFFu);
        stb(dst + uint32_t(op) + 1, offset >> 8);
      }
      op += 2;
      const int mc0 = wave_count(src + uint32_t(ip + kLz4MinMatch),
                                 src + uint32_t(match + kLz4MinMatch),
                                 matchlimit - (ip + kLz4MinMatch), lane);
      uint32_t matchCode = uint32_t(mc0);
      ip += mc0 + kLz4MinMatch;
      if (op + (1 + kLz4LastLiterals) + int((matchCode + 240u) / 255u) > olimit) return 0;
      if (matchCode >= 15u) {
        token += 15u;
        matchCode -= 15u;
        put_run(dst + uint32_t(op), matchCode / 255u, matchCode % 255u, lane);
        op += int(matchCode / 255u) + 1;
      } else {
        token += matchCode;
      }
      if (lane == 0) stb(dst + token_at, token);
      anchor = ip;
      if (ip >= mflimitPlusOne) goto last_literals;  // lz4.c:1081
      // fill table with ip-2, then test the next position (lz4.c:1084-1134)
      const uint32_t h2 = lz4_hash(ld32u(src + uint32_t(ip - 2)));
      if (lane == 0) table[h2] = uint16_t(ip - 2);
      const uint32_t seq = ld32u(src + uint32_t(ip));
      const uint32_t h = lz4_hash(seq);
      const int mi = int(uni(table[h]));
      if (lane == 0) table[h] = uint16_t(ip);
      if (ld32u(src + uint32_t(mi)) == seq) {
        token_at = uint32_t(op++);
        token = 0;
        match = mi;
        continue;
      }
      ip++;
      break;
    }
  }

last_literals : {  // lz4.c:1141-1166
  const uint32_t lastRun = uint32_t(n - anchor);
  if (op + int(lastRun) + 1 + int((lastRun + 255u - 15u) / 255u) > olimit) return 0;
  if (lastRun >= 15u) {
    if (lane == 0) stb(dst + uint32_t(op), 15u << 4);
    op++;
    const uint32_t acc = lastRun - 15u;
    put_run(dst + uint32_t(op), acc / 255u, acc % 255u, lane);
    op += int(acc / 255u) + 1;
  } else {
    if (lane == 0) stb(dst + uint32_t(op), lastRun << 4);
    op++;
  }
  wave_copy(dst + uint32_t(op), src + uint32_t(anchor), lastRun, lane);
  op += int(lastRun);
}
  return op;
}

// One wavefront per block.  Block k of frame f goes to the worst-case slot
// at out_offs[f] + 7 + k*kSlot as [LE32 size word][payload]; a block stored
// raw gets only its size word (payload is taken from the input later).
__global__ __launch_bounds__(64) void lz4_compress_blocks_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ out_offs, uint32_t n, int accel) {
  __shared__ __attribute__((aligned(16))) uint16_t table_mem[1u << kHashLog];
  lds_u16 *table = (lds_u16 *)table_mem;
  const int lane = threadIdx.x;
  const uint64_t items = uint64_t(n) * kEncMaxItems;
  for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const uint32_t f = uint32_t(it / kEncMaxItems), kk = uint32_t(it % kEncMaxItems);
    const uint32_t len = uni(in_lens[f]);
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    for (uint32_t k = kk; k < nb; k += kEncMaxItems) {
      const uint32_t bn = (len - k * kLz4Block) < kLz4Block ? (len - k * kLz4Block) : kLz4Block;
      const uintptr_t src = reinterpret_cast<uintptr_t>(in) + in_offs[f] + uint64_t(k) * kLz4Block;
      const uintptr_t slot = reinterpret_cast<uintptr_t>(out) + out_offs[f] + 7u + uint64_t(k) * kSlot;
      int csize = 0;
      if (bn >= uint32_t(kLz4MFLimit + 1)) {  // LZ4_minLength: shorter blocks never fit
        // LZ4_prepareTable: a fresh zeroed byU16 table per block (lz4.c:739-785)
        typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) u32x4e lds_u4;
        lds_u4 *t4 = (lds_u4 *)table_mem;
        const u32x4e z = {0u, 0u, 0u, 0u};
        for (int i = lane; i < int((2u << kHashLog) / 16u); i += 64) t4[i] = z;
        asm volatile("" ::: "memory");
        csize = compress_block(src, int(bn), slot + 4u, accel, table, lane);
      }
      if (lane == 0) {
        const uint32_t w = csize ? uint32_t(csize) : (bn | 0x80000000u);  // LZ4F_makeBlock
        stb(slot, w & 0xFFu); stb(slot + 1, (w >> 8) & 0xFFu);
        stb(slot + 2, (w >> 16) & 0xFFu); stb(slot + 3, w >> 24);
      }
    }
  }
}

// One workgroup per frame: header (lz4frame.c:671-701), size words, blocks
// slid down from their slots (raw blocks copied from the input), end mark.
__global__ __launch_bounds__(256) void lz4f_assemble_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_offs,
    const uint32_t *__restrict__ in_lens, uint8_t *out, const uint64_t *__restrict__ out_offs,
    uint32_t *__restrict__ out_lens, uint32_t n) {
  const int t = threadIdx.x;
  for (uint32_t f = blockIdx.x; f < n; f += gridDim.x) {
    const uint32_t len = in_lens[f];
    const uint32_t nb = (len + kLz4Block - 1) / kLz4Block;
    const uintptr_t ob = reinterpret_cast<uintptr_t>(out) + out_offs[f];
    const uintptr_t ib = reinterpret_cast<uintptr_t>(in) + in_offs[f];
    if (t == 0) {  // magic, FLG 0x60 (v01, independent), BD 0x40 (64 KB), HC 0x82
      stb(ob + 0, 0x04); stb(ob + 1, 0x22); stb(ob + 2, 0x4D); stb(ob + 3, 0x18);
      stb(ob + 4, 0x60); stb(ob + 5, 0x40); stb(ob + 6, 0x82);
    }
    uint64_t pos = 7;
    for (uint32_t k = 0; k < nb; ++k) {
      const uintptr_t slot = ob + 7u + uint64_t(k) * kSlot;
      const uint32_t w = ldb(slot) | (ldb(slot + 1) << 8) | (ldb(slot + 2) << 16) | (ldb(slot + 3) << 24);
      __syncthreads();  // everyone has read the size word before it may be overwritten
      const bool raw = w & 0x80000000u;
      const uint32_t sz = w & 0x7FFFFFFFu;
      const uintptr_t from = raw ? ib + uint64_t(k) * kLz4Block : slot + 4u;
      const uintptr_t to = ob + pos + 4u;
      if (from != to) {
        for (uint32_t base = 0; base < sz; base += 256u * 16u) {
          uint32_t v[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const uint32_t i = base + uint32_t(t) + 256u * j;
            v[j] = i < sz ? ldb(from + i) : 0u;
          }
          __syncthreads();  // chunk fully read before any lane writes (dst < src)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const uint32_t i = base + uint32_t(t) + 256u * j;
            if (i < sz) stb(to + i, v[j]);
          }
          __syncthreads();
        }
      }
      if (t == 0) {
        stb(ob + pos, w & 0xFFu); stb(ob + pos + 1, (w >> 8) & 0xFFu);
        stb(ob + pos + 2, (w >> 16) & 0xFFu); stb(ob + pos + 3, w >> 24);
      }
      __syncthreads();
      pos += 4u + sz;
    }
    if (t == 0) {
      stb(ob + pos, 0); stb(ob + pos + 1, 0); stb(ob + pos + 2, 0); stb(ob + pos + 3, 0);
      out_lens[f] = uint32_t(pos + 4u);
    }
    __syncthreads();
  }
}

size_t lz4f_compress_bound(size_t len) {
  const size_t nb = (len + kLz4Block - 1) / kLz4Block;
  return 7u + nb * size_t(kSlot) + 4u;
}

void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s);

int lz4f_compress_device(Ctx *c, const uint8_t *d_in, const uint64_t *d_in_offs,
                         const uint32_t *d_in_lens, uint8_t *d_out, const uint64_t *d_out_offs,
                         uint32_t *d_out_lens, uint32_t n, int accel, hipStream_t s) {
  (void)c;
  if (!n) return 0;
  uint64_t items = uint64_t(n) * kEncMaxItems;
  const unsigned grid = unsigned(items < 2560u * 8u ? items : 2560u * 8u);
  hipLaunchKernelGGL(lz4_compress_blocks_kernel, dim3(grid), dim3(64), 0, s, d_in, d_in_offs,
                     d_in_lens, d_out, d_out_offs, n, accel);
  lz4f_assemble_launch(d_in, d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n, s);
  RDK_HIP_CHECK(hipGetLastError());
  return 0;
}

void lz4f_assemble_launch(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL(lz4f_assemble_kernel, dim3(n < 8192u ? n : 8192u), dim3(256), 0, s, d_in,
                     d_in_offs, d_in_lens, d_out, d_out_offs, d_out_lens, n);
}

int lz4f_compress_fast_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                              const uint32_t *d_in_lens, uint8_t *d_out,
                              const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                              hipStream_t s);
int lz4hc_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                          uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, int level, hipStream_t s);

}  // namespace rdk

using namespace rdk;

RDK_API size_t rdk_hip_lz4f_compress_bound(size_t len) { return lz4f_compress_bound(len); }

RDK_API int rdk_hip_lz4f_compress(const void *d_in, const uint64_t *d_in_offs,
                                  const uint32_t *d_in_lens, void *d_out,
                                  const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                                  int level, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (level >= 10)
    return set_error(RDK_HIP_E_INVAL, "LZ4HC optimal levels (>=10) are not implemented");
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_lens)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (level >= 3)  // LZ4F_selectCompression (lz4frame.c:797-805): LZ4HC hash chain
    return lz4hc_compress_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                 static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n, level, s);
  const int accel = level < 0 ? -level + 1 : 1;  // LZ4F_compressBlock, lz4frame.c:766
  return lz4f_compress_device(c, static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                              static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n, accel, s);
}

RDK_API int rdk_hip_lz4f_compress_fast(const void *d_in, const uint64_t *d_in_offs,
                                       const uint32_t *d_in_lens, void *d_out,
                                       const uint64_t *d_out_offs, uint32_t *d_out_lens,
                                       uint32_t n, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_in_offs || !d_in_lens || !d_out || !d_out_offs || !d_out_lens)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  return lz4f_compress_fast_device(static_cast<const uint8_t *>(d_in), d_in_offs, d_in_lens,
                                   static_cast<uint8_t *>(d_out), d_out_offs, d_out_lens, n,
                                   static_cast<hipStream_t>(stream));
}
