// records.hip -- MsgVersion 2 record serialisation and record index on gfx950.
//
// Replaces, for device-resident messages:
//   rd_kafka_msgset_writer_write_MessageSet_v2_header  rdkafka_msgset_writer.c:352-403
//   rd_kafka_msgset_writer_write_msg_v2                 rdkafka_msgset_writer.c:652-754
//   rd_kafka_msgset_writer_finalize_MessageSet_v2_header rdkafka_msgset_writer.c:1251-1295
//   (+ calc_crc_v2 :1229-1246 through rdk_hip_msgset_v2_crc FINALIZE)
// with the batch loop semantics of write_msgq (:804-902): OffsetDelta = index in
// the batch, TimestampDelta against the first message, MaxTimestamp from 0.
//
// Record index (rdkafka_msgset_reader.c:715-927): see v2_index_kernel.
//
// Workgroups of 256 threads work on chunks of 256 records (grid = chunks x batches):
//   sizes: a thread sizes one record (zig-zag varints, rdvarint.h:48-75), a chunk scan
//          plus a per-batch scan of chunk totals place it -> record offsets, batch size;
//   write: a thread writes its record's varints; key / value / header bytes are copied as
//          16-byte tasks, one per lane, by the whole workgroup (v2_write_kernel).
#include <hip/hip_runtime.h>

#include "common.h"
#include "specwalk.h"

#include <cstring>

namespace rdk {

struct Msgs {  // rdk_hip_msgs_t, by value
  const uint8_t *arena;
  const int64_t *ts;
  const uint64_t *key_off;
  const int32_t *key_len;
  const uint64_t *val_off;
  const int32_t *val_len;
  const uint64_t *hdr_off;
  const uint32_t *hdr_len;
  const int32_t *hdr_cnt;
};

struct Batch {  // rdk_hip_v2_batch_t
  uint32_t first_msg, msg_count;
  int64_t producer_id;
  int32_t base_sequence;
  int16_t producer_epoch;
  int16_t attributes;
};

__device__ __forceinline__ uint64_t zigzag(int64_t v) {
  return (uint64_t(v) << 1) ^ uint64_t(v >> 63);
}
// encoded size of an unsigned LEB128 value (rdvarint.h:48-63): at least one byte
__device__ __forceinline__ uint32_t vsize(uint64_t u) {
  const uint32_t bits = u ? 64u - uint32_t(__builtin_clzll(u)) : 1u;
  return (bits + 6u) / 7u;
}
// byte i of an n-byte LEB128 encoding of u
__device__ __forceinline__ uint32_t vbyte(uint64_t u, uint32_t i, uint32_t n) {
  return uint32_t((u >> (7u * i)) & 0x7fu) | (i + 1u < n ? 0x80u : 0u);
}

struct Rec {  // one record's fields (rdkafka_msgset_writer.c:684-716)
  uint64_t uL, uT, uO, uK, uV, uH;
  uint32_t sL, sT, sO, sK, sV, sH;
  uint32_t kb, vb, hb;
  uint32_t size;  // sL + MessageSize
};

__device__ __forceinline__ Rec rec_fields(const Msgs &m, uint32_t msg, uint32_t k, int64_t base_ts) {
  Rec r;
  const int32_t kl = m.key_len[msg], vl = m.val_len[msg];
  const int32_t hc = m.hdr_cnt ? m.hdr_cnt[msg] : 0;
  r.hb = m.hdr_len ? m.hdr_len[msg] : 0u;
  r.kb = kl > 0 ? uint32_t(kl) : 0u;
  r.vb = vl > 0 ? uint32_t(vl) : 0u;
  r.uT = zigzag(m.ts[msg] - base_ts);
  r.uO = zigzag(int64_t(k));
  r.uK = zigzag(kl);
  r.uV = zigzag(vl);
  r.uH = zigzag(hc);
  r.sT = vsize(r.uT);
  r.sO = vsize(r.uO);
  r.sK = vsize(r.uK);
  r.sV = vsize(r.uV);
  r.sH = vsize(r.uH);
  const uint32_t msz = 1u + r.sT + r.sO + r.sK + r.kb + r.sV + r.vb + r.sH + r.hb;  // :703
  r.uL = zigzag(int64_t(msz));
  r.sL = vsize(r.uL);
  r.size = r.sL + msz;
  return r;
}

constexpr int kRecBlock = 256;  // records per chunk = threads per workgroup

// ---- sizes, 1/3: per chunk of 256 records: sizes, chunk-local exclusive offsets,
// chunk total and chunk MaxTimestamp.  grid (chunks, batches)
__global__ __launch_bounds__(kRecBlock) void v2_chunk_kernel(Msgs m, const Batch *__restrict__ batches,
                                                            uint32_t nchunk,
                                                            uint32_t *__restrict__ rec_offs,
                                                            uint32_t *__restrict__ chunk_tot,
                                                            int64_t *__restrict__ chunk_max) {
  __shared__ uint32_t wsum[kRecBlock / 64];
  __shared__ int64_t wmax[kRecBlock / 64];
  const Batch b = batches[blockIdx.y];
  const uint32_t c = blockIdx.x;
  if (c * kRecBlock >= b.msg_count) {
    if (threadIdx.x == 0) {
      chunk_tot[blockIdx.y * nchunk + c] = 0u;
      chunk_max[blockIdx.y * nchunk + c] = 0;
    }
    return;
  }
  const int64_t base_ts = m.ts[b.first_msg];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t k = c * kRecBlock + threadIdx.x;
  const bool on = k < b.msg_count;
  const uint32_t sz = on ? rec_fields(m, b.first_msg + k, k, base_ts).size : 0u;
  int64_t mx = on ? m.ts[b.first_msg + k] : 0;  // MaxTimestamp from 0 (write_msgq :813)
  uint32_t x = sz;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
    const int64_t z = __shfl_xor(mx, d);
    mx = z > mx ? z : mx;
  }
  if (lane == 63) wsum[w] = x;
  if (lane == 0) wmax[w] = mx;
  __syncthreads();
  uint32_t before = 0, total = 0;
  int64_t M = 0;
#pragma unroll
  for (int i = 0; i < kRecBlock / 64; ++i) {
    before += i < w ? wsum[i] : 0u;
    total += wsum[i];
    M = wmax[i] > M ? wmax[i] : M;
  }
  if (on) rec_offs[b.first_msg + k] = before + x - sz;
  if (threadIdx.x == 0) {
    chunk_tot[blockIdx.y * nchunk + c] = total;
    chunk_max[blockIdx.y * nchunk + c] = M;
  }
}

// ---- sizes, 2/3: per batch: scan of its chunk totals (in place -> chunk bases from
// the batch start, header included), batch size, MaxTimestamp.  grid (batches), 64 threads
__global__ __launch_bounds__(64) void v2_batch_kernel(uint32_t nchunk, uint32_t *__restrict__ chunk_tot,
                                                     const int64_t *__restrict__ chunk_max,
                                                     uint32_t *__restrict__ batch_sizes,
                                                     int64_t *__restrict__ max_ts) {
  const int lane = threadIdx.x;
  uint32_t *t = chunk_tot + blockIdx.x * nchunk;
  const int64_t *cm = chunk_max + blockIdx.x * nchunk;
  uint32_t run = 61u;  // RD_KAFKAP_MSGSET_V2_SIZE
  int64_t mx = 0;
  for (uint32_t c0 = 0; c0 < nchunk; c0 += 64) {
    const uint32_t c = c0 + uint32_t(lane);
    const uint32_t v = c < nchunk ? t[c] : 0u;
    int64_t z = c < nchunk ? cm[c] : 0;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
      const int64_t q = __shfl_xor(z, d);
      z = q > z ? q : z;
    }
    if (c < nchunk) t[c] = run + x - v;
    run += __shfl(x, 63);
    mx = z > mx ? z : mx;
  }
  if (lane == 0) {
    batch_sizes[blockIdx.x] = run;
    max_ts[blockIdx.x] = mx;
  }
}

// ---- sizes, 3/3: record offsets from the batch start.  grid (chunks, batches)
__global__ __launch_bounds__(kRecBlock) void v2_fixup_kernel(const Batch *__restrict__ batches,
                                                            uint32_t nchunk,
                                                            const uint32_t *__restrict__ chunk_base,
                                                            uint32_t *__restrict__ rec_offs) {
  const Batch b = batches[blockIdx.y];
  const uint32_t k = blockIdx.x * kRecBlock + threadIdx.x;
  if (k < b.msg_count) rec_offs[b.first_msg + k] += chunk_base[blockIdx.y * nchunk + blockIdx.x];
}

__device__ __forceinline__ void st_be(uint8_t *p, uint64_t v, int n) {
  for (int i = 0; i < n; ++i) p[i] = uint8_t(v >> (8 * (n - 1 - i)));
}

// ---- write: grid (chunks, batches); chunk 0 also writes the header.
// One lane per record writes the varints and Attributes (a tenth of the bytes), and key /
// value / header bytes shorter than 16; longer ones become copy segments (destination, arena
// offset, length) in LDS, cut into 16-byte tasks.  One lane per task then moves 16 bytes from
// the arena at byte alignment (one unaligned dwordx4 load; consecutive tasks of a segment sit
// in consecutive lanes, so a wave reads contiguous runs).  A segment's last task ends at the
// segment's end and overlaps the task before it with the same bytes, so no task is partial.
// Where the bytes go: memory takes whole aligned sectors well and everything else badly --
// measured on this kernel, a byte store per lane to scattered records wrote 25 bytes to HBM
// per byte stored, and 16-byte stores at byte alignment three times their size.  So the
// chunk's bytes are put together in LDS, kTile of them at a time (256 records of up to ~140
// bytes are one tile; larger chunks take several passes, each over the records and tasks that
// reach into its window), and each tile is written with aligned 16-byte stores, every sector
// once.
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) uint8_t rec_lds_u8;
typedef __attribute__((address_space(3))) u32x4_a1 rec_lds_u32x4_a1;

constexpr uint32_t kCopyTask = 16;  // bytes per task
constexpr uint32_t kTile = 36864;   // LDS bytes for a chunk's records

struct ToTile {  // the whole chunk is in the tile, which starts at batch byte `first`
  rec_lds_u8 *t;
  uint32_t first;
  __device__ __forceinline__ void st8(uint32_t q, uint32_t v) const { t[q - first] = uint8_t(v); }
  __device__ __forceinline__ void st16(uint32_t q, u32x4_a1 v) const {
    *reinterpret_cast<rec_lds_u32x4_a1 *>(t + (q - first)) = v;
  }
};
struct ToWindow {  // the tile holds batch bytes [first, first + kTile); others are dropped
  rec_lds_u8 *t;
  uint32_t first;
  __device__ __forceinline__ void st8(uint32_t q, uint32_t v) const {
    if (q - first < kTile) t[q - first] = uint8_t(v);
  }
  __device__ __forceinline__ void st16(uint32_t q, u32x4_a1 v) const {
    const uint32_t a = q - first;  // (wraps for a byte in front of the window)
    if (a <= kTile - kCopyTask) {
      *reinterpret_cast<rec_lds_u32x4_a1 *>(t + a) = v;
    } else if (a < kTile || a + (kCopyTask - 1u) < kTile) {  // cut by an end of the window
#pragma unroll
      for (uint32_t j = 0; j < kCopyTask; ++j)
        if (a + j < kTile) t[a + j] = uint8_t(v[j >> 2] >> (8u * (j & 3u)));
    }
  }
};

template <class To>
__device__ __forceinline__ uint32_t put_varint(const To &to, uint32_t q, uint64_t u, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) to.st8(q + i, vbyte(u, i, n));
  return q + n;
}

struct WriteLds {
  uint32_t last[kRecBlock];      // tasks of the records up to and including this one
  uint32_t roff[kRecBlock + 1];  // record starts from the batch start, then the chunk's end
  uint32_t sdst[3][kRecBlock];   // a record's segments: key, value, headers
  uint32_t slen[3][kRecBlock];   // (0: none)
  uint64_t ssrc[3][kRecBlock];
  uint32_t wsum[kRecBlock / 64];
};

__device__ __forceinline__ uint32_t seg_tasks(uint32_t len) { return (len + kCopyTask - 1u) / kCopyTask; }

// the records' segments and task counts into LDS; returns the chunk's tasks
__device__ __forceinline__ uint32_t chunk_prepare(const Msgs &m, WriteLds &L, const Rec &r, uint32_t off,
                                                  uint32_t msg, uint32_t nrec) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t mine = 0;
  if (threadIdx.x < nrec) {
    const uint32_t flen[3] = {r.kb, r.vb, r.hb};
    const uint32_t fs[3] = {r.sK, r.sV, r.sH};
    const uint64_t fsrc[3] = {r.kb ? m.key_off[msg] : 0, r.vb ? m.val_off[msg] : 0,
                              r.hb ? m.hdr_off[msg] : 0};
    uint32_t q = off + r.sL + 1u + r.sT + r.sO;
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      q += fs[f];
      const bool seg = flen[f] >= kCopyTask;
      L.sdst[f][threadIdx.x] = q;
      L.slen[f][threadIdx.x] = seg ? flen[f] : 0u;
      L.ssrc[f][threadIdx.x] = fsrc[f];
      mine += seg ? seg_tasks(flen[f]) : 0u;
      q += flen[f];
    }
    L.roff[threadIdx.x] = off;
    if (threadIdx.x == nrec - 1u) L.roff[nrec] = off + r.size;
  }
  uint32_t x = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) L.wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int i = 0; i < kRecBlock / 64; ++i) {
    before += i < w ? L.wsum[i] : 0u;
    total += L.wsum[i];
  }
  L.last[threadIdx.x] = before + x;
  __syncthreads();
  return total;
}

// this thread's record: varints, Attributes and the fields that are no segments
template <class To>
__device__ __forceinline__ void chunk_small(const To &to, const Msgs &m, const Rec &r, uint32_t off,
                                            uint32_t msg) {
  uint32_t q = put_varint(to, off, r.uL, r.sL);  // Length (:706)
  to.st8(q++, 0u);                               // Attributes (:722)
  q = put_varint(to, q, r.uT, r.sT);             // TimestampDelta (:725)
  q = put_varint(to, q, r.uO, r.sO);             // OffsetDelta (:729)
  const uint32_t flen[3] = {r.kb, r.vb, r.hb};
  const uint64_t fu[3] = {r.uK, r.uV, r.uH};     // KeyLen, ValueLen, HeaderCount varints
  const uint32_t fs[3] = {r.sK, r.sV, r.sH};
  const uint64_t fsrc[3] = {r.kb ? m.key_off[msg] : 0, r.vb ? m.val_off[msg] : 0,
                            r.hb ? m.hdr_off[msg] : 0};
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    q = put_varint(to, q, fu[f], fs[f]);
    if (flen[f] < kCopyTask)
      for (uint32_t i = 0; i < flen[f]; ++i) to.st8(q + i, m.arena[fsrc[f] + i]);
    q += flen[f];
  }
}

// tasks [t0, t1) of the chunk, one per lane
template <class To>
__device__ __forceinline__ void chunk_tasks(const To &to, const Msgs &m, const WriteLds &L, uint32_t nrec,
                                            uint32_t t0, uint32_t t1) {
  for (uint32_t t = t0 + threadIdx.x; t < t1; t += kRecBlock) {
    uint32_t lo = 0, hi = nrec - 1u;  // the first record with last[rec] > t
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (L.last[mid] > t) hi = mid; else lo = mid + 1u;
    }
    const uint32_t rec = lo;
    uint32_t k = t - (rec ? L.last[rec - 1u] : 0u);
    const uint32_t n0 = seg_tasks(L.slen[0][rec]), n1 = seg_tasks(L.slen[1][rec]);
    const int f = k < n0 ? 0 : (k < n0 + n1 ? 1 : 2);
    k -= f == 0 ? 0u : (f == 1 ? n0 : n0 + n1);
    const uint32_t len = L.slen[f][rec];
    const uint32_t o = min(k * kCopyTask, len - kCopyTask);
    to.st16(L.sdst[f][rec] + o, *reinterpret_cast<const u32x4_a1 *>(m.arena + L.ssrc[f][rec] + o));
  }
}

// tile -> memory: tile[lo, hi) to g[lo, hi), g + 0 aligned to 16; whole 16-byte pieces with
// aligned stores, the cut ones (a chunk's first and last: the neighbours' bytes stay) bytewise
__device__ __forceinline__ void tile_out(const uint8_t *tile, uint8_t *g, uint32_t lo, uint32_t hi) {
  for (uint32_t i = threadIdx.x * 16u; i < hi; i += kRecBlock * 16u) {
    if (i >= lo && i + 16u <= hi) {
      *reinterpret_cast<uint4 *>(g + i) = *reinterpret_cast<const uint4 *>(tile + i);
    } else {
      const uint32_t j0 = i > lo ? i : lo, j1 = i + 16u < hi ? i + 16u : hi;
      for (uint32_t j = j0; j < j1; ++j) g[j] = tile[j];
    }
  }
}

__global__ __launch_bounds__(kRecBlock) void v2_write_kernel(Msgs m, const Batch *__restrict__ batches,
                                                            const uint32_t *__restrict__ rec_offs,
                                                            const uint32_t *__restrict__ batch_sizes,
                                                            const int64_t *__restrict__ max_ts,
                                                            const uint64_t *__restrict__ out_offs,
                                                            uint8_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kTile];
  __shared__ WriteLds L;
  const Batch b = batches[blockIdx.y];
  uint8_t *bo = out + out_offs[blockIdx.y];
  const uint32_t c0 = blockIdx.x * kRecBlock;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t base_ts = b.msg_count ? m.ts[b.first_msg] : 0;
    st_be(bo + 0, 0, 8);                                   // BaseOffset (:362)
    st_be(bo + 8, batch_sizes[blockIdx.y] - 12u, 4);       // Length (:1265)
    st_be(bo + 12, 0, 4);                                  // PartitionLeaderEpoch (:368)
    bo[16] = 2;                                            // Magic (:371)
    st_be(bo + 17, 0, 4);                                  // CRC: calc_crc_v2 later
    st_be(bo + 21, uint16_t(b.attributes), 2);             // Attributes (:1271)
    st_be(bo + 23, uint32_t(b.msg_count - 1u), 4);         // LastOffsetDelta (:1275)
    st_be(bo + 27, uint64_t(base_ts), 8);                  // BaseTimestamp (:1279)
    st_be(bo + 35, uint64_t(max_ts[blockIdx.y]), 8);       // MaxTimestamp (:1283)
    st_be(bo + 43, uint64_t(b.producer_id), 8);            // ProducerId (:392)
    st_be(bo + 51, uint16_t(b.producer_epoch), 2);         // ProducerEpoch (:395)
    st_be(bo + 53, uint32_t(b.base_sequence), 4);          // BaseSequence (:1287)
    st_be(bo + 57, b.msg_count, 4);                        // RecordCount (:1291)
  }
  if (c0 >= b.msg_count) return;
  const uint32_t nrec = b.msg_count - c0 < kRecBlock ? b.msg_count - c0 : kRecBlock;
  const bool on = threadIdx.x < nrec;
  Rec r = {};
  uint32_t off = 0, msg = 0;
  if (on) {
    const uint32_t k = c0 + threadIdx.x;
    msg = b.first_msg + k;
    r = rec_fields(m, msg, k, m.ts[b.first_msg]);
    off = rec_offs[msg];
  }
  const uint32_t total = chunk_prepare(m, L, r, off, msg, nrec);
  const uint32_t s0 = L.roff[0], s1 = L.roff[nrec];
  // the tiles start at the 16-byte boundary of memory at or in front of the chunk's first byte
  const uint32_t mis = uint32_t((reinterpret_cast<uintptr_t>(bo) + s0) & 15u);
  const uint32_t used = mis + (s1 - s0);
  rec_lds_u8 *lt = (rec_lds_u8 *)tile;
  if (used <= kTile) {
    const ToTile to{lt, s0 - mis};
    if (on) chunk_small(to, m, r, off, msg);
    chunk_tasks(to, m, L, nrec, 0u, total);
    __syncthreads();
    tile_out(tile, bo + s0 - mis, mis, used);
    return;
  }
  for (uint32_t w0 = 0; w0 < used; w0 += kTile) {
    const uint32_t first = s0 - mis + w0, lim = first + kTile;
    const ToWindow to{lt, first};
    // records that reach into [first, lim): from the last one that starts at or before
    // `first` to the last one that starts before `lim`
    uint32_t lo = 0, hi = nrec - 1u;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1u) >> 1;
      if (L.roff[mid] <= first) lo = mid; else hi = mid - 1u;
    }
    const uint32_t r_lo = lo;
    hi = nrec - 1u;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1u) >> 1;
      if (L.roff[mid] < lim) lo = mid; else hi = mid - 1u;
    }
    const uint32_t r_hi = lo;
    if (threadIdx.x >= r_lo && threadIdx.x <= r_hi) chunk_small(to, m, r, off, msg);
    // their tasks, less those of the first record that end in front of the window and those
    // of the last that start behind it (a record can be many windows long); one task of
    // slack at either end, the window drops what lies outside
    uint32_t ta = L.last[r_lo], tb = r_hi ? L.last[r_hi - 1u] : 0u;
    {
      uint32_t t = r_lo ? L.last[r_lo - 1u] : 0u;
      for (int f = 0; f < 3; ++f) {
        const uint32_t len = L.slen[f][r_lo], dst = L.sdst[f][r_lo], n = seg_tasks(len);
        if (n && dst + len > first) {
          const uint32_t k = dst >= first ? 0u : (first - dst) / kCopyTask;
          ta = t + (k ? k - 1u : 0u);
          break;
        }
        t += n;
      }
      t = L.last[r_hi];
      for (int f = 2; f >= 0; --f) {
        const uint32_t len = L.slen[f][r_hi], dst = L.sdst[f][r_hi], n = seg_tasks(len);
        t -= n;
        if (n && dst < lim) {
          const uint32_t k = (lim - dst + kCopyTask - 1u) / kCopyTask + 1u;
          tb = t + (k < n ? k : n);
          break;
        }
      }
    }
    chunk_tasks(to, m, L, nrec, ta, tb);
    __syncthreads();
    const uint32_t rest = used - w0;
    tile_out(tile, bo + first, w0 ? 0u : mis, rest < kTile ? rest : kTile);
    __syncthreads();
  }
}

// ---- record index: rd_kafka_msgset_reader_msg_v2
// (rdkafka_msgset_reader.c:715-927) for every record of a batch, one row each.
// One wavefront per batch.  The records are staged through an 8 KiB LDS window (16-byte
// buffer loads): lane 0 walks the Length chain (:736-737) over it -- one LDS round trip
// per record --
// and lists the records that lie wholly inside it; then every lane parses one listed
// record's fields (:738-878) from LDS.  Records larger than the window are parsed by
// lane 0 straight from global memory.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Rows {  // rdk_hip_v2_rows_t
  int64_t *offset, *timestamp;
  uint32_t *key_off;
  int32_t *key_len;
  uint32_t *val_off;
  int32_t *val_len;
  uint32_t *hdr_off, *hdr_len;
};

constexpr uint32_t kIdxWin = 8192;            // LDS window per wavefront
constexpr uint32_t kIdxList = kIdxWin / 6;    // a record is at least 6 bytes
constexpr int kIdxWaves = 4;

typedef __attribute__((address_space(3))) uint8_t lds_b;
typedef __attribute__((address_space(3))) uint16_t lds_h;

// zig-zag varint at p (rdvarint.h:114-141, rdbuf.c:877-912) with bytes [p, lim)
// readable through get(); returns bytes read, 0 on underflow or more than 10 bytes
template <class Get>
__device__ __forceinline__ uint32_t idx_varint(Get get, uint32_t p, uint32_t lim, int64_t &v) {
  uint64_t num = 0;
  for (uint32_t k = 0; k < 10; ++k) {
    if (p + k >= lim) return 0;
    const uint32_t b = get(p + k);
    num |= uint64_t(b & 0x7fu) << (7u * k);
    if (!(b & 0x80u)) {
      v = int64_t(num >> 1) ^ -int64_t(num & 1u);
      return k + 1u;
    }
  }
  return 0;
}

// fields of the record whose Length varint starts at r (positions through get(), all
// below `lim`); false = parse failure (rd_kafka_buf_parse_fail / underflow)
struct IdxRow {
  int64_t tsd, od;
  int32_t kl, vl;
  uint32_t ko, vo, ho, hl;
};
template <class Get>
__device__ __forceinline__ bool idx_record(Get get, uint32_t r, uint32_t lim, IdxRow &o,
                                           uint32_t &next) {
  int64_t L, kl, vl;
  uint32_t n = idx_varint(get, r, lim, L);  // :736
  if (!n) return false;
  uint32_t p = r + n;
  if (L < 0 || uint64_t(L) > uint64_t(lim - p)) return false;
  const uint32_t end = p + uint32_t(L);     // :737
  if (p + 1u > end) return false;
  p += 1u;                                  // Attributes :738
  if (!(n = idx_varint(get, p, end, o.tsd))) return false;  // :740
  p += n;
  if (!(n = idx_varint(get, p, end, o.od))) return false;   // :741
  p += n;
  if (!(n = idx_varint(get, p, end, kl))) return false;     // :871
  p += n;
  if (kl < -1 || (kl > 0 && uint64_t(kl) > uint64_t(end - p))) return false;
  o.ko = p;
  o.kl = int32_t(kl);
  if (kl > 0) p += uint32_t(kl);
  if (!(n = idx_varint(get, p, end, vl))) return false;     // :872
  p += n;
  if (vl < -1 || (vl > 0 && uint64_t(vl) > uint64_t(end - p))) return false;
  o.vo = p;
  o.vl = int32_t(vl);
  if (vl > 0) p += uint32_t(vl);
  o.ho = p;                                 // binhdrs: HeaderCount + headers, :876-878
  o.hl = end - p;
  next = end;
  return true;
}

__device__ __forceinline__ int64_t ld_be64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return int64_t(v);
}

__global__ __launch_bounds__(64 * kIdxWaves) void v2_index_kernel(
    const uint8_t *__restrict__ hdr_base, const uint64_t *__restrict__ hdr_offs,
    const uint8_t *__restrict__ rec_base, const uint64_t *__restrict__ rec_offs,
    const uint32_t *__restrict__ rec_lens, const uint64_t *__restrict__ row_offs,
    const uint32_t *__restrict__ row_caps, Rows rows, int32_t *__restrict__ count, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[kIdxWaves][kIdxWin + 32];
  __shared__ uint16_t list_all[kIdxWaves][kIdxList];
  // wave index through readfirstlane: the compiler then knows everything derived from the
  // batch (pointers, lengths, the Length walk) is wave-uniform and keeps it scalar
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t bi = blockIdx.x * kIdxWaves + uint32_t(wv);
  if (bi >= n) return;
  lds_b *win = (lds_b *)win_all[wv];
  lds_h *list = (lds_h *)list_all[wv];
  const uint8_t *hdr = hdr_base + hdr_offs[bi];
  const int64_t base_off = ld_be64(hdr + 0);   // BaseOffset (msetr_v2_hdr, :742)
  const int64_t base_ts = ld_be64(hdr + 27);   // BaseTimestamp (:911-912)
  const uint8_t *rec = rec_base + rec_offs[bi];
  const uint32_t len = rec_lens[bi];
  const uint64_t row0 = row_offs[bi];
  const uint32_t cap = row_caps[bi];
  uint32_t pos = 0, nrow = 0;
  int32_t err = -1;  // first failing record index
  auto gget = [&](uint32_t p) -> uint32_t { return rec[p]; };
  while (pos < len && err < 0) {
    // stage [pos, pos + kIdxWin): 16-byte buffer loads from the 16-byte aligned address
    // below, all issued before their LDS stores; bytes past the batch read as 0
    const uint32_t base = pos, wl = len - base < kIdxWin ? len - base : kIdxWin;
    const uintptr_t ga = reinterpret_cast<uintptr_t>(rec + base);
    const uintptr_t al = ga & ~uintptr_t(15);
    const uint32_t sh = uint32_t(ga - al);  // window byte q is LDS byte q + sh
    // (range checks are per dword: round up so the batch's last bytes are read; the bytes
    // after them in that dword share its page and are never used)
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(al), 0,
                                                        int((sh + wl + 3u) & ~3u), 0x00020000);
    {
      constexpr int kV = int((kIdxWin + 16) / (64 * 16)) + 1;  // 16-byte vectors per lane
      u32x4 v[kV];
#pragma unroll
      for (int it = 0; it < kV; ++it)
        v[it] = __builtin_amdgcn_raw_buffer_load_b128(rs, uint32_t((lane + 64 * it) * 16), 0, 0);
#pragma unroll
      for (int it = 0; it < kV; ++it) {
        const uint32_t o = uint32_t((lane + 64 * it) * 16);
        if (o < kIdxWin + 16) *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(win + o) = v[it];
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    auto lget = [&](uint32_t p) -> uint32_t { return win[p - base + sh]; };
    // walk: records wholly inside the window go to the list
    // the walk is wave-uniform: LDS bytes are read as broadcasts and moved to scalar
    // registers, so its arithmetic runs on the scalar unit
    uint32_t nl = 0, stop = pos;
    int32_t werr = -1;
    auto sget = [&](uint32_t p) -> uint32_t { return __builtin_amdgcn_readfirstlane(lget(p)); };
    {
      uint32_t p = pos;
      const uint32_t wend = base + wl;
      while (p < len && nl < kIdxList) {
        int64_t L;
        uint32_t sz;
        // Length varints of this workload are 1-2 bytes: both bytes in one LDS round trip
        const uint32_t b0 = sget(p), b1 = sget(p + 1u);
        if (b0 < 0x80u && p + 1u <= wend) {
          sz = 1u;
          L = int64_t(b0 >> 1) ^ -int64_t(b0 & 1u);
        } else if (b1 < 0x80u && p + 2u <= wend) {
          const uint64_t u = (b0 & 0x7fu) | (uint64_t(b1) << 7);
          sz = 2u;
          L = int64_t(u >> 1) ^ -int64_t(u & 1u);
        } else {
          sz = idx_varint(sget, p, wend, L);
        }
        if (!sz) {
          if (wend < len && p > base) break;  // varint cut by the window: next window
          werr = 0;                           // underflow at the batch end (or huge varint)
          break;
        }
        if (L < 0 || uint64_t(L) > uint64_t(len - p - sz)) { werr = 0; break; }
        const uint32_t e = p + sz + uint32_t(L);
        if (e > wend) break;  // ends past the window: next window (or the big path)
        if (lane == 0) list[nl] = uint16_t(p - base);
        ++nl;
        p = e;
      }
      stop = p;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // parse the listed records, 64 at a time
    int32_t bad = 0x7fffffff;
    for (uint32_t i0 = 0; i0 < nl; i0 += 64) {
      const uint32_t i = i0 + uint32_t(lane);
      if (i < nl) {
        const uint32_t r = base + list[i];
        IdxRow o;
        uint32_t nx;
        if (!idx_record(lget, r, base + wl, o, nx) || nrow + i >= cap) {
          bad = int32_t(i) < bad ? int32_t(i) : bad;
        } else {
          const uint64_t row = row0 + nrow + i;
          rows.offset[row] = base_off + o.od;        // :742
          rows.timestamp[row] = base_ts + o.tsd;     // :911-912 (CreateTime)
          rows.key_off[row] = o.ko;
          rows.key_len[row] = o.kl;
          rows.val_off[row] = o.vo;
          rows.val_len[row] = o.vl;
          rows.hdr_off[row] = o.ho;
          rows.hdr_len[row] = o.hl;
        }
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const int32_t y = __shfl_xor(bad, d);
      bad = y < bad ? y : bad;
    }
    bad = __builtin_amdgcn_readfirstlane(bad);  // uniform after the reduction
    if (bad != 0x7fffffff) {
      err = int32_t(nrow) + bad;
      break;
    }
    nrow += nl;
    if (werr >= 0) {
      err = int32_t(nrow);
      break;
    }
    pos = stop;
    if (nl == 0 && pos < len) {
      // a record larger than the window (or whose Length varint is cut at the batch
      // end): lane 0 parses it from global memory
      IdxRow o;
      uint32_t nx = pos;
      bool ok = false;
      if (lane == 0) ok = idx_record(gget, pos, len, o, nx) && nrow < cap;
      ok = __builtin_amdgcn_readfirstlane(ok ? 1 : 0) != 0;
      nx = __builtin_amdgcn_readfirstlane(nx);
      if (!ok) {
        err = int32_t(nrow);
        break;
      }
      if (lane == 0) {
        const uint64_t row = row0 + nrow;
        rows.offset[row] = base_off + o.od;
        rows.timestamp[row] = base_ts + o.tsd;
        rows.key_off[row] = o.ko;
        rows.key_len[row] = o.kl;
        rows.val_off[row] = o.vo;
        rows.val_len[row] = o.vl;
        rows.hdr_off[row] = o.ho;
        rows.hdr_len[row] = o.hl;
      }
      nrow += 1;
      pos = nx;
    }
  }
  if (lane == 0) count[bi] = err >= 0 ? -(1 + err) : int32_t(nrow);
}

// ---- the default record index: one 512-thread workgroup per batch, the records found by
// the speculative parallel walk of specwalk.h (record p is [p, p + |Length varint| +
// Length), :736-737), every verified thread then parsing its own records (:738-878) from
// the LDS window.  Results are identical to v2_index_kernel (kept as RDK_HIP_IDX_V1=1).
struct V2Idx {
  // the walk's record classification, as v2_index_kernel's Length walk decides it
  __device__ __forceinline__ uint32_t classify(const spec::Win &W, uint32_t p,
                                               uint32_t &next) const {
    if (p == W.len) return spec::kDone;
    int64_t L;
    const uint32_t sz = idx_varint([&](uint32_t q) { return W.b(q); }, p, W.end, L);
    if (!sz) return (W.end < W.len && p + 10u > W.end) ? spec::kCut : spec::kErr;
    if (L < 0 || uint64_t(L) > uint64_t(W.len - p - sz)) return spec::kErr;
    const uint32_t e = p + sz + uint32_t(L);
    if (e > W.end) return spec::kCut;
    next = e;
    return spec::kOk;
  }
  // heuristic record-start test (never decides a result): a Length of at least 6 whose
  // record ends inside the batch, Attributes 0 (the writer's, rdkafka_msgset_writer.c:722),
  // TimestampDelta and OffsetDelta varints, and the record after it looking the same with
  // a larger OffsetDelta
  __device__ __forceinline__ bool head(const spec::Win &W, uint32_t q, uint32_t &e,
                                       int64_t &od) const {
    auto g = [&](uint32_t x) { return W.b(x); };
    int64_t L, tsd;
    const uint32_t sz = idx_varint(g, q, q + 3u < W.end ? q + 3u : W.end, L);
    if (!sz || L < 6 || uint64_t(L) > uint64_t(W.len - q - sz)) return false;
    const uint32_t a = q + sz;
    if (W.b(a) != 0u) return false;
    const uint32_t n1 = idx_varint(g, a + 1u, W.end, tsd);
    if (!n1) return false;
    const uint32_t n2 = idx_varint(g, a + 1u + n1, W.end, od);
    if (!n2 || od < 0) return false;
    e = q + sz + uint32_t(L);
    return true;
  }
  __device__ __forceinline__ bool plausible(const spec::Win &W, uint32_t q) const {
    if (q + 24u > W.end) return false;
    uint32_t e, e2;
    int64_t od, od2;
    if (!head(W, q, e, od)) return false;
    if (e == W.len) return true;
    if (e + 24u > W.end || !head(W, e, e2, od2)) return false;
    return od2 > od && od2 - od < (int64_t(1) << 31);
  }
  // prefilter: byte q even and nonzero (the first byte of a positive zig-zag Length) and
  // a zero byte (Attributes) at q+1 or q+2
  __device__ __forceinline__ uint32_t scan(const spec::Win &W, uint32_t s0, uint32_t lim) const {
    auto pre = [](const uint32_t *D, int k) {
      return spec::nzb(D[k]) & spec::evb(D[k]) &
             (spec::zb(__builtin_amdgcn_alignbyte(D[k + 1], D[k], 1u)) |
              spec::zb(__builtin_amdgcn_alignbyte(D[k + 1], D[k], 2u)));
    };
    return spec::scan(W, s0, lim, pre, [&](uint32_t q) { return plausible(W, q); });
  }
};

__global__ __launch_bounds__(spec::kThreads, 1) void v2_index_spec_kernel(
    const uint8_t *__restrict__ hdr_base, const uint64_t *__restrict__ hdr_offs,
    const uint8_t *__restrict__ rec_base, const uint64_t *__restrict__ rec_offs,
    const uint32_t *__restrict__ rec_lens, const uint64_t *__restrict__ row_offs,
    const uint32_t *__restrict__ row_caps, Rows rows, int32_t *__restrict__ count) {
  __shared__ spec::Shared S;
  __shared__ uint32_t big_s[2];
  const uint32_t bi = blockIdx.x, t = threadIdx.x;
  const uint8_t *hdr = hdr_base + hdr_offs[bi];
  const int64_t base_off = ld_be64(hdr + 0);   // BaseOffset (msetr_v2_hdr, :742)
  const int64_t base_ts = ld_be64(hdr + 27);   // BaseTimestamp (:911-912)
  const uint8_t *rec = rec_base + rec_offs[bi];
  const uint64_t row0 = row_offs[bi];
  const uint32_t cap = row_caps[bi];
  auto put = [&](uint32_t r, const IdxRow &o) {
    const uint64_t row = row0 + r;
    rows.offset[row] = base_off + o.od;        // :742
    rows.timestamp[row] = base_ts + o.tsd;     // :911-912 (CreateTime)
    rows.key_off[row] = o.ko;
    rows.key_len[row] = o.kl;
    rows.val_off[row] = o.vo;
    rows.val_len[row] = o.vl;
    rows.hdr_off[row] = o.ho;
    rows.hdr_len[row] = o.hl;
  };
  auto emit = [&](const spec::Win &W, uint32_t c, uint32_t k, uint32_t rb) -> uint32_t {
    auto g = [&](uint32_t q) { return W.b(q); };
    uint32_t p = c;
    for (uint32_t i = 0; i < k && rb + i < cap; ++i) {
      IdxRow o;
      uint32_t nx;
      if (!idx_record(g, p, W.end, o, nx)) return rb + i;
      put(rb + i, o);
      p = nx;
    }
    return spec::kNone;
  };
  auto big = [&](const spec::Win &W, uint32_t base, uint32_t r, uint32_t &next) -> bool {
    (void)W;
    if (t == 0) {  // a record larger than the window: thread 0 from global memory
      IdxRow o;
      uint32_t nx = base;
      const bool ok = idx_record([&](uint32_t q) -> uint32_t { return rec[q]; }, base,
                                 rec_lens[bi], o, nx);
      if (ok) put(r, o);
      big_s[0] = ok;
      big_s[1] = nx;
    }
    __syncthreads();
    const bool ok = big_s[0] != 0;
    next = big_s[1];
    __syncthreads();
    return ok;
  };
  const int32_t res = spec::walk(rec, rec_lens[bi], cap, S, V2Idx(), emit, big);
  if (t == 0) count[bi] = res;
}

}  // namespace rdk

using namespace rdk;

static_assert(sizeof(rdk_hip_msgs_t) == sizeof(Msgs), "rdk_hip_msgs_t layout");
static_assert(sizeof(rdk_hip_v2_batch_t) == sizeof(Batch), "rdk_hip_v2_batch_t layout");

static bool msgs_ok(const rdk_hip_msgs_t *m) {
  return m && m->arena && m->timestamp && m->key_off && m->key_len && m->value_off &&
         m->value_len && (!m->header_count || (m->headers_off && m->headers_len));
}

static Msgs to_msgs(const rdk_hip_msgs_t *m) {
  Msgs r;
  r.arena = m->arena;
  r.ts = m->timestamp;
  r.key_off = m->key_off;
  r.key_len = m->key_len;
  r.val_off = m->value_off;
  r.val_len = m->value_len;
  r.hdr_off = m->header_count ? m->headers_off : nullptr;
  r.hdr_len = m->header_count ? m->headers_len : nullptr;
  r.hdr_cnt = m->header_count;
  return r;
}

// host batch descriptors -> a device copy on the stream; returns the chunk count
static int upload_batches(const rdk_hip_v2_batch_t *batches, uint32_t n, hipStream_t s,
                          Batch **d, uint32_t *nchunk) {
  uint32_t mx = 1;
  for (uint32_t i = 0; i < n; ++i) mx = batches[i].msg_count > mx ? batches[i].msg_count : mx;
  *nchunk = (mx + kRecBlock - 1) / kRecBlock;
  RDK_HIP_CHECK(hipMallocAsync(reinterpret_cast<void **>(d), size_t(n) * sizeof(Batch), s));
  RDK_HIP_CHECK(hipMemcpyAsync(*d, batches, size_t(n) * sizeof(Batch), hipMemcpyHostToDevice, s));
  return 0;
}

RDK_API int rdk_hip_msgset_v2_sizes(const rdk_hip_msgs_t *msgs, const rdk_hip_v2_batch_t *batches,
                                    uint32_t n, uint32_t *d_rec_offs, uint32_t *d_batch_sizes,
                                    int64_t *d_max_ts, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!msgs_ok(msgs) || !batches || !d_rec_offs || !d_batch_sizes || !d_max_ts)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  Batch *db = nullptr;
  uint32_t nchunk = 0;
  int rc = upload_batches(batches, n, s, &db, &nchunk);
  if (rc) return rc;
  uint32_t *tot = nullptr;
  int64_t *cmax = nullptr;
  const size_t nc = size_t(n) * nchunk;
  RDK_HIP_CHECK(hipMallocAsync(reinterpret_cast<void **>(&tot), nc * 4, s));
  RDK_HIP_CHECK(hipMallocAsync(reinterpret_cast<void **>(&cmax), nc * 8, s));
  const Msgs m = to_msgs(msgs);
  hipLaunchKernelGGL(v2_chunk_kernel, dim3(nchunk, n), dim3(kRecBlock), 0, s, m, db, nchunk,
                     d_rec_offs, tot, cmax);
  hipLaunchKernelGGL(v2_batch_kernel, dim3(n), dim3(64), 0, s, nchunk, tot, cmax, d_batch_sizes,
                     d_max_ts);
  hipLaunchKernelGGL(v2_fixup_kernel, dim3(nchunk, n), dim3(kRecBlock), 0, s, db, nchunk, tot,
                     d_rec_offs);
  RDK_HIP_CHECK(hipGetLastError());
  RDK_HIP_CHECK(hipFreeAsync(tot, s));
  RDK_HIP_CHECK(hipFreeAsync(cmax, s));
  RDK_HIP_CHECK(hipFreeAsync(db, s));
  return RDK_HIP_OK;
}

RDK_API int rdk_hip_msgset_v2_write(const rdk_hip_msgs_t *msgs, const rdk_hip_v2_batch_t *batches,
                                    uint32_t n, const uint32_t *d_rec_offs,
                                    const uint32_t *d_batch_sizes, const int64_t *d_max_ts,
                                    const uint64_t *d_out_offs, uint8_t *d_out, uint32_t *d_crc,
                                    void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!msgs_ok(msgs) || !batches || !d_rec_offs || !d_batch_sizes || !d_max_ts || !d_out_offs ||
      !d_out)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  Batch *db = nullptr;
  uint32_t nchunk = 0;
  int rc = upload_batches(batches, n, s, &db, &nchunk);
  if (rc) return rc;
  hipLaunchKernelGGL(v2_write_kernel, dim3(nchunk, n), dim3(kRecBlock), 0, s, to_msgs(msgs), db,
                     d_rec_offs, d_batch_sizes, d_max_ts, d_out_offs, d_out);
  RDK_HIP_CHECK(hipGetLastError());
  RDK_HIP_CHECK(hipFreeAsync(db, s));
  if (d_crc)  // calc_crc_v2 (:1229-1246): the batch size is its capacity
    return rdk_hip_msgset_v2_crc(d_out, d_out_offs, d_batch_sizes, d_crc, n,
                                 RDK_HIP_V2_CRC_FINALIZE, stream);
  return RDK_HIP_OK;
}

static_assert(sizeof(rdk_hip_v2_rows_t) == sizeof(Rows), "rdk_hip_v2_rows_t layout");

RDK_API int rdk_hip_msgset_v2_index(const void *d_hdr_base, const uint64_t *d_hdr_offs,
                                    const void *d_rec_base, const uint64_t *d_rec_offs,
                                    const uint32_t *d_rec_lens, const uint64_t *d_row_offs,
                                    const uint32_t *d_row_caps, const rdk_hip_v2_rows_t *rows,
                                    int32_t *d_count, uint32_t n, void *stream) {
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (!n) return RDK_HIP_OK;
  if (!d_hdr_base || !d_hdr_offs || !d_rec_base || !d_rec_offs || !d_rec_lens || !d_row_offs ||
      !d_row_caps || !rows || !rows->offset || !rows->timestamp || !rows->key_off ||
      !rows->key_len || !rows->value_off || !rows->value_len || !rows->headers_off ||
      !rows->headers_len || !d_count)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  Rows r;
  std::memcpy(&r, rows, sizeof r);
  static const bool v1 = getenv("RDK_HIP_IDX_V1") && atoi(getenv("RDK_HIP_IDX_V1"));
  if (v1)
    hipLaunchKernelGGL(v2_index_kernel, dim3((n + kIdxWaves - 1) / kIdxWaves),
                       dim3(64 * kIdxWaves), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t *>(d_hdr_base), d_hdr_offs,
                       static_cast<const uint8_t *>(d_rec_base), d_rec_offs, d_rec_lens,
                       d_row_offs, d_row_caps, r, d_count, n);
  else
    hipLaunchKernelGGL(v2_index_spec_kernel, dim3(n), dim3(spec::kThreads), 0,
                       static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t *>(d_hdr_base), d_hdr_offs,
                       static_cast<const uint8_t *>(d_rec_base), d_rec_offs, d_rec_lens,
                       d_row_offs, d_row_caps, r, d_count);
  RDK_HIP_CHECK(hipGetLastError());
  return RDK_HIP_OK;
}
