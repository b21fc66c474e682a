// producer.hip -- the producer-side batching front-end (north_star: "the
// batching front-end collects ready batches from many toppars per broker
// thread into a pinned host staging ring") and the device kernel that turns
// compressed records into finished MsgVersion 2 record batches.
//
// Per broker thread one rdk_hip_producer_t owns a ring of `nslots` slots.
// Each slot is pinned host staging in/out + device buffers + its own HIP
// stream.  produce() gathers a batch (61-byte v2 header + records) into the
// filling slot -- the rd_slice gather the reference does before
// rd_kafka_lz4_compress (rdkafka_lz4.c:390) -- and a full slot is launched as
//
//   H2D -> rdk_hip_msgset_v2_finalize, two kernels:
//          LZ4F block compress of every batch's records (exact or fast engine), each
//          wave also leaving the raw CRC32C register of the block it wrote;
//          frame assembly + codec choice exactly as rd_kafka_msgset_writer_compress
//          (rdkafka_msgset_writer.c:1179: a frame larger than the records is thrown
//          away), Attributes |= LZ4 (:1187), Length = size-12 (:1265-1267), and the
//          CRC32C over [21, 12+Length) combined from the block registers, stored BE
//          at 17 (:1229-1246) -- no separate CRC pass over the frame
//       -> the finished batches packed into pinned host memory
//
// on the slot's stream, so slot k+1's copies overlap slot k's kernels.
// poll() hands finished batches back in submission order.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <ctime>
#include <new>
#include <vector>

#include "common.h"
#include "lz4_device.h"
#include "lz4_engine.h"

namespace rdk {

constexpr uint32_t kV2Hdr = 61;       // RD_KAFKAP_MSGSET_V2_SIZE (rdkafka_proto.h:540)

namespace {

enum SlotState { FREE = 0, FILLING, INFLIGHT };

struct Slot {
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;
  uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  uint8_t *dh_out = nullptr;  // h_out as seen by the device (the pack kernel writes it)
  // The batch table lives in mapped pinned memory: the kernels read the few words per batch
  // that they need, and write their results, straight over PCIe (dh_meta is h_meta as the
  // device sees it).  Small copies would queue behind the other slots' bulk input copies on
  // the copy engine and hold this slot's completion back by milliseconds.
  uint8_t *h_meta = nullptr, *dh_meta = nullptr;
  unsigned long long *d_cursor = nullptr;  // the pack kernel's output cursor (device atomics)
  size_t in_used = 0, out_used = 0;
  uint32_t nb = 0, polled = 0;
  SlotState st = FREE;
  std::vector<uint64_t> cookies;
};

}  // namespace

size_t lz4f_compress_bound(size_t len);
size_t snappy_max_compressed_length(size_t len);
int snappy_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                           uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                           uint32_t n, hipStream_t s);
int lz4f_compress_device(Ctx *c, const uint8_t *d_in, const uint64_t *d_in_offs,
                         const uint32_t *d_in_lens, uint8_t *d_out, const uint64_t *d_out_offs,
                         uint32_t *d_out_lens, uint32_t n, int accel, hipStream_t s,
                         const FuseCrc *fuse);
int lz4f_compress_fast_device(const uint8_t *d_in, const uint64_t *d_in_offs,
                              const uint32_t *d_in_lens, uint8_t *d_out,
                              const uint64_t *d_out_offs, uint32_t *d_out_lens, uint32_t n,
                              hipStream_t s, const FuseCrc *fuse);
bool lz4f_fast_engine_is_units();
void stage_copy(void *dst, const void *src, size_t n);  // hostcopy.cpp: streaming stores
void stage_fence();

}  // namespace rdk

using namespace rdk;

struct rdk_hip_producer_s {
  int device = 0, mode = 0;
  size_t slot_bytes = 0, out_bytes = 0;
  uint32_t max_batches = 0;
  std::vector<Slot> slots;
  int fill = 0;   // slot being filled
  int next = 0;   // oldest slot not fully polled
  // RDK_HIP_PRODUCER_PROF=1: host nanoseconds spent in the gather, in launch() and in
  // blocking polls, printed when the producer is destroyed
  uint64_t ns_gather = 0, ns_launch = 0, ns_wait = 0, n_launch = 0;
};

namespace {

// per-slot batch table (pinned host + device mirror), arrays of B entries:
//   rec_offs, out_offs, frame_offs, pack_offs (u64) | caps, rec_lens, frame_lens,
//   batch_lens, crcs (u32); then the pack cursor (u64)
struct Meta {
  uint64_t *rec_offs, *out_offs, *frame_offs, *pack_offs;
  uint32_t *caps, *rec_lens, *frame_lens, *batch_lens, *crcs;
  unsigned long long *cursor;
};
Meta meta_at(uint8_t *base, uint32_t B) {
  Meta m;
  m.rec_offs = reinterpret_cast<uint64_t *>(base);
  m.out_offs = m.rec_offs + B;
  m.frame_offs = m.out_offs + B;
  m.pack_offs = m.frame_offs + B;
  m.caps = reinterpret_cast<uint32_t *>(m.pack_offs + B);
  m.rec_lens = m.caps + B;
  m.frame_lens = m.rec_lens + B;
  m.batch_lens = m.frame_lens + B;
  m.crcs = m.batch_lens + B;
  m.cursor = reinterpret_cast<unsigned long long *>(
      (reinterpret_cast<uintptr_t>(m.crcs + B) + 7) & ~uintptr_t(7));
  return m;
}
size_t meta_bytes(uint32_t B) { return size_t(B) * (4 * 8 + 5 * 4) + 16; }

size_t out_span(size_t len, int mode) {
  const size_t bound = mode == RDK_HIP_PRODUCER_SNAPPY ? snappy_max_compressed_length(len)
                                                       : lz4f_compress_bound(len);
  return (kV2Hdr + bound + 255) & ~size_t(255);
}

// compression.codec=snappy: the writer's codec choice and header for batch i, whose snappy
// stream (d_frame_lens[i] bytes) sits 61 bytes into its output slot.  A stream larger than
// the records is thrown away (rdkafka_msgset_writer.c:1179), else Attributes |= SNAPPY
// (:1187); Length = size - 12 (:1265).  The CRC32C pass follows.  One workgroup per batch.
__global__ __launch_bounds__(256) void snappy_v2_header_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ rec_offs,
    const uint32_t *__restrict__ rec_lens, uint8_t *out, const uint64_t *__restrict__ out_offs,
    const uint32_t *__restrict__ frame_lens, uint32_t *__restrict__ batch_lens, uint32_t n) {
  const uint32_t t = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t len = rec_lens[i], clen = frame_lens[i];
    const uint8_t *rec = in + rec_offs[i];
    uint8_t *ob = out + out_offs[i];
    const bool compressed = clen <= len;
    const uint32_t payload = compressed ? clen : len;
    if (!compressed)
      for (uint32_t k = t; k < len; k += 256u) ob[kV2Hdr + k] = rec[k];
    if (t < kV2Hdr) {
      uint32_t v = rec[int(t) - int(kV2Hdr)];
      const uint32_t length = kV2Hdr + payload - 12u;
      if (t >= 8 && t < 12) v = (length >> (8u * (3u - (t - 8u)))) & 0xFFu;
      if (t == 22 && compressed) v |= 2u;  // RD_KAFKA_COMPRESSION_SNAPPY
      ob[t] = uint8_t(v);
    }
    if (t == 0) batch_lens[i] = kV2Hdr + payload;
  }
}

// d_crcs[i] = the CRC stored big-endian at offset 17 of batch i
__global__ void v2_crc_gather_kernel(const uint8_t *__restrict__ out, const uint64_t *__restrict__ out_offs,
                                     uint32_t *__restrict__ crcs, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *p = out + out_offs[i] + 17;
  crcs[i] = (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}

// Finished batches -> the slot's pinned host buffer, packed back to back (16-byte aligned,
// in completion order of an atomic cursor) by the GPU itself: only the batches' own bytes
// cross PCIe, not the compress-bound slots of d_out.  One workgroup per batch.
__global__ __launch_bounds__(256) void pack_to_host_kernel(const uint8_t *__restrict__ d_out,
                                                          const uint64_t *__restrict__ out_offs,
                                                          const uint32_t *__restrict__ batch_lens,
                                                          uint32_t n, uint8_t *__restrict__ h_out,
                                                          uint64_t *__restrict__ pack_offs,
                                                          unsigned long long *__restrict__ cursor) {
  __shared__ uint64_t at;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t len = batch_lens[i];
    if (threadIdx.x == 0) {
      at = atomicAdd(cursor, (unsigned long long)((len + 15u) & ~15u));
      pack_offs[i] = at;
    }
    __syncthreads();
    const uint4 *src = reinterpret_cast<const uint4 *>(d_out + out_offs[i]);  // 256-aligned
    uint4 *dst = reinterpret_cast<uint4 *>(h_out + at);                        // 16-aligned
    for (uint32_t v = threadIdx.x; v < (len + 15u) / 16u; v += blockDim.x) dst[v] = src[v];
    __syncthreads();
  }
}

}  // namespace

// The writer's finalize for n device-resident MessageSets (see the header): compress,
// codec choice + header, CRC32C.  Three stages on `stream`, no host synchronisation.
RDK_API int rdk_hip_msgset_v2_finalize(const void *d_in, const uint64_t *d_rec_offs,
                                       const uint32_t *d_rec_lens, void *d_out,
                                       const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                                       uint32_t *d_frame_lens, uint32_t *d_batch_lens,
                                       uint32_t *d_crcs, uint32_t n, int mode, void *stream) {
  if (!n) return RDK_HIP_OK;
  if (!d_in || !d_rec_offs || !d_rec_lens || !d_out || !d_out_offs || !d_out_caps ||
      !d_frame_lens || !d_batch_lens || !d_crcs)
    return set_error(RDK_HIP_E_INVAL, "null pointer");
  if (mode != RDK_HIP_PRODUCER_EXACT && mode != RDK_HIP_PRODUCER_FAST &&
      mode != RDK_HIP_PRODUCER_SNAPPY)
    return set_error(RDK_HIP_E_INVAL, "bad mode %d", mode);
  hipStream_t s = static_cast<hipStream_t>(stream);
  Ctx *c = ctx();
  if (!c) return RDK_HIP_E_NODEV;
  if (mode == RDK_HIP_PRODUCER_SNAPPY) {
    // snappy: fragments + assembly, then the codec choice and header, then the CRC32C pass
    // over the finished batches (the CRC is not fused into this compressor)
    uint8_t *ob = static_cast<uint8_t *>(d_out);
    int rc = snappy_compress_device(static_cast<const uint8_t *>(d_in), d_rec_offs, d_rec_lens,
                                    ob + kV2Hdr, d_out_offs, d_frame_lens, n, s);
    if (rc) return rc;
    hipLaunchKernelGGL(snappy_v2_header_kernel, dim3(n < 4096u ? n : 4096u), dim3(256), 0, s,
                       static_cast<const uint8_t *>(d_in), d_rec_offs, d_rec_lens, ob, d_out_offs,
                       d_frame_lens, d_batch_lens, n);
    RDK_HIP_CHECK(hipGetLastError());
    // d_crcs doubles as the CRC pass's status array, then takes the CRC values
    rc = rdk_hip_msgset_v2_crc(d_out, d_out_offs, d_out_caps, d_crcs, n, RDK_HIP_V2_CRC_FINALIZE, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(v2_crc_gather_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, ob, d_out_offs,
                       d_crcs, n);
    RDK_HIP_CHECK(hipGetLastError());
    return RDK_HIP_OK;
  }
  (void)d_out_caps;  // slots are sized by the caller from the codec's bound
  // Two launches: the block kernel, which also leaves the raw CRC32C register of every
  // block it writes (crc_wave.h), and the frame assembler, which also makes the writer's
  // codec choice, finishes the header and combines the batch's CRC from those registers.
  // Frame i goes 61 bytes into batch i's output slot: same offsets on a shifted base.
  FuseCrc fz;
  fz.block_crc = crc_scratch(c, s, (size_t(n) * 64 + 16) * sizeof(uint32_t));
  if (!fz.block_crc) return RDK_HIP_E_NOMEM;
  if (n > kMaxNbFrames) fz.max_nb = fz.block_crc + size_t(n) * 64;
  fz.t0 = crc_tables_dev(c->device);
  fz.x2n = crc_x2n_dev(c->device);
  fz.batch_lens = d_batch_lens;
  fz.crcs = d_crcs;
  uint8_t *fbase = static_cast<uint8_t *>(d_out) + kV2Hdr;
  if (mode == RDK_HIP_PRODUCER_FAST && lz4f_fast_engine_is_units()) {
    // The workgroup-per-block engine leaves no block registers: compress + assemble (codec
    // choice, header, CRC field zero), then the batched CRC32C pass over the finished
    // batches -- a third of the input's bytes, at memory speed -- as for snappy above.
    fz.block_crc = nullptr;
    int rc = lz4f_compress_fast_device(static_cast<const uint8_t *>(d_in), d_rec_offs, d_rec_lens,
                                       fbase, d_out_offs, d_frame_lens, n, s, &fz);
    if (rc) return rc;
    rc = rdk_hip_msgset_v2_crc(d_out, d_out_offs, d_out_caps, d_crcs, n, RDK_HIP_V2_CRC_FINALIZE, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(v2_crc_gather_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s,
                       static_cast<const uint8_t *>(d_out), d_out_offs, d_crcs, n);
    RDK_HIP_CHECK(hipGetLastError());
    return RDK_HIP_OK;
  }
  if (mode == RDK_HIP_PRODUCER_FAST)
    return lz4f_compress_fast_device(static_cast<const uint8_t *>(d_in), d_rec_offs, d_rec_lens,
                                     fbase, d_out_offs, d_frame_lens, n, s, &fz);
  return lz4f_compress_device(c, static_cast<const uint8_t *>(d_in), d_rec_offs, d_rec_lens, fbase,
                              d_out_offs, d_frame_lens, n, 1, s, &fz);
}

namespace {

inline uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}
const bool g_prof = getenv("RDK_HIP_PRODUCER_PROF") != nullptr;

int launch(rdk_hip_producer_s *p, Slot &sl) {
  const uint32_t B = p->max_batches, n = sl.nb;
  stage_fence();  // the gather's streaming stores, before the copy engine reads them
  const Meta dm = meta_at(sl.dh_meta, B);
  RDK_HIP_CHECK(hipMemcpyAsync(sl.d_in, sl.h_in, sl.in_used, hipMemcpyHostToDevice, sl.s));
  int rc = rdk_hip_msgset_v2_finalize(sl.d_in, dm.rec_offs, dm.rec_lens, sl.d_out, dm.out_offs,
                                      dm.caps, dm.frame_lens, dm.batch_lens, dm.crcs, n, p->mode,
                                      sl.s);
  if (rc) return rc;
  RDK_HIP_CHECK(hipMemsetAsync(sl.d_cursor, 0, 8, sl.s));
  hipLaunchKernelGGL(pack_to_host_kernel, dim3(n < 2048u ? n : 2048u), dim3(256), 0, sl.s,
                     sl.d_out, dm.out_offs, dm.batch_lens, n, sl.dh_out, dm.pack_offs,
                     sl.d_cursor);
  RDK_HIP_CHECK(hipGetLastError());
  RDK_HIP_CHECK(hipEventRecord(sl.done, sl.s));
  sl.st = INFLIGHT;
  sl.polled = 0;
  return 0;
}

void release(rdk_hip_producer_s *p) {
  for (Slot &sl : p->slots) {
    if (sl.s) (void)hipStreamSynchronize(sl.s);
    if (sl.done) (void)hipEventDestroy(sl.done);
    if (sl.s) (void)hipStreamDestroy(sl.s);
    if (sl.h_in) (void)hipHostFree(sl.h_in);
    if (sl.h_out) (void)hipHostFree(sl.h_out);
    if (sl.h_meta) (void)hipHostFree(sl.h_meta);
    if (sl.d_in) (void)hipFree(sl.d_in);
    if (sl.d_out) (void)hipFree(sl.d_out);
    if (sl.d_cursor) (void)hipFree(sl.d_cursor);
  }
}

}  // namespace

RDK_API rdk_hip_producer_t *rdk_hip_producer_new(int device, size_t slot_bytes, int nslots,
                                                  int mode) {
  if (rdk_hip_init(device)) return nullptr;
  if (nslots < 1 || slot_bytes < 4096 ||
      (mode != RDK_HIP_PRODUCER_EXACT && mode != RDK_HIP_PRODUCER_FAST &&
       mode != RDK_HIP_PRODUCER_SNAPPY)) {
    set_error(RDK_HIP_E_INVAL, "producer: bad arguments");
    return nullptr;
  }
  rdk_hip_producer_s *p = new (std::nothrow) rdk_hip_producer_s();
  if (!p) return nullptr;
  p->device = device;
  p->mode = mode;
  p->slot_bytes = slot_bytes;
  p->max_batches = uint32_t(slot_bytes / 512 + 64);
  // worst case: every batch at most slot_bytes, spans rounded up
  p->out_bytes = out_span(slot_bytes, mode) + size_t(p->max_batches) * 512;
  p->slots.resize(size_t(nslots));
  const size_t mb = meta_bytes(p->max_batches);
  for (Slot &sl : p->slots) {
    if (hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&sl.h_in), slot_bytes, 0) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&sl.h_out), p->out_bytes,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&sl.dh_out), sl.h_out, 0) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&sl.h_meta), mb,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&sl.dh_meta), sl.h_meta, 0) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&sl.d_in), slot_bytes + 256) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&sl.d_out), p->out_bytes) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&sl.d_cursor), 8) != hipSuccess) {
      set_error(RDK_HIP_E_NOMEM, "producer: staging allocation failed");
      release(p);
      delete p;
      return nullptr;
    }
  }
  return p;
}

RDK_API int rdk_hip_producer_produce(rdk_hip_producer_t *p, const void *hdr61, const void *records,
                                     uint32_t len, uint64_t cookie) {
  if (!p || !hdr61 || (!records && len)) return set_error(RDK_HIP_E_INVAL, "null pointer");
  const size_t need_in = (kV2Hdr + size_t(len) + 64 + 15) & ~size_t(15);
  const size_t need_out = out_span(len, p->mode);
  if (need_in > p->slot_bytes || need_out > p->out_bytes)
    return set_error(RDK_HIP_E_INVAL, "batch of %u bytes exceeds the slot", len);
  Slot *sl = &p->slots[size_t(p->fill)];
  if (sl->st == FILLING && (sl->in_used + need_in > p->slot_bytes ||
                            sl->out_used + need_out > p->out_bytes || sl->nb == p->max_batches)) {
    int rc = rdk_hip_producer_flush(p);
    if (rc) return rc;
    sl = &p->slots[size_t(p->fill)];
  }
  if (sl->st == INFLIGHT) return RDK_HIP_E_BUSY;  // the ring is full: poll() first
  if (sl->st == FREE) {
    sl->st = FILLING;
    sl->in_used = sl->out_used = 0;
    sl->nb = 0;
    sl->cookies.clear();
  }
  Meta hm = meta_at(sl->h_meta, p->max_batches);
  std::memcpy(sl->h_in + sl->in_used, hdr61, kV2Hdr);
  const uint64_t g0 = g_prof ? now_ns() : 0;
  if (len) stage_copy(sl->h_in + sl->in_used + kV2Hdr, records, len);
  if (g_prof) p->ns_gather += now_ns() - g0;
  hm.rec_offs[sl->nb] = sl->in_used + kV2Hdr;
  hm.rec_lens[sl->nb] = len;
  hm.out_offs[sl->nb] = sl->out_used;
  hm.caps[sl->nb] = uint32_t(need_out);
  sl->cookies.push_back(cookie);
  sl->in_used += need_in;
  sl->out_used += need_out;
  sl->nb++;
  return RDK_HIP_OK;
}

RDK_API int rdk_hip_producer_flush(rdk_hip_producer_t *p) {
  if (!p) return set_error(RDK_HIP_E_INVAL, "null producer");
  Slot &sl = p->slots[size_t(p->fill)];
  if (sl.st != FILLING || !sl.nb) return RDK_HIP_OK;
  const uint64_t l0 = g_prof ? now_ns() : 0;
  int rc = launch(p, sl);
  if (g_prof) {
    p->ns_launch += now_ns() - l0;
    p->n_launch++;
  }
  if (rc) return rc;
  p->fill = (p->fill + 1) % int(p->slots.size());
  return RDK_HIP_OK;
}

RDK_API int rdk_hip_producer_poll(rdk_hip_producer_t *p, rdk_hip_batch_t *out, int max,
                                  int block) {
  if (!p || (!out && max > 0)) return set_error(RDK_HIP_E_INVAL, "null pointer");
  int got = 0;
  while (got < max) {
    Slot &sl = p->slots[size_t(p->next)];
    if (sl.st != INFLIGHT) break;
    if (sl.polled == 0) {
      const uint64_t w0 = g_prof ? now_ns() : 0;
      const hipError_t e = block ? hipEventSynchronize(sl.done) : hipEventQuery(sl.done);
      if (g_prof) p->ns_wait += now_ns() - w0;
      if (e == hipErrorNotReady) break;
      if (e != hipSuccess)
        return set_error(RDK_HIP_E_HIP, "producer slot: %s", hipGetErrorString(e));
    }
    Meta hm = meta_at(sl.h_meta, p->max_batches);
    while (got < max && sl.polled < sl.nb) {
      const uint32_t i = sl.polled++;
      out[got].data = sl.h_out + hm.pack_offs[i];
      out[got].len = hm.batch_lens[i];
      out[got].crc = hm.crcs[i];
      out[got].cookie = sl.cookies[i];
      ++got;
    }
    if (sl.polled == sl.nb) {
      sl.st = FREE;
      p->next = (p->next + 1) % int(p->slots.size());
    }
  }
  return got;
}

RDK_API void rdk_hip_producer_destroy(rdk_hip_producer_t *p) {
  if (!p) return;
  if (g_prof)
    fprintf(stderr, "producer %p: gather %.1f ms, launch %.1f ms (%llu launches), blocked in poll %.1f ms\n",
            (void *)p, p->ns_gather / 1e6, p->ns_launch / 1e6, (unsigned long long)p->n_launch, p->ns_wait / 1e6);
  release(p);
  delete p;
}
