// driver.cpp -- TEST INFRASTRUCTURE: broker-like threads calling the drop-in symbols at once
// (rdkafka_broker.c:5082), every result checked; run under ThreadSanitizer against
// hip_stub.cpp.  usage: driver <threads> <iterations> [expect_host_crcs]
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "librdkafka_hip.h"
#include "rdbuf_abi.h"

static uint32_t bitwise(uint32_t poly, uint32_t init, const uint8_t *p, size_t n) {
  uint32_t c = ~init;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? poly : 0u);
  }
  return ~c;
}

static std::atomic<int> g_bad{0};
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "MISMATCH: " __VA_ARGS__);           \
      fprintf(stderr, "\n");                               \
      g_bad++;                                             \
      return;                                              \
    }                                                      \
  } while (0)

struct Slice {  // a slice over `cuts` segments of one buffer, as rd_slice_init_full makes it
  std::vector<rd_segment_t> segs;
  rd_slice_s s;
  Slice(uint8_t *p, size_t n, const std::vector<size_t> &cuts) {
    segs.resize(cuts.size() + 1);
    size_t at = 0;
    for (size_t i = 0; i < segs.size(); ++i) {
      const size_t end = i < cuts.size() ? cuts[i] : n;
      std::memset(&segs[i], 0, sizeof segs[i]);
      segs[i].seg_p = reinterpret_cast<char *>(p + at);
      segs[i].seg_of = segs[i].seg_size = end - at;
      segs[i].seg_absof = at;
      at = end;
    }
    for (size_t i = 0; i + 1 < segs.size(); ++i) segs[i].seg_link.tqe_next = &segs[i + 1];
    s.buf = nullptr;
    s.seg = &segs[0];
    s.rof = 0;
    s.start = 0;
    s.end = n;
  }
};

static void worker(int id, int iters) {
  uint32_t seed = 12345u + 977u * uint32_t(id);
  auto rnd = [&] { return seed = seed * 1664525u + 1013904223u; };
  std::vector<uint8_t> buf(300000);
  for (int it = 0; it < iters; ++it) {
    const size_t n = it % 7 == 0 ? 0 : 1 + rnd() % (it % 5 == 0 ? buf.size() : 20000);
    for (size_t i = 0; i < n; ++i) buf[i] = uint8_t((rnd() >> 24) % (it % 3 ? 7 : 251));
    const uint32_t init = it % 4 == 0 ? rnd() : 0u;
    CHECK(crc32c(init, buf.data(), n) == bitwise(0x82f63b78u, init, buf.data(), n), "crc32c thread %d n %zu", id, n);
    {
      Slice sl(buf.data(), n, n > 100 ? std::vector<size_t>{61, n / 2} : std::vector<size_t>{});
      CHECK(rd_slice_crc32c(reinterpret_cast<rd_slice_t *>(&sl.s)) == bitwise(0x82f63b78u, 0, buf.data(), n),
            "rd_slice_crc32c thread %d n %zu", id, n);
      CHECK(sl.s.end - (sl.s.seg ? sl.s.seg->seg_absof + sl.s.rof : sl.s.end) == 0, "slice not consumed");
    }
    {
      Slice sl(buf.data(), n, n > 100 ? std::vector<size_t>{n / 3} : std::vector<size_t>{});
      CHECK(rd_slice_crc32(reinterpret_cast<rd_slice_t *>(&sl.s)) == bitwise(0xedb88320u, 0, buf.data(), n),
            "rd_slice_crc32 thread %d n %zu", id, n);
    }
    {
      Slice sl(buf.data(), n, n > 100 ? std::vector<size_t>{n / 4, n / 2} : std::vector<size_t>{});
      void *frame = nullptr, *back = nullptr;
      size_t flen = 0, blen = 0;
      const int hc = it % 2, level = it % 6 == 5 ? 9 : 0;
      int rc = rd_kafka_lz4_compress(nullptr, hc, level, reinterpret_cast<rd_slice_t *>(&sl.s), &frame, &flen);
      if (rc) {  // forced device failure: the documented error, nothing owned
        CHECK((rc == RDK_HIP_RESP_ERR__BAD_COMPRESSION || rc == RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE) &&
                  frame == nullptr, "compress rc %d", rc);
        continue;
      }
      rc = rd_kafka_lz4_decompress(nullptr, hc, 0, static_cast<char *>(frame), flen, &back, &blen);
      if (rc) {
        CHECK((rc == RDK_HIP_RESP_ERR__BAD_COMPRESSION || rc == RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE) &&
                  back == nullptr, "decompress rc %d", rc);
        free(frame);
        continue;
      }
      CHECK(blen == n && (n == 0 || !std::memcmp(back, buf.data(), n)), "lz4 round trip thread %d n %zu", id, n);
      free(frame);
      free(back);
    }
    if (it % 11 == 3) {  // a frame that is not one: the frame's own error, per request
      char junk[32] = "not an lz4 frame at all........";
      void *back = nullptr;
      size_t blen = 0;
      CHECK(rd_kafka_lz4_decompress(nullptr, 1, 0, junk, sizeof junk, &back, &blen) ==
                    RDK_HIP_RESP_ERR__BAD_COMPRESSION && back == nullptr, "junk frame");
    }
  }
}

int main(int argc, char **argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 8, iters = argc > 2 ? atoi(argv[2]) : 200;
  for (int wave = 0; wave < 2; ++wave) {  // two generations of threads: contexts end with them
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(worker, wave * 100 + t, iters);
    for (auto &t : ts) t.join();
  }
  uint64_t comb[4], ctxs[2];
  rdk_hip_dropin_combined(comb);
  rdk_hip_ctx_counts(ctxs);
  printf("bad=%d combined_batches=%llu requests=%llu largest=%llu fallbacks=%llu host_crcs=%llu ctx=%llu/%llu\n",
         g_bad.load(), (unsigned long long)comb[0], (unsigned long long)comb[1], (unsigned long long)comb[2],
         (unsigned long long)comb[3], (unsigned long long)rdk_hip_dropin_host_crcs(),
         (unsigned long long)ctxs[0], (unsigned long long)ctxs[1]);
  return g_bad.load() ? 1 : 0;
}
