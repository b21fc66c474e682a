// hostcopy.cpp -- host memcpy into pinned staging with non-temporal stores.
//
// A staging buffer is written once by a broker thread and then read by the GPU's DMA engine.
// Ordinary stores leave the lines dirty in the CPU caches: every line is first read for
// ownership, and the DMA read then has to pull it back out of a cache.  Streaming stores
// go to memory directly (glibc's memcpy only switches to streaming stores far above a 1 MiB
// batch).  Measured on the producer front-end the two are within noise of each other on an
// MI355X host (the pipeline is bound elsewhere); the streaming form is kept because it leaves
// the broker thread's caches to the application.
#include <immintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace rdk {

__attribute__((target("avx2"))) static void stream_avx2(uint8_t *d, const uint8_t *s, size_t n) {
  // d is 32-byte aligned, n a multiple of 128
  for (size_t i = 0; i < n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 96), e);
  }
}

// memcpy whose bulk goes through streaming stores.  The caller issues stage_fence() before
// the device is told to read the buffer.
void stage_copy(void *dst, const void *src, size_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  uint8_t *d = static_cast<uint8_t *>(dst);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  if (!avx2 || n < 4096) {
    std::memcpy(d, s, n);
    return;
  }
  const size_t head = (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31;
  std::memcpy(d, s, head);
  const size_t bulk = (n - head) & ~size_t(127);
  stream_avx2(d + head, s + head, bulk);
  std::memcpy(d + head + bulk, s + head + bulk, n - head - bulk);
}

void stage_fence() { _mm_sfence(); }

}  // namespace rdk
