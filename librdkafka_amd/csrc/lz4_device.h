// lz4_device.h -- device helpers shared by the LZ4 block encoder/decoder.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rdk {

typedef __attribute__((address_space(1))) const uint8_t g_cu8;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
typedef __attribute__((address_space(1))) uint32_t g_u32;

constexpr int kLz4MinMatch = 4;
constexpr int kLz4LastLiterals = 5;   // lz4.c:192
constexpr int kLz4MFLimit = 12;       // lz4.c:193
constexpr uint32_t kLz4Block = 65536; // LZ4F max64KB (lz4frame.c:212)

__device__ __forceinline__ uint32_t ldb(uintptr_t a) { return *(g_cu8 *)a; }
__device__ __forceinline__ void stb(uintptr_t a, uint32_t v) { *(g_u8 *)a = uint8_t(v); }

// little-endian 32-bit read at any byte address through aligned dword loads
// (the second load only when the word straddles, so nothing past the dword
// holding byte a+3 is touched)
__device__ __forceinline__ uint32_t ld32u(uintptr_t a) {
  const uintptr_t b = a & ~uintptr_t(3);
  const uint32_t lo = *(g_cu32 *)b;
  uint32_t hi = 0;
  if (a & 3u) hi = *(g_cu32 *)(b + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, uint32_t(a & 3u));
}

// the same through two unconditional loads (no branch, so the loads can stay in flight
// across the code that follows); the caller guarantees that the dword behind the one holding
// byte a may be read
__device__ __forceinline__ uint32_t ld32u_nb(uintptr_t a) {
  const uintptr_t b = a & ~uintptr_t(3);
  const uint32_t lo = *(g_cu32 *)b;
  const uint32_t hi = *(g_cu32 *)(b + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, uint32_t(a & 3u));
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// lane mask of a predicate, straight from the compare (HIP's __ballot takes an int and
// costs a 0/1 round trip through a VGPR)
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ int ffs64(uint64_t m) { return m ? __builtin_ctzll(m) : 64; }

// Lanes of `among` whose NBITS-bit value h equals this lane's: one ballot per bit, and per
// bit and mask half one v_bitop3_b32 (eq & ~(ballot ^ own bit), truth table 0x90).
template <int NBITS>
__device__ __forceinline__ uint64_t same_value_lanes(uint32_t h, uint64_t among) {
  uint32_t lo = uint32_t(among), hi = uint32_t(among >> 32);
#pragma unroll
  for (int bit = 0; bit < NBITS; ++bit) {
    const int m = __builtin_amdgcn_sbfe(int(h), bit, 1);  // 0 or -1
    const uint64_t bm = ballot(m < 0);
    lo = __builtin_amdgcn_bitop3_b32(lo, uint32_t(bm), uint32_t(m), 0x90);
    hi = __builtin_amdgcn_bitop3_b32(hi, uint32_t(bm >> 32), uint32_t(m), 0x90);
  }
  return (uint64_t(hi) << 32) | lo;
}

// XXH32 (xxhash.c) over [p, p+len) by one lane; used only for frames that
// carry block/content checksums (never set by librdkafka's own frames).
__device__ inline uint32_t xxh32_lane(uintptr_t p, uint64_t len, uint32_t seed) {
  const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                 P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  uintptr_t e = p + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uintptr_t lim = e - 16;
    do {
      v1 = rotl(v1 + ld32u(p) * P2, 13) * P1;
      v2 = rotl(v2 + ld32u(p + 4) * P2, 13) * P1;
      v3 = rotl(v3 + ld32u(p + 8) * P2, 13) * P1;
      v4 = rotl(v4 + ld32u(p + 12) * P2, 13) * P1;
      p += 16;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  } else {
    h = seed + P5;
  }
  h += uint32_t(len);
  while (p + 4 <= e) { h += ld32u(p) * P3; h = rotl(h, 17) * P4; p += 4; }
  while (p < e) { h += ldb(p) * P5; h = rotl(h, 11) * P1; p++; }
  h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
  return h;
}

}  // namespace rdk
