// snappy_host.cpp -- drop-in definitions of the reference's snappy entry points
// (src/snappy.h) for host buffers: stage the bytes on the device, run the snappy
// kernels (snappy.hip), copy the result back.  Host work is limited to what the
// reference also does outside the codec: the iovec gather, the varint32 preamble and
// the snappy-java chunk walk.
#include <hip/hip_runtime.h>
#include <sys/uio.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace rdk {

int snappy_compress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                           uint8_t *d_out, const uint64_t *d_out_offs, uint32_t *d_out_lens,
                           uint32_t n, hipStream_t s);
int snappy_uncompress_device(const uint8_t *d_in, const uint64_t *d_in_offs, const uint32_t *d_in_lens,
                             uint8_t *d_out, const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                             uint32_t *d_out_lens, int32_t *d_status, uint32_t n, hipStream_t s);
size_t snappy_max_compressed_length(size_t len);

static std::atomic<uint64_t> g_sn_calls[2];  // compress, uncompress

// varint_parse32_with_limit (snappy.c:248-290)
static bool sn_varint(const uint8_t *p, size_t n, uint32_t *out) {
  uint32_t r = 0;
  for (int i = 0; i < 5; i++) {
    if (size_t(i) >= n) return false;
    const uint32_t b = p[i];
    r |= (b & 127u) << (7 * i);
    if (i == 4 ? b < 16u : b < 128u) {
      *out = r;
      return true;
    }
  }
  return false;
}

// c->h_stage[0, len) -> one snappy stream in c->h_stage[0, *outlen)
static int sn_compress_staged(Ctx *c, size_t len, size_t *outlen) {
  if (len >= 0x80000000ull) return set_error(RDK_HIP_E_INVAL, "snappy input too large");
  const size_t bound = snappy_max_compressed_length(len);
  const size_t in_bytes = (len + 255) & ~size_t(255);
  int rc;
  // the caller sized the pinned staging for `bound` BEFORE gathering the input into it
  // (ensure_host does not keep contents when it grows)
  if (c->h_cap < bound) return set_error(RDK_HIP_E_INVAL, "snappy staging smaller than the bound");
  if ((rc = ensure_dev(c, 0, in_bytes + bound + 64)) || (rc = ensure_desc(c, 64))) return rc;
  uint8_t *d_in = c->d_stage[0], *d_out = c->d_stage[0] + in_bytes;
  uint64_t *hd = reinterpret_cast<uint64_t *>(c->h_desc);
  hd[0] = 0;
  hd[1] = 0;
  reinterpret_cast<uint32_t *>(hd + 2)[0] = uint32_t(len);
  uint64_t *dd = reinterpret_cast<uint64_t *>(c->d_desc);
  uint32_t *d_len = reinterpret_cast<uint32_t *>(dd + 2), *d_olen = d_len + 1;
  if (len) RDK_HIP_CHECK(hipMemcpyAsync(d_in, c->h_stage, len, hipMemcpyHostToDevice, c->stream));
  RDK_HIP_CHECK(hipMemcpyAsync(dd, hd, 24, hipMemcpyHostToDevice, c->stream));
  if ((rc = snappy_compress_device(d_in, dd, d_len, d_out, dd + 1, d_olen, 1, c->stream))) return rc;
  RDK_HIP_CHECK(hipMemcpyAsync(c->h_desc + 32, d_olen, 4, hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  uint32_t clen;
  std::memcpy(&clen, c->h_desc + 32, 4);
  RDK_HIP_CHECK(hipMemcpyAsync(c->h_stage, d_out, clen, hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  *outlen = clen;
  return 0;
}

// nstreams streams laid out in `in` (offs / lens), outputs back to back in `out`
// (ooffs / declared lengths).  0, -EIO, or a positive engine failure marker.
static int sn_uncompress_many(Ctx *c, const uint8_t *in, size_t inlen, const uint64_t *offs,
                              const uint32_t *lens, const uint64_t *ooffs, const uint32_t *ulens,
                              uint32_t nstreams, uint8_t *out, size_t outlen) {
  const size_t in_bytes = (inlen + 255) & ~size_t(255);
  // descriptor block (32 bytes per stream) + a host copy of the status words behind it
  const size_t desc = (size_t(nstreams) * 32 + 63) & ~size_t(63);
  int rc;
  if ((rc = ensure_host(c, inlen > outlen ? inlen : outlen)) ||
      (rc = ensure_dev(c, 0, in_bytes + outlen + 64)) ||
      (rc = ensure_desc(c, desc + size_t(nstreams) * 4 + 64)))
    return rc;
  uint8_t *d_in = c->d_stage[0], *d_out = c->d_stage[0] + in_bytes;
  // descriptors: in_offs, out_offs (u64 x n) | in_lens, out_caps, out_lens (u32 x n) | status
  uint64_t *hd = reinterpret_cast<uint64_t *>(c->h_desc);
  uint32_t *hw = reinterpret_cast<uint32_t *>(hd + 2 * size_t(nstreams));
  for (uint32_t i = 0; i < nstreams; i++) {
    hd[i] = offs[i];
    hd[nstreams + i] = ooffs[i];
    hw[i] = lens[i];
    hw[nstreams + i] = ulens[i];
  }
  uint64_t *dd = reinterpret_cast<uint64_t *>(c->d_desc);
  uint32_t *dw = reinterpret_cast<uint32_t *>(dd + 2 * size_t(nstreams));
  std::memcpy(c->h_stage, in, inlen);
  if (inlen) RDK_HIP_CHECK(hipMemcpyAsync(d_in, c->h_stage, inlen, hipMemcpyHostToDevice, c->stream));
  RDK_HIP_CHECK(hipMemcpyAsync(dd, hd, size_t(nstreams) * 24, hipMemcpyHostToDevice, c->stream));
  int32_t *d_status = reinterpret_cast<int32_t *>(dw + 3 * size_t(nstreams));
  if ((rc = snappy_uncompress_device(d_in, dd, dw, d_out, dd + nstreams, dw + nstreams,
                                     dw + 2 * size_t(nstreams), d_status, nstreams, c->stream)))
    return rc;
  uint8_t *hs = c->h_desc + desc;
  RDK_HIP_CHECK(hipMemcpyAsync(hs, d_status, size_t(nstreams) * 4, hipMemcpyDeviceToHost, c->stream));
  if (outlen) RDK_HIP_CHECK(hipMemcpyAsync(c->h_stage, d_out, outlen, hipMemcpyDeviceToHost, c->stream));
  RDK_HIP_CHECK(hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < nstreams; i++) {
    int32_t st;
    std::memcpy(&st, hs + size_t(i) * 4, 4);
    if (st) return -EIO;
  }
  if (outlen) std::memcpy(out, c->h_stage, outlen);
  return 0;
}

static void sn_report(const char *who) {
  static std::atomic<int> once{0};
  if (!once.exchange(1)) fprintf(stderr, "librdkafka_hip: %s failed on the device: %s\n", who, last_error());
}

}  // namespace rdk

using namespace rdk;

struct snappy_env {  // src/snappy.h:7-11; nothing is kept in it
  unsigned short *hash_table;
  void *scratch;
  void *scratch_output;
};

RDK_API int rd_kafka_snappy_init_env(struct snappy_env *env) {
  std::memset(env, 0, sizeof(*env));
  return 0;
}
RDK_API int rd_kafka_snappy_init_env_sg(struct snappy_env *env, bool sg) {
  (void)sg;
  return rd_kafka_snappy_init_env(env);
}
RDK_API void rd_kafka_snappy_free_env(struct snappy_env *env) { std::memset(env, 0, sizeof(*env)); }

RDK_API size_t rd_kafka_snappy_max_compressed_length(size_t source_len) {
  return snappy_max_compressed_length(source_len);
}

RDK_API bool rd_kafka_snappy_uncompressed_length(const char *start, size_t n, size_t *result) {
  uint32_t v;
  if (!sn_varint(reinterpret_cast<const uint8_t *>(start), n, &v)) return false;
  *result = v;
  return true;
}

// Replaces rd_kafka_snappy_compress_iov (snappy.c:1488-1507): 0 or a negative errno; the
// writer then sends the MessageSet uncompressed (rdkafka_msgset_writer.c:1065-1077).
RDK_API int rd_kafka_snappy_compress_iov(struct snappy_env *env, const struct iovec *iov_in,
                                         size_t iov_in_cnt, size_t input_length,
                                         struct iovec *iov_out) {
  (void)env;
  g_sn_calls[0]++;
  Ctx *c = ctx();
  if (!c) {
    sn_report("rd_kafka_snappy_compress_iov");
    return -EIO;
  }
  // one sizing for both uses of the staging: the gathered input now, the stream later
  int rc = input_length >= 0x80000000ull
               ? set_error(RDK_HIP_E_INVAL, "snappy input too large")
               : ensure_host(c, snappy_max_compressed_length(input_length));
  size_t of = 0;
  for (size_t i = 0; !rc && i < iov_in_cnt && of < input_length; i++) {
    const size_t take = iov_in[i].iov_len < input_length - of ? iov_in[i].iov_len : input_length - of;
    std::memcpy(c->h_stage + of, iov_in[i].iov_base, take);
    of += take;
  }
  if (!rc && of < input_length) return -EIO;  // sn_compress: the source ran dry (snappy.c:1424)
  size_t clen = 0;
  if (!rc) rc = sn_compress_staged(c, input_length, &clen);
  if (rc) {
    sn_report("rd_kafka_snappy_compress_iov");
    return rc == RDK_HIP_E_NOMEM ? -ENOMEM : -EIO;
  }
  std::memcpy(iov_out->iov_base, c->h_stage, clen);
  iov_out->iov_len = clen;
  return 0;
}

RDK_API int rd_kafka_snappy_compress(struct snappy_env *env, const char *input, size_t input_length,
                                     char *compressed, size_t *compressed_length) {
  struct iovec in = {const_cast<char *>(input), input_length};
  struct iovec out = {compressed, 0xffffffff};
  const int r = rd_kafka_snappy_compress_iov(env, &in, 1, input_length, &out);
  *compressed_length = out.iov_len;
  return r;
}

// Replaces rd_kafka_snappy_uncompress (snappy.c:1572): 0 or -EIO.  `uncompressed` holds
// rd_kafka_snappy_uncompressed_length() bytes, as the reader allocates it.
RDK_API int rd_kafka_snappy_uncompress(const char *compressed, size_t n, char *uncompressed) {
  g_sn_calls[1]++;
  uint32_t ulen;
  const uint8_t *in = reinterpret_cast<const uint8_t *>(compressed);
  // a literal-free stream expands by at most 64/3 per byte (a 3-byte copy element yields
  // up to 64 bytes); anything declared beyond that, or beyond the 31 bits the engine
  // handles, is refused before any staging is sized from the untrusted preamble
  if (n >= 0x80000000ull || !sn_varint(in, n, &ulen) || ulen > 0x7FFFFFF0u ||
      uint64_t(ulen) > uint64_t(n) * 22u + 64u) {
    // read_uncompressed_length accepts a fifth byte up to 127 where the strict parse does
    // not; such a preamble declares more than the 31 bits the engine handles
    return -EIO;
  }
  Ctx *c = ctx();
  if (!c) {
    sn_report("rd_kafka_snappy_uncompress");
    return -EIO;
  }
  const uint64_t off0 = 0;
  const uint32_t len32 = uint32_t(n);
  const int rc = sn_uncompress_many(c, in, n, &off0, &len32, &off0, &ulen, 1,
                                    reinterpret_cast<uint8_t *>(uncompressed), ulen);
  if (rc > 0 || (rc < 0 && rc != -EIO)) sn_report("rd_kafka_snappy_uncompress");
  return rc ? -EIO : 0;
}

// Replaces rd_kafka_snappy_java_uncompress (snappy.c:1588-1697): the chunks behind the
// snappy-java header, all decoded in one launch.  A malloc()ed buffer or NULL + errstr.
RDK_API char *rd_kafka_snappy_java_uncompress(const char *inbuf, size_t inlen, size_t *outlenp,
                                              char *errstr, size_t errstr_size) {
  g_sn_calls[1]++;
  const uint8_t *in = reinterpret_cast<const uint8_t *>(inbuf);
  // pass 1 (snappy.c:1601-1640): chunk table and total length
  size_t of = 0, uof = 0;
  uint32_t nchunks = 0, cap = 0;
  uint64_t *offs = nullptr, *ooffs = nullptr;
  uint32_t *lens = nullptr, *ulens = nullptr;
  auto fail = [&](const char *msg) -> char * {
    std::snprintf(errstr, errstr_size, "%s", msg);
    std::free(offs); std::free(ooffs); std::free(lens); std::free(ulens);
    return nullptr;
  };
  while (of + 4 <= inlen) {
    const uint32_t clen = (uint32_t(in[of]) << 24) | (uint32_t(in[of + 1]) << 16) |
                          (uint32_t(in[of + 2]) << 8) | in[of + 3];
    of += 4;
    if (clen > inlen - of) return fail("Invalid snappy-java chunk length");
    uint32_t ulen;
    if (!sn_varint(in + of, clen, &ulen))
      return fail("Failed to get length of (snappy-java framed) Snappy compressed payload");
    if (nchunks == cap) {
      cap = cap ? cap * 2 : 64;
      offs = static_cast<uint64_t *>(std::realloc(offs, cap * sizeof(uint64_t)));
      ooffs = static_cast<uint64_t *>(std::realloc(ooffs, cap * sizeof(uint64_t)));
      lens = static_cast<uint32_t *>(std::realloc(lens, cap * sizeof(uint32_t)));
      ulens = static_cast<uint32_t *>(std::realloc(ulens, cap * sizeof(uint32_t)));
      if (!offs || !ooffs || !lens || !ulens) return fail("Failed to allocate memory");
    }
    offs[nchunks] = of;
    ooffs[nchunks] = uof;
    lens[nchunks] = clen;
    ulens[nchunks] = ulen;
    nchunks++;
    of += clen;
    uof += ulen;
  }
  if (of != inlen) return fail("trailing bytes in Snappy-java framed compressed data");
  if (uof == 0) return fail("Empty Snappy-java framed data");
  if (inlen >= 0x80000000ull || uof >= 0x80000000ull) return fail("Snappy-java framed data too large");
  char *outbuf = static_cast<char *>(std::malloc(uof));
  if (!outbuf) return fail("Failed to allocate memory for uncompressed Snappy data");
  // pass 2: every chunk in one launch
  Ctx *c = ctx();
  int rc = c ? sn_uncompress_many(c, in, inlen, offs, lens, ooffs, ulens, nchunks,
                                  reinterpret_cast<uint8_t *>(outbuf), uof)
             : RDK_HIP_E_NODEV;
  if (rc) {
    if (rc != -EIO) sn_report("rd_kafka_snappy_java_uncompress");
    std::free(outbuf);
    return fail("Failed to decompress Snappy-java framed payload");
  }
  std::free(offs); std::free(ooffs); std::free(lens); std::free(ulens);
  *outlenp = uof;
  return outbuf;
}

// how often the snappy drop-ins ran: [0] compress, [1] uncompress (bare or snappy-java)
RDK_API void rdk_hip_snappy_dropin_calls(uint64_t out[2]) {
  out[0] = g_sn_calls[0].load();
  out[1] = g_sn_calls[1].load();
}
