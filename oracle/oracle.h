/*
 * oracle.h -- CPU restatement of librdkafka's record-batch hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by
 * or called from the product (librdkafka_amd/librdkafka_hip.so).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it,
 * and only as the checker / the timed CPU baseline.
 *
 * Each function cites the reference file:line it restates
 * (reference = bluelichen19/librdkafka v1.3.0 with its vendored lz4 1.9.2).
 *
 * Parity pinning:
 *   - CRC32C: crc32c.c depends on the generated ../config.h (rd.h:64) and is
 *     therefore unbuildable here; the restatement is pinned by the reference's
 *     own known-answer test (crc32c.c:388-438, 0x7dcde113), the standard check
 *     value and an independent bit-serial implementation.
 *   - LZ4 / LZ4F / XXH32: the vendored sources (src/lz4.c, src/lz4frame.c,
 *     src/xxhash.c) compile standalone; oracle/Makefile builds them from
 *     /root/reference into oracle/_ref/ and tests/golden/ holds frames made by
 *     that build.  The restatement below is checked byte-for-byte against it.
 */
#ifndef RDK_ORACLE_H
#define RDK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- CRC32C (Castagnoli, reflected poly 0x82f63b78) ---------------------- */
void     or_crc32c_init(void);
/* crc32c.c:97-134 (slicing-by-8 software path) -- chainable like crc32c(). */
uint32_t or_crc32c(uint32_t crc, const void *buf, size_t len);
/* Independent bit-at-a-time definition, used to cross-check the above. */
uint32_t or_crc32c_bitwise(uint32_t crc, const void *buf, size_t len);
/* crc32c.c:144-231 generalised: crc(A||B) from crc(A), crc(B), len(B). */
uint32_t or_crc32c_combine(uint32_t crcA, uint32_t crcB, size_t lenB);
/* Multi-threaded batch CRC used as the timed CPU baseline (bench.py). */
void     or_crc32c_batches_mt(const uint8_t *base, const uint64_t *offs,
                              const uint32_t *lens, uint32_t *out, size_t n,
                              int threads);
/* Same batch shape through the SSE4.2 crc32q path restated from
 * crc32c.c:255-338 (3-way interleave + shift merge); returns 0 when the
 * host CPU lacks SSE4.2 (caller then uses the table path). */
int      or_crc32c_hw_available(void);
uint32_t or_crc32c_hw(uint32_t crc, const void *buf, size_t len);

/* ---- XXH32 (xxhash.c:392, used for the LZ4F header checksum) ------------- */
uint32_t or_xxh32(const void *p, size_t len, uint32_t seed);

/* ---- LZ4 block codec ----------------------------------------------------- */
/* LZ4_compress_generic(byU16, limitedOutput, noDict, noDictIssue) on a zeroed
 * table, as reached from LZ4F_compressBlock (lz4frame.c:764) through
 * LZ4_compress_fast_extState_fastReset (lz4.c:1211).  Returns the compressed
 * size, or 0 when the block does not fit in dst_cap (LZ4F stores it raw). */
int or_lz4_compress_block(const uint8_t *src, int n, uint8_t *dst, int dst_cap,
                          int acceleration);
/* LZ4_decompress_safe_usingDict (lz4.c:2307 -> 1654) without a dictionary
 * (independent blocks) or with `dict_size` bytes of history directly in front
 * of dst (linked blocks).  Returns decoded size or a negative error. */
int or_lz4_decompress_block(const uint8_t *src, int csize, uint8_t *dst,
                            int dst_cap, int dict_size);
/* LZ4HC hash chain (lz4hc_oracle.c): LZ4HC_compress_hashChain (lz4hc.c:532-746)
 * as LZ4F_compressBlockHC (lz4frame.c:782) reaches it for levels 3..9: fresh
 * window per block, limitedOutput, and LZ4HC_compress_optimal (lz4hc.c:1278)
 * for levels 10..12.  Returns the size, or 0 if it does not fit. */
int or_lz4hc_compress_block(const uint8_t *src, int n, uint8_t *dst, int dst_cap, int level);
/* nbSearches of clTable (lz4hc.c:775-789) for a hash-chain level */
int or_lz4hc_attempts(int level);

/* ---- LZ4F frame ---------------------------------------------------------- */
/* Error codes returned by the rd_kafka_lz4_* restatements (rdkafka.h:258-268) */
#define OR_ERR_NO_ERROR            0
#define OR_ERR__BAD_MSG         (-199)
#define OR_ERR__BAD_COMPRESSION (-198)
#define OR_ERR__CRIT_SYS_RESOURCE (-194)

/* rd_kafka_lz4_compress (rdkafka_lz4.c:329-442) with the reference's prefs
 * {blockIndependent, comp_level}.  Levels 3..9 go through the LZ4HC hash
 * chain (lz4hc_oracle.c); levels >= 10 (LZ4HC optimal) are not restated and
 * return OR_ERR__BAD_COMPRESSION.  *out is malloc()ed. */
int or_rdk_lz4_compress(int proper_hc, int comp_level, const uint8_t *src,
                        size_t len, uint8_t **out, size_t *outlen);
/* rd_kafka_lz4_decompress (rdkafka_lz4.c:167-317): one frame, trailing bytes
 * -> BAD_MSG, decode errors -> BAD_COMPRESSION, truncated frame -> the
 * prefix decoded so far.  May modify in[] when !proper_hc.  *out malloc()ed. */
int or_rdk_lz4_decompress(int proper_hc, uint8_t *in, size_t inlen,
                          uint8_t **out, size_t *outlen);
/* Upper bound used for output buffers (LZ4F_compressBound + 1000). */
size_t or_lz4f_compress_bound(size_t len);
void   or_free(void *p);

/* Multi-threaded frame compression / decompression of independent batches
 * (CPU baseline for the LZ4F legs). Returns 0 on success. */
int or_lz4f_compress_batches_mt(const uint8_t *base, const uint64_t *offs,
                                const uint32_t *lens, size_t n,
                                uint8_t *out, const uint64_t *out_offs,
                                uint32_t *out_lens, int threads);
/* Same at compression.level `level` (3..9: the LZ4HC hash chain). */
int or_lz4f_compress_batches_level_mt(const uint8_t *base, const uint64_t *offs,
                                      const uint32_t *lens, size_t n,
                                      uint8_t *out, const uint64_t *out_offs,
                                      uint32_t *out_lens, int level, int threads);
int or_lz4f_decompress_batches_mt(const uint8_t *base, const uint64_t *offs,
                                  const uint32_t *lens, size_t n,
                                  uint8_t *out, const uint64_t *out_offs,
                                  const uint32_t *out_caps, uint32_t *out_lens,
                                  int threads);


/* ---- MsgVersion 2 records: writer and parser (msgset_oracle.c) -------------- */
/* rdvarint.h:48-75 / :114-141 (zig-zag varints) */
size_t   or_varint_enc_i64(uint8_t *dst, int64_t num);
size_t   or_varint_dec_i64(const uint8_t *src, size_t srcsize, int64_t *nump);
/* rdkafka_msgset_writer.c:352-403 + :652-754 + :1251-1295: one uncompressed batch */
size_t   or_msgset_v2_write(const uint8_t *arena, const int64_t *ts, const uint64_t *key_off,
                            const int32_t *key_len, const uint64_t *val_off,
                            const int32_t *val_len, const uint64_t *hdr_off,
                            const uint32_t *hdr_len, const int32_t *hdr_cnt, uint32_t first,
                            uint32_t cnt, int64_t producer_id, int16_t producer_epoch,
                            int32_t base_sequence, int16_t attributes, uint8_t *out);
/* rdkafka_msgset_reader.c:715-927: index rows of a batch's records */
long     or_msgset_v2_index(const uint8_t *rec, size_t len, int64_t base_offset,
                            int64_t base_ts, int64_t *offset, int64_t *timestamp,
                            uint32_t *key_off, int32_t *key_len, uint32_t *val_off,
                            int32_t *val_len, uint32_t *hdr_off, uint32_t *hdr_len,
                            long max_rows);

/* ---- MsgVersion 0/1 (msgset_oracle.c) ------------------------------------ */
/* zlib crc32() (rdcrc32.h:93-131 WITH_ZLIB), chainable. */
uint32_t or_crc32(uint32_t crc, const void *buf, size_t len);
size_t or_msgset_v01_write(const uint8_t *arena, const int64_t *ts, const uint64_t *key_off,
                           const int32_t *key_len, const uint64_t *val_off,
                           const int32_t *val_len, uint32_t first, uint32_t cnt, int magic,
                           int64_t base_offset, int8_t attributes, uint8_t *out);
long or_msgset_v01_crc(uint8_t *set, size_t len, int mode, uint32_t *pos, uint32_t *out,
                       long max_rows);
/* same walk, CRC through the system zlib (the reference's crc32): the CPU baseline */
long or_msgset_v01_crc_zlib(uint8_t *set, size_t len, int mode, uint32_t *pos, uint32_t *out,
                            long max_rows);

/* ---- snappy (snappy_oracle.c; parity unpinned, see its header) ------------ */
/* rd_kafka_snappy_max_compressed_length (snappy.c:639) */
size_t or_snappy_max_compressed_length(size_t n);
/* rd_kafka_snappy_compress_iov (snappy.c:1488) over one contiguous input */
int or_snappy_compress(const uint8_t *src, size_t n, uint8_t *dst, size_t *outlen);
/* rd_kafka_snappy_uncompressed_length (snappy.c:751): 1 ok, 0 failure */
int or_snappy_uncompressed_length(const uint8_t *p, size_t n, size_t *result);
/* rd_kafka_snappy_uncompress (snappy.c:1572): 0 or -EIO */
int or_snappy_uncompress(const uint8_t *p, size_t n, uint8_t *out);
/* the reader's snappy case (rdkafka_msgset_reader.c:299-390), snappy-java framing
 * included: 0 and a malloc()ed payload (or_free), or an OR_ERR_ code */
int or_rdk_snappy_decompress(const uint8_t *in, size_t inlen, uint8_t **out, size_t *outlen);
/* threaded batch driver for the timed CPU baseline: dec = 0 compress, 1 uncompress */
int or_snappy_batches_mt(const uint8_t *base, const uint64_t *offs, const uint32_t *lens, size_t n,
                         uint8_t *out, const uint64_t *out_offs, uint32_t *out_lens, int dec,
                         int threads);

#ifdef __cplusplus
}
#endif
#endif
