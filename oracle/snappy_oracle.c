/*
 * snappy_oracle.c -- CPU restatement of the snappy codec that librdkafka v1.3.0
 * vendors (src/snappy.c, the C port of snappy 1.1.0) and of the two call sites
 * that drive it.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Writer: rd_kafka_msgset_writer_compress_snappy (rdkafka_msgset_writer.c:1041)
 *   -> rd_kafka_snappy_compress_iov (snappy.c:1488) -> sn_compress (:1408):
 *   varint32 of the input length, then every 64 KiB fragment through
 *   compress_fragment (:957) with a hash table zeroed per fragment (:790).
 * Reader: rdkafka_msgset_reader.c:299-390: snappy-java framing
 *   (rd_kafka_snappy_java_uncompress, snappy.c:1588) or a bare stream
 *   (rd_kafka_snappy_uncompressed_length :751, rd_kafka_snappy_uncompress :1572
 *   -> internal_uncompress :1383 -> decompress_all_tags :1226).
 *
 * PARITY UNPINNED: snappy.c cannot be compiled here (snappy_compat.h includes
 * rdkafka_int.h and with it the generated config.h), and the reference holds no
 * snappy fixtures.  What the tests can and do check: streams made here decode
 * with an independent implementation of the published format (the snappy
 * bundled in pyarrow) to the input, and streams made by that implementation
 * decode here to its input; byte identity with snappy.c's output is by
 * restatement only.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define SN_BLOCK 65536u               /* kblock_size, snappy.c:774 */
#define SN_MAX_TABLE (1u << 14)       /* kmax_hash_table_size, snappy.c:781 */
#define SN_EIO (-5)

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

size_t or_snappy_max_compressed_length(size_t n) { return 32 + n + n / 6; }   /* snappy.c:639 */

/* emit_literal (snappy.c:652-695); the 16-byte fast path writes the same bytes */
static uint8_t *sn_emit_literal(uint8_t *op, const uint8_t *lit, int len) {
    int n = len - 1;
    if (n < 60) {
        *op++ = (uint8_t)(n << 2);
    } else {
        uint8_t *base = op++;
        int count = 0;
        while (n > 0) { *op++ = (uint8_t)(n & 0xff); n >>= 8; count++; }
        *base = (uint8_t)((59 + count) << 2);
    }
    memcpy(op, lit, (size_t)len);
    return op + len;
}

/* emit_copy_less_than64 / emit_copy (snappy.c:697-741) */
static uint8_t *sn_emit_copy64(uint8_t *op, int offset, int len) {
    if (len < 12 && offset < 2048) {
        *op++ = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
        *op++ = (uint8_t)(offset & 0xff);
    } else {
        *op++ = (uint8_t)(2 + ((len - 1) << 2));
        *op++ = (uint8_t)(offset & 0xff);
        *op++ = (uint8_t)(offset >> 8);
    }
    return op;
}
static uint8_t *sn_emit_copy(uint8_t *op, int offset, int len) {
    while (len >= 68) { op = sn_emit_copy64(op, offset, 64); len -= 64; }
    if (len > 64) { op = sn_emit_copy64(op, offset, 60); len -= 60; }
    return sn_emit_copy64(op, offset, len);
}

/* compress_fragment (snappy.c:957-1103); table zeroed, table_size a power of two */
static uint8_t *sn_compress_fragment(const uint8_t *in, size_t n, uint8_t *op, uint16_t *table,
                                     unsigned table_size) {
    int lg = 0;
    while ((2u << lg) <= table_size) lg++;
    const int shift = 32 - lg;
    const uint8_t *ip = in, *ip_end = in + n, *next_emit = in;
    if (n >= 15) {
        const uint8_t *ip_limit = in + n - 15;
        uint32_t next_hash = (ld32(++ip) * 0x1e35a7bdu) >> shift;
        for (;;) {
            uint32_t skip = 32;
            const uint8_t *next_ip = ip, *cand;
            do {                                   /* :1015-1031 */
                ip = next_ip;
                uint32_t h = next_hash;
                next_ip = ip + (skip++ >> 5);
                if (next_ip > ip_limit) goto remainder;
                next_hash = (ld32(next_ip) * 0x1e35a7bdu) >> shift;
                cand = in + table[h];
                table[h] = (uint16_t)(ip - in);
            } while (ld32(ip) != ld32(cand));
            op = sn_emit_literal(op, next_emit, (int)(ip - next_emit));
            uint32_t at1, cand_bytes;
            do {                                   /* :1054-1088 */
                const uint8_t *base = ip, *s1 = cand + 4, *s2 = ip + 4;
                int matched = 4;
                /* find_match_length (:823-866): 8 bytes at a time, then the tail */
                while (s2 + 8 <= ip_end) {
                    uint64_t a, b;
                    memcpy(&a, s1, 8);
                    memcpy(&b, s2, 8);
                    if (a == b) { s1 += 8; s2 += 8; matched += 8; continue; }
                    matched += __builtin_ctzll(a ^ b) >> 3;
                    goto counted;
                }
                while (s2 < ip_end && *s1 == *s2) { s1++; s2++; matched++; }
            counted:
                ip += matched;
                op = sn_emit_copy(op, (int)(base - cand), matched);
                next_emit = ip;
                if (ip >= ip_limit) goto remainder;
                table[(ld32(ip - 1) * 0x1e35a7bdu) >> shift] = (uint16_t)(ip - in - 1);
                at1 = ld32(ip);
                uint32_t h = (at1 * 0x1e35a7bdu) >> shift;
                cand = in + table[h];
                cand_bytes = ld32(cand);
                table[h] = (uint16_t)(ip - in);
            } while (at1 == cand_bytes);
            next_hash = (ld32(ip + 1) * 0x1e35a7bdu) >> shift;
            ++ip;
        }
    }
remainder:
    if (next_emit < ip_end) op = sn_emit_literal(op, next_emit, (int)(ip_end - next_emit));
    return op;
}

/* sn_compress (snappy.c:1408-1484) over one contiguous input (the iovec gather of
 * rd_kafka_snappy_compress_iov changes no byte).  dst holds
 * or_snappy_max_compressed_length(n) bytes.  Returns 0. */
int or_snappy_compress(const uint8_t *src, size_t n, uint8_t *dst, size_t *outlen) {
    uint16_t *table = (uint16_t *)malloc(SN_MAX_TABLE * sizeof(uint16_t));
    if (!table) return -12;
    uint8_t *op = dst;
    uint32_t v = (uint32_t)n;                      /* varint_encode32, snappy.c:297 */
    while (v >= 128) { *op++ = (uint8_t)(v | 128); v >>= 7; }
    *op++ = (uint8_t)v;
    for (size_t pos = 0; pos < n; pos += SN_BLOCK) {
        const size_t fn = n - pos < SN_BLOCK ? n - pos : SN_BLOCK;
        unsigned ht = 256;                         /* get_hash_table, snappy.c:790-807 */
        while (ht < SN_MAX_TABLE && ht < fn) ht <<= 1;
        memset(table, 0, ht * sizeof(uint16_t));
        op = sn_compress_fragment(src + pos, fn, op, table, ht);
    }
    free(table);
    *outlen = (size_t)(op - dst);
    return 0;
}

/* rd_kafka_snappy_uncompressed_length (snappy.c:751) = varint_parse32_with_limit (:248) */
int or_snappy_uncompressed_length(const uint8_t *p, size_t n, size_t *result) {
    uint32_t r = 0;
    for (int i = 0; i < 5; i++) {
        if ((size_t)i >= n) return 0;
        const uint32_t b = p[i];
        r |= (b & 127) << (7 * i);
        if (i == 4 ? b < 16 : b < 128) { *result = r; return 1; }
        if (i == 4) return 0;
    }
    return 0;
}

/* rd_kafka_snappy_uncompress (snappy.c:1572) -> internal_uncompress (:1383): 0 or -EIO.
 * out holds the declared length. */
int or_snappy_uncompress(const uint8_t *p, size_t n, uint8_t *out) {
    size_t ip = 0;
    uint32_t ulen = 0, shift = 0;
    for (;;) {                                     /* read_uncompressed_length, :1193-1218 */
        if (shift >= 32 || ip >= n) return SN_EIO;
        const uint8_t c = p[ip++];
        ulen |= (uint32_t)(c & 0x7f) << shift;
        if (c < 128) break;
        shift += 7;
    }
    size_t op = 0;
    for (;;) {                                     /* decompress_all_tags, :1226-1312 */
        if (ip == n) break;                        /* refill_tag: end of input at a tag */
        const uint8_t c = p[ip];
        const unsigned kind = c & 3;
        /* bytes after the tag that belong to the element header (char_table, :1129) */
        const unsigned extra = kind == 0 ? ((c >> 2) >= 60 ? (unsigned)(c >> 2) - 59 : 0)
                             : kind == 1 ? 1 : kind == 2 ? 2 : 4;
        if (n - ip < 1 + extra) return SN_EIO;     /* refill_tag cannot complete the header */
        ip++;
        uint32_t trailer = 0;
        for (unsigned i = 0; i < extra; i++) trailer |= (uint32_t)p[ip + i] << (8 * i);
        ip += extra;
        if (kind == 0) {
            const uint64_t len = (c >> 2) < 60 ? (uint64_t)(c >> 2) + 1 : (uint64_t)trailer + 1;
            if (n - ip < len) return SN_EIO;       /* premature end of input (:1283) */
            if (ulen - op < len) return SN_EIO;    /* writer_append (:572) */
            memcpy(out + op, p + ip, (size_t)len);
            op += (size_t)len;
            ip += (size_t)len;
        } else {
            const uint32_t len = kind == 1 ? 4u + ((uint32_t)(c >> 2) & 7u) : 1u + (uint32_t)(c >> 2);
            const uint32_t off = kind == 1 ? ((uint32_t)(c >> 5) << 8) | trailer : trailer;
            if ((uint32_t)op <= off - 1u) return SN_EIO;   /* writer_append_from_self (:543) */
            if (ulen - op < len) return SN_EIO;
            if (off >= len) {                      /* no overlap: one block copy */
                memcpy(out + op, out + op - off, len);
            } else {                               /* incremental_copy (:484): the pattern repeats */
                for (uint32_t i = 0; i < len; i++) out[op + i] = out[op + i - off];
            }
            op += len;
        }
    }
    return op == ulen ? 0 : SN_EIO;                /* eof && writer_check_length (:1403) */
}

/* rd_kafka_snappy_java_uncompress (snappy.c:1588-1697) on the bytes behind the 16-byte
 * snappy-java header.  0 and a malloc()ed buffer, or -1. */
static int sn_java_uncompress(const uint8_t *in, size_t inlen, uint8_t **out, size_t *outlen) {
    uint8_t *buf = NULL;
    for (int pass = 1; pass <= 2; pass++) {
        size_t of = 0, uof = 0;
        while (of + 4 <= inlen) {
            const uint32_t clen = ((uint32_t)in[of] << 24) | ((uint32_t)in[of + 1] << 16) |
                                  ((uint32_t)in[of + 2] << 8) | in[of + 3];
            size_t ulen;
            of += 4;
            if (clen > inlen - of) { free(buf); return -1; }
            if (!or_snappy_uncompressed_length(in + of, clen, &ulen)) { free(buf); return -1; }
            if (pass == 2 && or_snappy_uncompress(in + of, clen, buf + uof)) { free(buf); return -1; }
            of += clen;
            uof += ulen;
        }
        if (of != inlen) { free(buf); return -1; }
        if (pass == 1) {
            if (uof == 0) return -1;               /* "Empty Snappy-java framed data" */
            buf = (uint8_t *)malloc(uof);
            if (!buf) return -1;
        } else {
            *outlen = uof;
        }
    }
    *out = buf;
    return 0;
}

/* The reader's RD_KAFKA_COMPRESSION_SNAPPY case (rdkafka_msgset_reader.c:299-390):
 * 0 with a malloc()ed payload (free with or_free), or __BAD_COMPRESSION. */
int or_rdk_snappy_decompress(const uint8_t *in, size_t inlen, uint8_t **out, size_t *outlen) {
    static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    *out = NULL;
    *outlen = 0;
    if (inlen > 16 + 4 && !memcmp(in, magic, 8))
        return sn_java_uncompress(in + 16, inlen - 16, out, outlen) ? OR_ERR__BAD_COMPRESSION : 0;
    size_t ulen;
    if (!or_snappy_uncompressed_length(in, inlen, &ulen)) return OR_ERR__BAD_COMPRESSION;
    uint8_t *buf = (uint8_t *)malloc(ulen ? ulen : 1);
    if (!buf) return OR_ERR__CRIT_SYS_RESOURCE;
    if (or_snappy_uncompress(in, inlen, buf)) { free(buf); return OR_ERR__BAD_COMPRESSION; }
    *out = buf;
    *outlen = ulen;
    return 0;
}

/* ---- threaded drivers (bench.py's cpu_baseline leg) ----------------------- */
#include <pthread.h>

struct sn_job {
    const uint8_t *base; const uint64_t *offs; const uint32_t *lens; size_t lo, hi;
    uint8_t *out; const uint64_t *out_offs; uint32_t *out_lens; int dec; int rc;
};

static void *sn_worker(void *arg) {
    struct sn_job *j = (struct sn_job *)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        if (j->dec) {
            size_t ulen;
            if (!or_snappy_uncompressed_length(j->base + j->offs[i], j->lens[i], &ulen) ||
                or_snappy_uncompress(j->base + j->offs[i], j->lens[i], j->out + j->out_offs[i])) {
                j->rc = SN_EIO;
                continue;
            }
            j->out_lens[i] = (uint32_t)ulen;
        } else {
            size_t clen;
            if (or_snappy_compress(j->base + j->offs[i], j->lens[i], j->out + j->out_offs[i], &clen)) {
                j->rc = -12;
                continue;
            }
            j->out_lens[i] = (uint32_t)clen;
        }
    }
    return NULL;
}

/* n inputs -> n streams (dec = 0) or n streams -> n payloads (dec = 1) on `threads` threads;
 * every output slot holds the bound / the declared length */
int or_snappy_batches_mt(const uint8_t *base, const uint64_t *offs, const uint32_t *lens, size_t n,
                         uint8_t *out, const uint64_t *out_offs, uint32_t *out_lens, int dec,
                         int threads) {
    if (threads < 1) threads = 1;
    if (threads > 512) threads = 512;
    pthread_t th[512];
    struct sn_job jobs[512];
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (struct sn_job){base, offs, lens, n * t / threads, n * (t + 1) / threads,
                                  out, out_offs, out_lens, dec, 0};
        pthread_create(&th[t], NULL, sn_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); if (jobs[t].rc) rc = jobs[t].rc; }
    return rc;
}
