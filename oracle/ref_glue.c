/*
 * ref_glue.c -- thin driver that calls the REFERENCE's own vendored LZ4F /
 * LZ4 / XXH32 sources (compiled in place from /root/reference/src by
 * oracle/Makefile into oracle/_ref/libreflz4.so).
 * TEST INFRASTRUCTURE ONLY.
 *
 * rdkafka_lz4.c itself cannot be compiled here (it needs rdkafka_int.h and the
 * generated config.h), so its two entry points are re-driven through the same
 * public LZ4F calls with the same preferences and the same outer loop:
 *   ref_rdk_lz4_compress   <- rd_kafka_lz4_compress   (rdkafka_lz4.c:329-442)
 *   ref_rdk_lz4_decompress <- rd_kafka_lz4_decompress (rdkafka_lz4.c:167-317)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define LZ4_STATIC_LINKING_ONLY
#define LZ4_HC_STATIC_LINKING_ONLY
#include "lz4.h"
#include "lz4frame.h"
#include "lz4hc.h"
#include "xxhash.h"

#define ERR_BAD_MSG (-199)
#define ERR_BAD_COMPRESSION (-198)
#define ERR_CRIT_SYS_RESOURCE (-194)

uint32_t ref_xxh32(const void *p, size_t len, uint32_t seed) {
    return XXH32(p, len, seed);
}

int ref_lz4_decompress_safe(const char *src, char *dst, int csize, int cap) {
    return LZ4_decompress_safe(src, dst, csize, cap);
}

/* One LZ4F block exactly as LZ4F_compressBlock reaches it: a fresh stream
 * state, fastReset, dstCapacity = srcSize-1 (lz4frame.c:739-773). */
int ref_lz4_compress_block(const char *src, int n, char *dst, int cap, int accel) {
    LZ4_stream_t st;
    LZ4_initStream(&st, sizeof st);
    return LZ4_compress_fast_extState_fastReset(&st, src, dst, n, cap, accel);
}

/* One LZ4HC block as LZ4F_compressBlockHC reaches it (lz4frame.c:782-789):
 * LZ4_compress_HC_extStateHC_fastReset, dstCapacity = srcSize-1. */
int ref_lz4hc_compress_block(const char *src, int n, char *dst, int cap, int level) {
    static __thread LZ4_streamHC_t st;
    LZ4_initStreamHC(&st, sizeof st);
    return LZ4_compress_HC_extStateHC_fastReset(&st, src, dst, n, cap, level);
}

static int break_framing(char *out, size_t outlen) {
    static const char magic[4] = {0x04, 0x22, 0x4d, 0x18};
    size_t of = 4;
    if (outlen < 7 || memcmp(out, magic, 4)) return ERR_BAD_COMPRESSION;
    uint8_t FLG = (uint8_t)out[of++];
    of++;
    if ((FLG >> 3) & 1) of += 8;
    if (of >= outlen) return ERR_BAD_COMPRESSION;
    out[of] = (char)((XXH32(out, of, 0) >> 8) & 0xff);
    return 0;
}

static int fixup_framing(char *in, size_t inlen) {
    static const char magic[4] = {0x04, 0x22, 0x4d, 0x18};
    size_t of = 4;
    if (inlen < 7 || memcmp(in, magic, 4)) return ERR_BAD_COMPRESSION;
    uint8_t FLG = (uint8_t)in[of++];
    of++;
    if ((FLG >> 3) & 1) of += 8;
    if (of >= inlen) return ERR_BAD_COMPRESSION;
    in[of] = (char)((XXH32(in + 4, of - 4, 0) >> 8) & 0xff);
    return 0;
}

/* Segments are passed as an iovec-like (ptr,len) list to reproduce the
 * per-rd_slice-segment LZ4F_compressUpdate calls of rdkafka_lz4.c:390-407. */
int ref_rdk_lz4_compress(int proper_hc, int comp_level, const char *const *segs,
                         const size_t *seglens, int nsegs, char **outbuf,
                         size_t *outlenp) {
    LZ4F_compressionContext_t cctx;
    size_t len = 0, out_of = 0, r;
    for (int i = 0; i < nsegs; i++) len += seglens[i];
    LZ4F_preferences_t prefs;
    memset(&prefs, 0, sizeof prefs);
    prefs.frameInfo.blockMode = LZ4F_blockIndependent;
    prefs.compressionLevel = comp_level;
    *outbuf = NULL;
    size_t out_sz = LZ4F_compressBound(len, NULL) + 1000;
    char *out = malloc(out_sz);
    if (!out) return ERR_CRIT_SYS_RESOURCE;
    if (LZ4F_isError(LZ4F_createCompressionContext(&cctx, LZ4F_VERSION))) {
        free(out);
        return ERR_CRIT_SYS_RESOURCE;
    }
    int err = 0;
    r = LZ4F_compressBegin(cctx, out, out_sz, &prefs);
    if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
    out_of += r;
    for (int i = 0; i < nsegs; i++) {
        if (!seglens[i]) continue;
        r = LZ4F_compressUpdate(cctx, out + out_of, out_sz - out_of, segs[i], seglens[i], NULL);
        if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
        out_of += r;
    }
    r = LZ4F_compressEnd(cctx, out + out_of, out_sz - out_of, NULL);
    if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
    out_of += r;
    if (!proper_hc && (err = break_framing(out, out_of))) goto done;
    *outbuf = out;
    *outlenp = out_of;
done:
    LZ4F_freeCompressionContext(cctx);
    if (err) free(out);
    return err;
}

/* max_msg_size plays the role of rkb->rkb_rk->rk_conf.max_msg_size;
 * *zbuf_grow counts the x1.75 regrowths (rdkafka_lz4.c:268-286). */
int ref_rdk_lz4_decompress(int proper_hc, char *inbuf, size_t inlen,
                           size_t max_msg_size, char **outbuf, size_t *outlenp,
                           int *zbuf_grow) {
    LZ4F_decompressionContext_t dctx;
    LZ4F_frameInfo_t fi;
    size_t in_sz, out_sz, in_of, out_of, r, est, outlen;
    int err = 0;
    char *out = NULL;
    *outbuf = NULL;
    *zbuf_grow = 0;
    if (LZ4F_isError(LZ4F_createDecompressionContext(&dctx, LZ4F_VERSION)))
        return ERR_CRIT_SYS_RESOURCE;
    if (!proper_hc && (err = fixup_framing(inbuf, inlen))) goto done;
    in_sz = inlen;
    r = LZ4F_getFrameInfo(dctx, &fi, inbuf, &in_sz);
    if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
    if (fi.contentSize == 0 || fi.contentSize > inlen * 255)
        est = inlen * 4 < max_msg_size ? inlen * 4 : max_msg_size;
    else
        est = (size_t)fi.contentSize;
    out = malloc(est ? est : 1);
    if (!out) { err = ERR_CRIT_SYS_RESOURCE; goto done; }
    outlen = est;
    in_of = in_sz;
    out_of = 0;
    while (in_of < inlen) {
        out_sz = outlen - out_of;
        in_sz = inlen - in_of;
        r = LZ4F_decompress(dctx, out + out_of, &out_sz, inbuf + in_of, &in_sz, NULL);
        if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
        out_of += out_sz;
        in_of += in_sz;
        if (r == 0) break;
        if (out_of == outlen) {
            size_t extra = outlen * 3 / 4 > 1024 ? outlen * 3 / 4 : 1024;
            char *tmp;
            (*zbuf_grow)++;
            if (!(tmp = realloc(out, outlen + extra))) { err = ERR_CRIT_SYS_RESOURCE; goto done; }
            out = tmp;
            outlen += extra;
        }
    }
    if (in_of < inlen) { err = ERR_BAD_MSG; goto done; }
    *outbuf = out;
    *outlenp = out_of;
done:
    LZ4F_freeDecompressionContext(dctx);
    if (err && out) free(out);
    return err;
}

void ref_free(void *p) { free(p); }

/* Frames with non-default preferences (linked blocks, larger blocks, block /
 * content checksums, content size, small flushed blocks) made by the
 * reference LZ4F encoder, to exercise every decode path.  `flush_every` > 0
 * calls LZ4F_flush after each chunk of that many bytes (irregular blocks). */
int ref_lz4f_compress_prefs(const char *src, size_t len, int block_linked, int block_size_id,
                            int block_checksum, int content_checksum, int content_size,
                            int level, size_t flush_every, char **outbuf, size_t *outlenp) {
    LZ4F_compressionContext_t cctx;
    LZ4F_preferences_t prefs;
    size_t out_of = 0, r;
    memset(&prefs, 0, sizeof prefs);
    prefs.frameInfo.blockMode = block_linked ? LZ4F_blockLinked : LZ4F_blockIndependent;
    prefs.frameInfo.blockSizeID = (LZ4F_blockSizeID_t)block_size_id;
    prefs.frameInfo.blockChecksumFlag = block_checksum ? LZ4F_blockChecksumEnabled : LZ4F_noBlockChecksum;
    prefs.frameInfo.contentChecksumFlag = content_checksum ? LZ4F_contentChecksumEnabled : LZ4F_noContentChecksum;
    prefs.frameInfo.contentSize = content_size ? len : 0;
    prefs.compressionLevel = level;
    size_t out_sz = LZ4F_compressBound(len, &prefs) * 2 + 4096 + (flush_every ? (len / flush_every + 1) * 16 : 0);
    char *out = malloc(out_sz);
    *outbuf = NULL;
    if (!out) return ERR_CRIT_SYS_RESOURCE;
    if (LZ4F_isError(LZ4F_createCompressionContext(&cctx, LZ4F_VERSION))) { free(out); return ERR_CRIT_SYS_RESOURCE; }
    int err = 0;
    r = LZ4F_compressBegin(cctx, out, out_sz, &prefs);
    if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
    out_of += r;
    size_t step = flush_every ? flush_every : (len ? len : 1);
    for (size_t pos = 0; pos < len; pos += step) {
        size_t n = len - pos < step ? len - pos : step;
        r = LZ4F_compressUpdate(cctx, out + out_of, out_sz - out_of, src + pos, n, NULL);
        if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
        out_of += r;
        if (flush_every) {
            r = LZ4F_flush(cctx, out + out_of, out_sz - out_of, NULL);
            if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
            out_of += r;
        }
    }
    r = LZ4F_compressEnd(cctx, out + out_of, out_sz - out_of, NULL);
    if (LZ4F_isError(r)) { err = ERR_BAD_COMPRESSION; goto done; }
    out_of += r;
    *outbuf = out;
    *outlenp = out_of;
done:
    LZ4F_freeCompressionContext(cctx);
    if (err) free(out);
    return err;
}

/* ---- timed CPU baseline: many batches on `threads` host threads, each batch through
 * the drivers above, i.e. through the reference's own compiled lz4frame.c / lz4.c /
 * lz4hc.c with rd_kafka_lz4_compress's / _decompress's allocation pattern (malloc of
 * LZ4F_compressBound+1000 and a fresh LZ4F context per call, rdkafka_lz4.c:351-376;
 * inlen*4 estimate and x1.75 regrowth, :218-286).  out_lens[i] = frame / payload size;
 * the bytes are copied to out + out_offs[i] when out is not NULL. */
#include <pthread.h>

struct ref_job {
    int decompress, level, threads, tid;
    const char *base;
    const uint64_t *offs;
    const uint32_t *lens;
    size_t n, max_msg_size;
    char *out;
    const uint64_t *out_offs;
    uint32_t *out_lens;
    int err;
};

static void *ref_worker(void *arg) {
    struct ref_job *j = arg;
    for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->threads) {
        char *o = NULL;
        size_t olen = 0;
        int e;
        if (j->decompress) {
            int grow;
            /* the reader hands rd_kafka_lz4_decompress a contiguous, writable slice */
            e = ref_rdk_lz4_decompress(1, (char *)j->base + j->offs[i], j->lens[i],
                                       j->max_msg_size, &o, &olen, &grow);
        } else {
            const char *seg = j->base + j->offs[i];
            size_t sl = j->lens[i];
            e = ref_rdk_lz4_compress(1, j->level, &seg, &sl, 1, &o, &olen);
        }
        if (e) { j->err = e; continue; }
        j->out_lens[i] = (uint32_t)olen;
        if (j->out) memcpy(j->out + j->out_offs[i], o, olen);
        free(o);
    }
    return NULL;
}

static int ref_run_mt(struct ref_job proto, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    struct ref_job jobs[256];
    int err = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].threads = threads;
        jobs[t].tid = t;
        jobs[t].err = 0;
        pthread_create(&th[t], NULL, ref_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].err) err = jobs[t].err;
    }
    return err;
}

int ref_lz4f_compress_batches_mt(const char *base, const uint64_t *offs, const uint32_t *lens,
                                 size_t n, char *out, const uint64_t *out_offs,
                                 uint32_t *out_lens, int level, int threads) {
    struct ref_job p = {0};
    p.level = level; p.base = base; p.offs = offs; p.lens = lens; p.n = n;
    p.out = out; p.out_offs = out_offs; p.out_lens = out_lens;
    return ref_run_mt(p, threads);
}

int ref_lz4f_decompress_batches_mt(const char *base, const uint64_t *offs, const uint32_t *lens,
                                   size_t n, size_t max_msg_size, char *out,
                                   const uint64_t *out_offs, uint32_t *out_lens, int threads) {
    struct ref_job p = {0};
    p.decompress = 1; p.base = base; p.offs = offs; p.lens = lens; p.n = n;
    p.max_msg_size = max_msg_size;
    p.out = out; p.out_offs = out_offs; p.out_lens = out_lens;
    return ref_run_mt(p, threads);
}
