/*
 * lz4_oracle.c -- CPU restatement of the LZ4 / LZ4F / XXH32 code that
 * librdkafka v1.3.0 runs on its record-batch path (vendored lz4 1.9.2).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The product never links this file.  It exists to check the HIP engine and
 * is itself checked byte-for-byte against the reference sources compiled by
 * oracle/Makefile into oracle/_ref/ (tests/test_oracle_vs_ref.py).
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MINMATCH 4
#define LASTLITERALS 5   /* lz4.c:192 */
#define MFLIMIT 12       /* lz4.c:193 */
#define ML_BITS 4
#define ML_MASK 15u
#define RUN_MASK 15u
#define HASHLOG_U16 13   /* LZ4_HASHLOG+1 for byU16, lz4.c:633 */
#define LZ4_64KLIMIT (65536 + MFLIMIT - 1) /* lz4.c:566 */
#define FASTLOOP_SAFE_DISTANCE 64
#define MATCH_SAFEGUARD_DISTANCE 12 /* (2*WILDCOPYLENGTH)-MINMATCH, lz4.c:194 */

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint32_t rd_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void wr_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* ======================================================================= */
/* XXH32 -- xxhash.c:392 (XXH32) restated.                                  */
/* ======================================================================= */
#define P32_1 2654435761u
#define P32_2 2246822519u
#define P32_3 3266489917u
#define P32_4 668265263u
#define P32_5 374761393u
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t xxh_round(uint32_t acc, uint32_t in) {
    return rotl32(acc + in * P32_2, 13) * P32_1;
}

uint32_t or_xxh32(const void *input, size_t len, uint32_t seed) {
    const uint8_t *p = (const uint8_t *)input, *end = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + P32_1 + P32_2, v2 = seed + P32_2, v3 = seed, v4 = seed - P32_1;
        const uint8_t *limit = end - 16;
        do {
            v1 = xxh_round(v1, rd_le32(p)); v2 = xxh_round(v2, rd_le32(p + 4));
            v3 = xxh_round(v3, rd_le32(p + 8)); v4 = xxh_round(v4, rd_le32(p + 12));
            p += 16;
        } while (p <= limit);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P32_5;
    }
    h += (uint32_t)len;
    while (p + 4 <= end) { h += rd_le32(p) * P32_3; h = rotl32(h, 17) * P32_4; p += 4; }
    while (p < end) { h += (*p++) * P32_5; h = rotl32(h, 11) * P32_1; }
    h ^= h >> 15; h *= P32_2; h ^= h >> 13; h *= P32_3; h ^= h >> 16;
    return h;
}

/* ======================================================================= */
/* LZ4 block compression: LZ4_compress_generic (lz4.c:789-1177) for the     */
/* case the LZ4F frame code reaches (byU16 table, zeroed per block,         */
/* limitedOutput with dstCapacity = srcSize-1, noDict, noDictIssue).        */
/* ======================================================================= */
static inline uint32_t hash4_u16(uint32_t seq) {      /* LZ4_hash4, lz4.c:631 */
    return (seq * 2654435761u) >> (32 - HASHLOG_U16);
}

/* LZ4_count (lz4.c:536-558): bytes equal from pIn/pMatch, never past limit. */
static int lz4_count(const uint8_t *s, int in, int match, int limit) {
    int start = in;
    while (in < limit && s[in] == s[match]) { in++; match++; }
    return in - start;
}

int or_lz4_compress_block(const uint8_t *src, int n, uint8_t *dst, int dst_cap,
                          int acceleration) {
    uint16_t table[1 << HASHLOG_U16];
    const int mflimitPlusOne = n - MFLIMIT + 1;   /* lz4.c:821 */
    const int matchlimit = n - LASTLITERALS;      /* lz4.c:822 */
    const int olimit = dst_cap;
    int ip = 0, anchor = 0, op = 0, match = 0, token = 0;
    uint32_t forwardH;

    if (acceleration < 1) acceleration = 1;
    if (n < 0 || n >= LZ4_64KLIMIT) return 0;     /* lz4.c:855 */
    memset(table, 0, sizeof table);               /* LZ4_prepareTable reset */
    if (n < MFLIMIT + 1) goto last_literals;      /* LZ4_minLength, lz4.c:876 */

    table[hash4_u16(rd32(src))] = 0;              /* first byte, lz4.c:879 */
    ip = 1;
    forwardH = hash4_u16(rd32(src + ip));

    for (;;) {
        /* Find a match (lz4.c:909-957) */
        {
            int fwd = ip, step = 1, searchMatchNb = acceleration << 6;
            for (;;) {
                uint32_t h = forwardH;
                int current = fwd;
                int mi = table[h];
                ip = fwd;
                fwd += step;
                step = (searchMatchNb++ >> 6);
                if (fwd > mflimitPlusOne) goto last_literals;
                match = mi;
                forwardH = hash4_u16(rd32(src + fwd));
                table[h] = (uint16_t)current;
                if (rd32(src + match) == rd32(src + ip)) break;
            }
        }
        /* Catch up (lz4.c:958-959) */
        while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) { ip--; match--; }

        /* Encode literals (lz4.c:961-988) */
        {
            unsigned litLength = (unsigned)(ip - anchor);
            token = op++;
            if (op + (int)litLength + (2 + 1 + LASTLITERALS) + (int)(litLength / 255) > olimit)
                return 0;
            if (litLength >= RUN_MASK) {
                int len = (int)(litLength - RUN_MASK);
                dst[token] = (uint8_t)(RUN_MASK << ML_BITS);
                for (; len >= 255; len -= 255) dst[op++] = 255;
                dst[op++] = (uint8_t)len;
            } else {
                dst[token] = (uint8_t)(litLength << ML_BITS);
            }
            memcpy(dst + op, src + anchor, litLength);
            op += (int)litLength;
        }

    next_match:
        /* Encode offset (lz4.c:1011-1015) */
        dst[op] = (uint8_t)(ip - match);
        dst[op + 1] = (uint8_t)((ip - match) >> 8);
        op += 2;
        /* Encode match length (lz4.c:1018-1074) */
        {
            unsigned matchCode = (unsigned)lz4_count(src, ip + MINMATCH, match + MINMATCH, matchlimit);
            ip += (int)matchCode + MINMATCH;
            if (op + (1 + LASTLITERALS) + (int)((matchCode + 240) / 255) > olimit) return 0;
            if (matchCode >= ML_MASK) {
                dst[token] = (uint8_t)(dst[token] + ML_MASK);
                matchCode -= ML_MASK;
                for (; matchCode >= 255; matchCode -= 255) dst[op++] = 255;
                dst[op++] = (uint8_t)matchCode;
            } else {
                dst[token] = (uint8_t)(dst[token] + matchCode);
            }
        }
        anchor = ip;
        if (ip >= mflimitPlusOne) break;           /* lz4.c:1081 */
        table[hash4_u16(rd32(src + ip - 2))] = (uint16_t)(ip - 2);   /* lz4.c:1084 */
        /* Test next position (lz4.c:1096-1134) */
        {
            uint32_t h = hash4_u16(rd32(src + ip));
            int mi = table[h];
            table[h] = (uint16_t)ip;
            if (rd32(src + mi) == rd32(src + ip)) {
                token = op++;
                dst[token] = 0;
                match = mi;
                goto next_match;
            }
        }
        ip++;
        forwardH = hash4_u16(rd32(src + ip));
    }

last_literals:
    {   /* lz4.c:1141-1166 */
        int lastRun = n - anchor;
        if (op + lastRun + 1 + (lastRun + 255 - (int)RUN_MASK) / 255 > olimit) return 0;
        if (lastRun >= (int)RUN_MASK) {
            int acc = lastRun - (int)RUN_MASK;
            dst[op++] = (uint8_t)(RUN_MASK << ML_BITS);
            for (; acc >= 255; acc -= 255) dst[op++] = 255;
            dst[op++] = (uint8_t)acc;
        } else {
            dst[op++] = (uint8_t)(lastRun << ML_BITS);
        }
        memcpy(dst + op, src + anchor, (size_t)lastRun);
        op += lastRun;
    }
    return op;
}

/* ======================================================================= */
/* LZ4 block decompression: LZ4_decompress_generic (lz4.c:1654-2068) with   */
/* endOnInputSize + decode_full_block, including the LZ4_FAST_DEC_LOOP      */
/* (lz4.c:1707-1824) and the safe-loop shortcut (lz4.c:1846-1889), whose    */
/* bounds checks decide which malformed blocks the reference accepts.       */
/* History (`dict_size` bytes) must sit contiguously before dst.            */
/* ======================================================================= */

/* read_variable_length (lz4.c:1625-1645).  Returns -1 on initial_error,
 * -2 on loop_error (length still accumulated), else 0. */
static int rvl(const uint8_t *s, int *ip, int lencheck, int initial_check, unsigned *len) {
    unsigned length = 0, b;
    if (initial_check && *ip >= lencheck) { *len = 0; return -1; }
    do {
        b = s[*ip];
        (*ip)++;
        length += b;
        if (*ip >= lencheck) { *len = length; return -2; }
    } while (b == 255);
    *len = length;
    return 0;
}

static void lz77_copy(uint8_t *dst, int op, long offset, int length) {
    /* LZ77 overlap semantics; offset 0 yields zeros exactly like the
     * reference's LZ4_write32(op,0) + self-copy (lz4.c:2026, 1799). */
    if (offset == 0) { memset(dst + op, 0, (size_t)length); return; }
    for (int i = 0; i < length; i++) dst[op + i] = dst[op - offset + i];
}

int or_lz4_decompress_block(const uint8_t *src, int csize, uint8_t *dst,
                            int dst_cap, int dict_size) {
    /* dict_size = bytes of history contiguous in front of dst.  LZ4F reaches
     * LZ4_decompress_safe_usingDict (lz4.c:2307): 0 -> noDict; >= 64K-1 ->
     * withPrefix64k (lowPrefix = dst-64K); else withSmallPrefix (lowPrefix =
     * dst-dict_size).  All three pass dictSize 0, so checkOffset is on. */
    const int iend = csize, oend = dst_cap;
    const int prefix64k = dict_size >= 65536 - 1;
    const long lowPrefix = dict_size <= 0 ? 0 : (prefix64k ? -65536L : -(long)dict_size);
    int ip = 0, op = 0;
    unsigned token, length;
    long match, offset;
    int cpy;

    if (dst_cap == 0) return (csize == 1 && src[0] == 0) ? 0 : -1;
    if (csize == 0) return -1;

    if (oend - op < FASTLOOP_SAFE_DISTANCE) goto safe_decode;
    for (;;) {                                    /* fast loop, lz4.c:1712 */
        token = src[ip++];
        length = token >> ML_BITS;
        if (length == RUN_MASK) {
            unsigned add;
            if (rvl(src, &ip, iend - (int)RUN_MASK, 1, &add) == -1) return -1;
            length += add;
            cpy = op + (int)length;
            if (cpy > oend - 32 || ip + (int)length > iend - 32) goto safe_literal_copy;
            memcpy(dst + op, src + ip, length);
            ip += (int)length; op = cpy;
        } else {
            cpy = op + (int)length;
            if (ip > iend - (16 + 1)) goto safe_literal_copy;
            memcpy(dst + op, src + ip, length);
            ip += (int)length; op = cpy;
        }
        offset = (long)src[ip] | ((long)src[ip + 1] << 8);
        ip += 2;
        match = op - offset;
        length = token & ML_MASK;
        if (length == ML_MASK) {
            unsigned add;
            if (match < lowPrefix) return -1;
            if (rvl(src, &ip, iend - LASTLITERALS + 1, 0, &add) != 0) return -1;
            length += add + MINMATCH;
            if (op + (int)length >= oend - FASTLOOP_SAFE_DISTANCE) goto safe_match_copy;
        } else {
            length += MINMATCH;
            if (op + (int)length >= oend - FASTLOOP_SAFE_DISTANCE) goto safe_match_copy;
            if ((prefix64k || match >= lowPrefix) && offset >= 8) {
                lz77_copy(dst, op, offset, (int)length);
                op += (int)length;
                continue;
            }
        }
        if (match < lowPrefix) return -1;
        lz77_copy(dst, op, offset, (int)length);
        op += (int)length;
    }

safe_decode:
    for (;;) {                                    /* safe loop, lz4.c:1827 */
        token = src[ip++];
        length = token >> ML_BITS;
        /* two-stage shortcut (lz4.c:1846-1889) */
        if (length != RUN_MASK && ip < iend - 16 && op <= oend - 32) {
            memcpy(dst + op, src + ip, length);
            op += (int)length; ip += (int)length;
            length = token & ML_MASK;
            offset = (long)src[ip] | ((long)src[ip + 1] << 8);
            ip += 2;
            match = op - offset;
            if (length != ML_MASK && offset >= 8 && (prefix64k || match >= lowPrefix)) {
                lz77_copy(dst, op, offset, (int)length + MINMATCH);
                op += (int)length + MINMATCH;
                continue;
            }
            goto copy_match;
        }
        if (length == RUN_MASK) {
            unsigned add;
            if (rvl(src, &ip, iend - (int)RUN_MASK, 1, &add) == -1) return -1;
            length += add;
        }
        cpy = op + (int)length;
    safe_literal_copy:
        if (cpy > oend - MFLIMIT || ip + (int)length > iend - (2 + 1 + LASTLITERALS)) {
            if (ip + (int)length != iend || cpy > oend) return -1;
            memmove(dst + op, src + ip, length);
            ip += (int)length; op += (int)length;
            break;
        }
        memcpy(dst + op, src + ip, length);
        ip += (int)length; op = cpy;
        offset = (long)src[ip] | ((long)src[ip + 1] << 8);
        ip += 2;
        match = op - offset;
        length = token & ML_MASK;
    copy_match:
        if (length == ML_MASK) {
            unsigned add;
            if (rvl(src, &ip, iend - LASTLITERALS + 1, 0, &add) != 0) return -1;
            length += add;
        }
        length += MINMATCH;
    safe_match_copy:
        if (match < lowPrefix) return -1;
        cpy = op + (int)length;
        if (cpy > oend - MATCH_SAFEGUARD_DISTANCE && cpy > oend - LASTLITERALS) return -1;
        lz77_copy(dst, op, offset, (int)length);
        op = cpy;
    }
    return op;
}

/* ======================================================================= */
/* LZ4F framing as driven by rd_kafka_lz4_compress (rdkafka_lz4.c:329-442)  */
/* ======================================================================= */
#define LZ4F_MAGIC 0x184D2204u
#define LZ4F_MAGIC_SKIPPABLE_START 0x184D2A50u
#define LZ4F_BLOCK_UNCOMPRESSED 0x80000000u
#define BLOCK64K 65536

size_t or_lz4f_compress_bound(size_t len) {
    /* LZ4F_compressBound(len, NULL) (lz4frame.c:358-391: worst-case prefs,
     * 4 MB blocks, checksums) + 1000, as rdkafka_lz4.c:354 allocates. */
    size_t const blockSize = (size_t)4 << 20;
    size_t const maxBuffered = blockSize - 1;
    size_t const bufferedSize = len < maxBuffered ? len : maxBuffered;
    size_t const maxSrcSize = len + bufferedSize;
    unsigned const nbFullBlocks = (unsigned)(maxSrcSize / blockSize);
    size_t const partialBlockSize = maxSrcSize & (blockSize - 1);
    size_t const lastBlockSize = partialBlockSize;
    unsigned const nbBlocks = nbFullBlocks + (lastBlockSize > 0);
    size_t const blockCRCSize = 4;
    size_t const frameEnd = 4 + 4;
    size_t const compressBound = ((4 + blockCRCSize) * nbBlocks) +
                                 (blockSize * nbFullBlocks) + lastBlockSize + frameEnd;
    return 19 + compressBound + 1000;
}

void or_free(void *p) { free(p); }

static size_t frame_header(uint8_t *out) {
    /* LZ4F_compressBegin_usingCDict (lz4frame.c:671-701) with
     * {blockIndependent, no checksums, no content size, 64 KB}. */
    out[0] = 0x04; out[1] = 0x22; out[2] = 0x4D; out[3] = 0x18;
    out[4] = (uint8_t)((1u << 6) | (1u << 5));   /* FLG 0x60 */
    out[5] = (uint8_t)(4u << 4);                 /* BD  0x40 */
    out[6] = (uint8_t)(or_xxh32(out + 4, 2, 0) >> 8);
    return 7;
}

static size_t make_block(uint8_t *dst, const uint8_t *src, size_t n, int level) {
    /* LZ4F_makeBlock (lz4frame.c:739-761) with LZ4F_selectCompression
     * (lz4frame.c:797-805): levels >= 3 take LZ4F_compressBlockHC */
    int accel = level < 0 ? -level + 1 : 1;              /* lz4frame.c:766 */
    int c = level >= 3 ? or_lz4hc_compress_block(src, (int)n, dst + 4, (int)n - 1, level)
                       : or_lz4_compress_block(src, (int)n, dst + 4, (int)n - 1, accel);
    if (c == 0) {
        wr_le32(dst, (uint32_t)n | LZ4F_BLOCK_UNCOMPRESSED);
        memcpy(dst + 4, src, n);
        return 4 + n;
    }
    wr_le32(dst, (uint32_t)c);
    return 4 + (size_t)c;
}

/* rd_kafka_lz4_compress_break_framing (rdkafka_lz4.c:108-155). */
static int break_framing(uint8_t *out, size_t outlen) {
    static const uint8_t magic[4] = {0x04, 0x22, 0x4d, 0x18};
    size_t of = 4;
    if (outlen < 7 || memcmp(out, magic, 4)) return OR_ERR__BAD_COMPRESSION;
    uint8_t FLG = out[of++];
    of++;
    if ((FLG >> 3) & 1) of += 8;
    if (of >= outlen) return OR_ERR__BAD_COMPRESSION;
    out[of] = (uint8_t)((or_xxh32(out, of, 0) >> 8) & 0xff);
    return OR_ERR_NO_ERROR;
}

/* rd_kafka_lz4_decompress_fixup_bad_framing (rdkafka_lz4.c:50-98). */
static int fixup_framing(uint8_t *in, size_t inlen) {
    static const uint8_t magic[4] = {0x04, 0x22, 0x4d, 0x18};
    size_t of = 4;
    if (inlen < 7 || memcmp(in, magic, 4)) return OR_ERR__BAD_COMPRESSION;
    uint8_t FLG = in[of++];
    of++;
    if ((FLG >> 3) & 1) of += 8;
    if (of >= inlen) return OR_ERR__BAD_COMPRESSION;
    in[of] = (uint8_t)((or_xxh32(in + 4, of - 4, 0) >> 8) & 0xff);
    return OR_ERR_NO_ERROR;
}

int or_rdk_lz4_compress(int proper_hc, int comp_level, const uint8_t *src,
                        size_t len, uint8_t **out, size_t *outlen) {
    *out = NULL;
    size_t cap = or_lz4f_compress_bound(len);
    uint8_t *o = (uint8_t *)malloc(cap);
    if (!o) return OR_ERR__CRIT_SYS_RESOURCE;
    size_t of = frame_header(o);
    /* LZ4F_compressUpdate/End cut the (concatenated) input into full 64 KB
     * blocks plus one final partial block (lz4frame.c:883-893, 936-972). */
    for (size_t pos = 0; pos < len; pos += BLOCK64K) {
        size_t n = len - pos < BLOCK64K ? len - pos : BLOCK64K;
        of += make_block(o + of, src + pos, n, comp_level);
    }
    wr_le32(o + of, 0);                                  /* end mark */
    of += 4;
    if (!proper_hc) {
        int e = break_framing(o, of);
        if (e) { free(o); return e; }
    }
    *out = o;
    *outlen = of;
    return OR_ERR_NO_ERROR;
}

/* Frame decode with rd_kafka_lz4_decompress's outer-loop semantics:
 * the whole input is fed; a frame that runs out of input is a success with
 * the blocks completed so far (raw blocks: the bytes present); bytes after a
 * complete frame are __BAD_MSG; anything LZ4F rejects is __BAD_COMPRESSION. */
int or_rdk_lz4_decompress(int proper_hc, uint8_t *in, size_t inlen,
                          uint8_t **out, size_t *outlen) {
    size_t pos, hsize;
    uint8_t *o = NULL;
    size_t olen = 0, ocap = 0;
    int err = OR_ERR_NO_ERROR;
    *out = NULL;
    *outlen = 0;

    if (!proper_hc) {
        int e = fixup_framing(in, inlen);
        if (e) return e;
    }
    if (inlen < 5) return OR_ERR__BAD_COMPRESSION;            /* LZ4F_headerSize */
    uint32_t magic = rd_le32(in);
    if ((magic & 0xFFFFFFF0u) == LZ4F_MAGIC_SKIPPABLE_START) {
        if (inlen < 8) return OR_ERR__BAD_COMPRESSION;
        size_t sz = rd_le32(in + 4);
        pos = 8 + sz;
        o = (uint8_t *)malloc(1);
        if (pos < inlen) { free(o); return OR_ERR__BAD_MSG; }
        *out = o;
        return OR_ERR_NO_ERROR;
    }
    if (magic != LZ4F_MAGIC) return OR_ERR__BAD_COMPRESSION;
    uint8_t FLG = in[4];
    unsigned blockChecksum = (FLG >> 4) & 1, blockMode = (FLG >> 5) & 1,
             contentSizeFlag = (FLG >> 3) & 1, contentChecksum = (FLG >> 2) & 1,
             dictIDFlag = FLG & 1;
    hsize = 7 + (contentSizeFlag ? 8 : 0) + (dictIDFlag ? 4 : 0);
    if (inlen < hsize) return OR_ERR__BAD_COMPRESSION;
    if ((FLG >> 1) & 1) return OR_ERR__BAD_COMPRESSION;       /* reserved */
    if (((FLG >> 6) & 3) != 1) return OR_ERR__BAD_COMPRESSION; /* version */
    uint8_t BD = in[5];
    unsigned bsid = (BD >> 4) & 7;
    if ((BD >> 7) & 1) return OR_ERR__BAD_COMPRESSION;
    if (bsid < 4) return OR_ERR__BAD_COMPRESSION;
    if (BD & 0x0F) return OR_ERR__BAD_COMPRESSION;
    if ((uint8_t)(or_xxh32(in + 4, hsize - 5, 0) >> 8) != in[hsize - 1])
        return OR_ERR__BAD_COMPRESSION;
    size_t maxBlock = (size_t)64 << (2 * (bsid - 4));
    uint64_t contentSize = 0;
    if (contentSizeFlag) {
        contentSize = (uint64_t)rd_le32(in + 6) | ((uint64_t)rd_le32(in + 10) << 32);
    }
    maxBlock *= 1024;
    uint64_t remaining = contentSize;
    int done = 0;

    /* output: grow as needed (zbuf_grow semantics do not change the bytes) */
    ocap = maxBlock;
    o = (uint8_t *)malloc(ocap + 1);
    if (!o) return OR_ERR__CRIT_SYS_RESOURCE;
    pos = hsize;
    while (pos < inlen) {
        if (inlen - pos < 4) { pos = inlen; break; }        /* truncated header */
        uint32_t bh = rd_le32(in + pos);
        size_t bsz = bh & 0x7FFFFFFFu;
        pos += 4;
        if (bsz == 0) {                                      /* end mark */
            if (remaining) { err = OR_ERR__BAD_COMPRESSION; goto out; }
            if (contentChecksum) {
                if (inlen - pos < 4) { pos = inlen; break; }
                if (rd_le32(in + pos) != or_xxh32(o, olen, 0)) { err = OR_ERR__BAD_COMPRESSION; goto out; }
                pos += 4;
            }
            done = 1;
            break;
        }
        if (bsz > maxBlock) { err = OR_ERR__BAD_COMPRESSION; goto out; }
        if (olen + maxBlock > ocap) {
            size_t ncap = ocap * 2 > olen + maxBlock ? ocap * 2 : olen + maxBlock;
            uint8_t *t = (uint8_t *)realloc(o, ncap + 1);
            if (!t) { err = OR_ERR__CRIT_SYS_RESOURCE; goto out; }
            o = t; ocap = ncap;
        }
        if (bh & LZ4F_BLOCK_UNCOMPRESSED) {
            size_t avail = inlen - pos, ncopy = bsz < avail ? bsz : avail;
            memcpy(o + olen, in + pos, ncopy);
            olen += ncopy;
            if (contentSize) remaining -= ncopy;
            pos += ncopy;
            if (ncopy < bsz) break;                          /* truncated */
            if (blockChecksum) {
                if (inlen - pos < 4) { pos = inlen; break; }
                if (rd_le32(in + pos) != or_xxh32(in + pos - bsz, bsz, 0)) { err = OR_ERR__BAD_COMPRESSION; goto out; }
                pos += 4;
            }
            continue;
        }
        size_t need = bsz + (blockChecksum ? 4 : 0);
        if (inlen - pos < need) { pos = inlen; break; }      /* truncated block */
        if (blockChecksum && rd_le32(in + pos + bsz) != or_xxh32(in + pos, bsz, 0)) {
            err = OR_ERR__BAD_COMPRESSION; goto out;
        }
        {
            size_t hist = blockMode == 0 ? olen : 0;         /* linked: prior output */
            if (hist > 65536) hist = 65536;
            int d = or_lz4_decompress_block(in + pos, (int)bsz, o + olen, (int)maxBlock, (int)hist);
            if (d < 0) { err = OR_ERR__BAD_COMPRESSION; goto out; }
            olen += (size_t)d;
            if (contentSize) remaining -= (uint64_t)d;
        }
        pos += need;
    }
    if (done && pos < inlen) { err = OR_ERR__BAD_MSG; goto out; }
out:
    if (err) { free(o); return err; }
    *out = o;
    *outlen = olen;
    return OR_ERR_NO_ERROR;
}

/* ---- threaded drivers (CPU baseline legs) ------------------------------- */
struct fjob {
    const uint8_t *base; const uint64_t *offs; const uint32_t *lens; size_t lo, hi;
    uint8_t *out; const uint64_t *out_offs; const uint32_t *out_caps; uint32_t *out_lens;
    int decompress; int rc; int level;
};

static void *fworker(void *arg) {
    struct fjob *j = (struct fjob *)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        uint8_t *r = NULL; size_t rl = 0; int e;
        if (j->decompress) {
            /* the reference may patch the header in place only when !proper_hc */
            e = or_rdk_lz4_decompress(1, (uint8_t *)(j->base + j->offs[i]), j->lens[i], &r, &rl);
            if (!e && rl <= j->out_caps[i]) memcpy(j->out + j->out_offs[i], r, rl);
            else if (!e) e = -1;
        } else {
            e = or_rdk_lz4_compress(1, j->level, j->base + j->offs[i], j->lens[i], &r, &rl);
            if (!e) memcpy(j->out + j->out_offs[i], r, rl);
        }
        free(r);
        if (e) { j->rc = e; continue; }
        j->out_lens[i] = (uint32_t)rl;
    }
    return NULL;
}

static int run_frames(const uint8_t *base, const uint64_t *offs, const uint32_t *lens,
                      size_t n, uint8_t *out, const uint64_t *out_offs,
                      const uint32_t *caps, uint32_t *out_lens, int threads, int dec,
                      int level) {
    if (threads < 1) threads = 1;
    if (threads > 512) threads = 512;
    pthread_t th[512];
    struct fjob jobs[512];
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (struct fjob){base, offs, lens, n * t / threads, n * (t + 1) / threads,
                                out, out_offs, caps, out_lens, dec, 0, level};
        pthread_create(&th[t], NULL, fworker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); if (jobs[t].rc) rc = jobs[t].rc; }
    return rc;
}

int or_lz4f_compress_batches_mt(const uint8_t *base, const uint64_t *offs,
                                const uint32_t *lens, size_t n, uint8_t *out,
                                const uint64_t *out_offs, uint32_t *out_lens, int threads) {
    return run_frames(base, offs, lens, n, out, out_offs, NULL, out_lens, threads, 0, 0);
}

int or_lz4f_compress_batches_level_mt(const uint8_t *base, const uint64_t *offs,
                                      const uint32_t *lens, size_t n, uint8_t *out,
                                      const uint64_t *out_offs, uint32_t *out_lens,
                                      int level, int threads) {
    return run_frames(base, offs, lens, n, out, out_offs, NULL, out_lens, threads, 0, level);
}

int or_lz4f_decompress_batches_mt(const uint8_t *base, const uint64_t *offs,
                                  const uint32_t *lens, size_t n, uint8_t *out,
                                  const uint64_t *out_offs, const uint32_t *out_caps,
                                  uint32_t *out_lens, int threads) {
    return run_frames(base, offs, lens, n, out, out_offs, out_caps, out_lens, threads, 1, 0);
}
