/*
 * lz4hc_oracle.c -- CPU restatement of the LZ4HC hash-chain compressor that
 * librdkafka v1.3.0 reaches for `compression.level` 3..9 (vendored lz4 1.9.2).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Path: rd_kafka_lz4_compress (rdkafka_lz4.c:329) -> LZ4F_compressUpdate ->
 * LZ4F_makeBlock (lz4frame.c:739, dstCapacity = srcSize-1) ->
 * LZ4F_compressBlockHC (lz4frame.c:782) -> LZ4_compress_HC_extStateHC_fastReset
 * (lz4hc.c:896, limitedOutput) -> LZ4HC_compress_generic_internal (lz4hc.c:758)
 * -> LZ4HC_compress_hashChain (lz4hc.c:532-746) with nbSearches from clTable
 * (lz4hc.c:775-789).  Levels 10..12 (LZ4HC_compress_optimal) are not restated.
 *
 * Positions are block-relative.  Every LZ4F block starts a fresh window: the
 * reference shifts `base` by 64 KB per block (LZ4HC_init_internal,
 * lz4hc.c:99-113), so stale hash entries fall below lowLimit and clamp to a
 * chain delta of 65535 exactly as an empty table would.  "No entry" is
 * therefore -65536 here and no table survives between blocks.  With
 * dictLimit == lowLimit == block start the extDict / dictCtx branches of
 * LZ4HC_InsertAndGetWiderMatch (lz4hc.c:294-310, :412-439) are unreachable,
 * and chainSwap is 0 on the hash-chain path (lz4hc.c:456, :580, :625).
 *
 * Pinned byte-for-byte against the reference's lz4hc.c compiled by
 * oracle/Makefile into oracle/_ref/ (tests/test_oracle_hc.py) and against the
 * frames in tests/golden/lz4hc_frames.json.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define HC_MINMATCH 4
#define HC_LASTLITERALS 5
#define HC_MFLIMIT 12
#define HC_HASHLOG 15                 /* lz4hc.h:196 */
#define HC_NONE (-65536)              /* an index below every window */
#define HC_MAXDIST 65535              /* LZ4_DISTANCE_MAX */
#define HC_OPTIMAL_ML 18              /* (ML_MASK-1)+MINMATCH, lz4hc.c:74 */

typedef struct {
    const uint8_t *s;                 /* block start (== lowPrefixPtr) */
    int32_t head[1 << HC_HASHLOG];    /* hashTable                     */
    uint16_t delta[65536];            /* chainTable (DELTANEXTU16)     */
    int next;                         /* nextToUpdate                  */
} hc_state;

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t hc_hash(uint32_t v) { return (v * 2654435761u) >> (32 - HC_HASHLOG); }

/* LZ4HC_Insert (lz4hc.c:117-135) */
static void hc_insert(hc_state *st, int upto) {
    for (int p = st->next; p < upto; p++) {
        uint32_t h = hc_hash(ld32(st->s + p));
        int d = p - st->head[h];
        st->delta[p & 0xffff] = (uint16_t)(d > HC_MAXDIST ? HC_MAXDIST : d);
        st->head[h] = p;
    }
    if (upto > st->next) st->next = upto;
}

/* LZ4_count: equal bytes from a / b, a never past lim */
static int hc_count(const uint8_t *s, int a, int b, int lim) {
    int a0 = a;
    while (a < lim && s[a] == s[b]) { a++; b++; }
    return a - a0;
}

/* LZ4HC_countPattern (lz4hc.c:171-199), 64-bit reg_t, little endian */
static int hc_count_pattern(const uint8_t *s, int p, int end, uint32_t pat32) {
    uint64_t pat = (uint64_t)pat32 | ((uint64_t)pat32 << 32);
    int p0 = p;
    while (p < end - 7) {
        uint64_t v;
        memcpy(&v, s + p, 8);
        uint64_t x = v ^ pat;
        if (!x) { p += 8; continue; }
        return p + (__builtin_ctzll(x) >> 3) - p0;
    }
    uint64_t b = pat;
    while (p < end && s[p] == (uint8_t)b) { p++; b >>= 8; }
    return p - p0;
}

/* LZ4HC_reverseCountPattern (lz4hc.c:204-219) */
static int hc_rcount_pattern(const uint8_t *s, int p, int low, uint32_t pat) {
    int p0 = p;
    while (p >= low + 4 && ld32(s + p - 4) == pat) p -= 4;
    int k = 3;
    while (k >= 0 && p > low && s[p - 1] == (uint8_t)(pat >> (8 * k))) { p--; k--; }
    return p0 - p;
}

/* LZ4HC_InsertAndGetWiderMatch (lz4hc.c:234-442), prefix-only, chainSwap 0,
 * favorCompressionRatio.  Returns the new longest; *mpos / *spos are updated
 * only on improvement. */
static int hc_wider(hc_state *st, int ip, int ilow, int ihigh, int longest,
                    int *mpos, int *spos, int attempts, int pa) {
    const uint8_t *s = st->s;
    const int back_room = ip - ilow;
    const uint32_t pat = ld32(s + ip);
    int repeat = 0;                   /* 0 untested, 1 not, 2 confirmed */
    int src_pat_len = 0;
    hc_insert(st, ip);
    int m = st->head[hc_hash(pat)];
    while (m >= 0 && attempts) {
        attempts--;
        if (ld16(s + ilow + longest - 1) == ld16(s + m - back_room + longest - 1) &&
            ld32(s + m) == pat) {
            int back = 0;
            if (back_room) {          /* LZ4HC_countBack (lz4hc.c:140-152) */
                int lim = (ilow - ip) > (0 - m) ? (ilow - ip) : (0 - m);
                while (back > lim && s[ip + back - 1] == s[m + back - 1]) back--;
            }
            int len = HC_MINMATCH + hc_count(s, ip + HC_MINMATCH, m + HC_MINMATCH, ihigh) - back;
            if (len > longest) { longest = len; *mpos = m + back; *spos = ip + back; }
        }
        int dnext = st->delta[m & 0xffff];
        if (pa && dnext == 1) {       /* pattern analysis (lz4hc.c:336-405) */
            int cand = m - 1;
            if (repeat == 0) {
                if (((pat & 0xFFFF) == (pat >> 16)) & ((pat & 0xFF) == (pat >> 24))) {
                    repeat = 2;
                    src_pat_len = hc_count_pattern(s, ip + 4, ihigh, pat) + 4;
                } else {
                    repeat = 1;
                }
            }
            if (repeat == 2 && cand >= 0 && ld32(s + cand) == pat) {
                int fwd = hc_count_pattern(s, cand + 4, ihigh, pat) + 4;
                int bwd = hc_rcount_pattern(s, cand, 0, pat);
                if (bwd > cand) bwd = cand;           /* not below lowestMatchIndex */
                int seg = bwd + fwd;
                if (seg >= src_pat_len && fwd <= src_pat_len) {
                    m = cand + fwd - src_pat_len;
                } else {
                    m = cand - bwd;
                    if (back_room == 0) {
                        int maxml = seg < src_pat_len ? seg : src_pat_len;
                        if (longest < maxml) {
                            if (ip - m > HC_MAXDIST) break;
                            longest = maxml; *mpos = m; *spos = ip;
                        }
                        m -= st->delta[m & 0xffff];
                    }
                }
                continue;
            }
        }
        m -= dnext;
    }
    return longest;
}

/* LZ4HC_encodeSequence (lz4hc.c:462-530), limitedOutput.  0 ok, 1 overflow. */
static int hc_encode(const uint8_t *s, uint8_t *d, int *op, int oend, int *ip, int *anchor,
                     int ml, int ref) {
    int o = *op;
    const int tok = o++;
    const int lit = *ip - *anchor;
    if (o + lit / 255 + lit + (2 + 1 + HC_LASTLITERALS) > oend) return 1;
    if (lit >= 15) {
        int l = lit - 15;
        d[tok] = 15 << 4;
        for (; l >= 255; l -= 255) d[o++] = 255;
        d[o++] = (uint8_t)l;
    } else {
        d[tok] = (uint8_t)(lit << 4);
    }
    memcpy(d + o, s + *anchor, (size_t)lit);
    o += lit;
    const int off = *ip - ref;
    d[o] = (uint8_t)off;
    d[o + 1] = (uint8_t)(off >> 8);
    o += 2;
    int l = ml - HC_MINMATCH;
    if (o + l / 255 + (1 + HC_LASTLITERALS) > oend) return 1;
    if (l >= 15) {
        d[tok] += 15;
        l -= 15;
        for (; l >= 510; l -= 510) { d[o++] = 255; d[o++] = 255; }
        if (l >= 255) { l -= 255; d[o++] = 255; }
        d[o++] = (uint8_t)l;
    } else {
        d[tok] += (uint8_t)l;
    }
    *ip += ml;
    *anchor = *ip;
    *op = o;
    return 0;
}

int or_lz4hc_attempts(int level) {   /* clTable, lz4hc.c:775-789 (hash-chain rows) */
    if (level < 1) level = 9;
    if (level < 3) return 2;
    return 1 << (level - 1);          /* 3 -> 4 ... 9 -> 256 */
}

int or_lz4hc_compress_block(const uint8_t *src, int n, uint8_t *dst, int dst_cap, int level) {
    if (level >= 10) return -1;       /* LZ4HC_compress_optimal: not restated */
    const int attempts = or_lz4hc_attempts(level);
    const int pa = attempts > 128;    /* lz4hc.c:544 */
    hc_state *st = (hc_state *)malloc(sizeof *st);
    if (!st) return -1;
    for (int i = 0; i < (1 << HC_HASHLOG); i++) st->head[i] = HC_NONE;
    st->s = src;
    st->next = 0;

    const int mflimit = n - HC_MFLIMIT, matchlimit = n - HC_LASTLITERALS;
    int ip = 0, anchor = 0, op = 0, unused = 0;
    int ml, ml0, ml2, ml3, start0, ref0, ref = 0, start2 = 0, ref2 = 0, start3 = 0, ref3 = 0;

    if (n < HC_MFLIMIT + 1) goto last;
    while (ip <= mflimit) {
        /* LZ4HC_InsertAndFindBestMatch (lz4hc.c:445-457) */
        ml = hc_wider(st, ip, ip, matchlimit, HC_MINMATCH - 1, &ref, &unused, attempts, pa);
        if (ml < HC_MINMATCH) { ip++; continue; }
        start0 = ip; ref0 = ref; ml0 = ml;
    search2:
        if (ip + ml <= mflimit)
            ml2 = hc_wider(st, ip + ml - 2, ip, matchlimit, ml, &ref2, &start2, attempts, pa);
        else
            ml2 = ml;
        if (ml2 == ml) {
            if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, ml, ref)) goto overflow;
            continue;
        }
        if (start0 < ip && start2 < ip + ml0) { ip = start0; ref = ref0; ml = ml0; }
        if (start2 - ip < 3) { ml = ml2; ip = start2; ref = ref2; goto search2; }
    search3:
        if (start2 - ip < HC_OPTIMAL_ML) {
            int nml = ml > HC_OPTIMAL_ML ? HC_OPTIMAL_ML : ml;
            if (ip + nml > start2 + ml2 - HC_MINMATCH) nml = start2 - ip + ml2 - HC_MINMATCH;
            int corr = nml - (start2 - ip);
            if (corr > 0) { start2 += corr; ref2 += corr; ml2 -= corr; }
        }
        if (start2 + ml2 <= mflimit)
            ml3 = hc_wider(st, start2 + ml2 - 3, start2, matchlimit, ml2, &ref3, &start3, attempts, pa);
        else
            ml3 = ml2;
        if (ml3 == ml2) {
            if (start2 < ip + ml) ml = start2 - ip;
            if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, ml, ref)) goto overflow;
            ip = start2;
            if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, ml2, ref2)) goto overflow;
            continue;
        }
        if (start3 < ip + ml + 3) {
            if (start3 >= ip + ml) {
                if (start2 < ip + ml) {
                    int corr = ip + ml - start2;
                    start2 += corr; ref2 += corr; ml2 -= corr;
                    if (ml2 < HC_MINMATCH) { start2 = start3; ref2 = ref3; ml2 = ml3; }
                }
                if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, ml, ref)) goto overflow;
                ip = start3; ref = ref3; ml = ml3;
                start0 = start2; ref0 = ref2; ml0 = ml2;
                goto search2;
            }
            start2 = start3; ref2 = ref3; ml2 = ml3;
            goto search3;
        }
        if (start2 < ip + ml) {
            if (start2 - ip < HC_OPTIMAL_ML) {
                if (ml > HC_OPTIMAL_ML) ml = HC_OPTIMAL_ML;
                if (ip + ml > start2 + ml2 - HC_MINMATCH) ml = start2 - ip + ml2 - HC_MINMATCH;
                int corr = ml - (start2 - ip);
                if (corr > 0) { start2 += corr; ref2 += corr; ml2 -= corr; }
            } else {
                ml = start2 - ip;
            }
        }
        if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, ml, ref)) goto overflow;
        ip = start2; ref = ref2; ml = ml2;
        start2 = start3; ref2 = ref3; ml2 = ml3;
        goto search3;
    }
last: {
        const int run = n - anchor;   /* lz4hc.c:709-734 */
        const int ext = (run + 255 - 15) / 255;
        if (op + 1 + ext + run > dst_cap) goto overflow;
        if (run >= 15) {
            int a = run - 15;
            dst[op++] = 15 << 4;
            for (; a >= 255; a -= 255) dst[op++] = 255;
            dst[op++] = (uint8_t)a;
        } else {
            dst[op++] = (uint8_t)(run << 4);
        }
        memcpy(dst + op, src + anchor, (size_t)run);
        op += run;
    }
    free(st);
    return op;
overflow:
    free(st);
    return 0;
}
