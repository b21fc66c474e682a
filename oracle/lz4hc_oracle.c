/*
 * lz4hc_oracle.c -- CPU restatement of the LZ4HC compressors that librdkafka
 * v1.3.0 reaches for `compression.level` 3..12 (vendored lz4 1.9.2): the
 * hash-chain parser (3..9) and the optimal parser (10..12).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Path: rd_kafka_lz4_compress (rdkafka_lz4.c:329) -> LZ4F_compressUpdate ->
 * LZ4F_makeBlock (lz4frame.c:739, dstCapacity = srcSize-1) ->
 * LZ4F_compressBlockHC (lz4frame.c:782) -> LZ4_compress_HC_extStateHC_fastReset
 * (lz4hc.c:896, limitedOutput) -> LZ4HC_compress_generic_internal (lz4hc.c:758)
 * -> LZ4HC_compress_hashChain (lz4hc.c:532-746) with nbSearches from clTable
 * (lz4hc.c:775-789), or LZ4HC_compress_optimal (lz4hc.c:1278-1538) for the
 * lz4opt rows of that table (10: 96 searches, sufficient length 64; 11: 512,
 * 128; 12: 16384, LZ4_OPT_NUM, full update), favorCompressionRatio.
 *
 * Positions are block-relative.  Every LZ4F block starts a fresh window: the
 * reference shifts `base` by 64 KB per block (LZ4HC_init_internal,
 * lz4hc.c:99-113), so stale hash entries fall below lowLimit and clamp to a
 * chain delta of 65535 exactly as an empty table would.  "No entry" is
 * therefore -65536 here and no table survives between blocks.  With
 * dictLimit == lowLimit == block start the extDict / dictCtx branches of
 * LZ4HC_InsertAndGetWiderMatch (lz4hc.c:294-310, :412-439) are unreachable.
 * chainSwap is 0 on the hash-chain path (lz4hc.c:456, :580, :625) and 1, with
 * pattern analysis, under the optimal parser (LZ4HC_FindLongerMatch, :1267).
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
#define HC_OPT_NUM (1 << 12)          /* LZ4_OPT_NUM, lz4hc.c:75 */
#define HC_TRAILING 3                 /* TRAILING_LITERALS, lz4hc.c:1290 */

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

/* LZ4HC_InsertAndGetWiderMatch (lz4hc.c:234-442), prefix-only,
 * favorCompressionRatio.  Returns the new longest; *mpos / *spos are updated
 * only on improvement. */
static int hc_wider(hc_state *st, int ip, int ilow, int ihigh, int longest,
                    int *mpos, int *spos, int attempts, int pa, int swap) {
    const uint8_t *s = st->s;
    const int back_room = ip - ilow;
    const uint32_t pat = ld32(s + ip);
    int repeat = 0;                   /* 0 untested, 1 not, 2 confirmed */
    int src_pat_len = 0;
    int chain_pos = 0;                /* matchChainPos */
    hc_insert(st, ip);
    int m = st->head[hc_hash(pat)];
    while (m >= 0 && attempts) {
        int len = 0;
        attempts--;
        if (ld16(s + ilow + longest - 1) == ld16(s + m - back_room + longest - 1) &&
            ld32(s + m) == pat) {
            int back = 0;
            if (back_room) {          /* LZ4HC_countBack (lz4hc.c:140-152) */
                int lim = (ilow - ip) > (0 - m) ? (ilow - ip) : (0 - m);
                while (back > lim && s[ip + back - 1] == s[m + back - 1]) back--;
            }
            len = HC_MINMATCH + hc_count(s, ip + HC_MINMATCH, m + HC_MINMATCH, ihigh) - back;
            if (len > longest) { longest = len; *mpos = m + back; *spos = ip + back; }
        }
        if (swap && len == longest && m + longest <= ip) {
            /* chain swap (lz4hc.c:312-334): follow the chain of the position inside
             * the match whose previous occurrence lies furthest back */
            int dist = 1, step = 1, accel = 1 << 4;
            const int end = longest - HC_MINMATCH + 1;
            for (int pos = 0; pos < end; pos += step) {
                int cd = st->delta[(m + pos) & 0xffff];
                step = accel++ >> 4;
                if (cd > dist) { dist = cd; chain_pos = pos; accel = 1 << 4; }
            }
            if (dist > 1) {
                /* `distanceToNextMatch > matchIndex` (lz4hc.c:331) compares with an
                 * index that starts at 64 KB: never true for a 16-bit delta */
                m -= dist;
                continue;
            }
        }
        int dnext = st->delta[m & 0xffff];
        if (pa && dnext == 1 && chain_pos == 0) {   /* pattern analysis (lz4hc.c:336-405) */
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
        m -= st->delta[(m + chain_pos) & 0xffff];
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

int or_lz4hc_attempts(int level) {   /* clTable, lz4hc.c:775-789 */
    if (level < 1) level = 9;
    if (level < 3) return 2;
    if (level >= 12) return 16384;
    if (level == 11) return 512;
    if (level == 10) return 96;
    return 1 << (level - 1);          /* 3 -> 4 ... 9 -> 256 */
}

/* LZ4HC_literalsPrice / LZ4HC_sequencePrice (lz4hc.c:1224-1247), in bytes */
static int hc_lit_price(int litlen) {
    int price = litlen;
    if (litlen >= 15) price += 1 + (litlen - 15) / 255;
    return price;
}
static int hc_seq_price(int litlen, int mlen) {
    int price = 1 + 2 + hc_lit_price(litlen);
    if (mlen >= 15 + HC_MINMATCH) price += 1 + (mlen - (15 + HC_MINMATCH)) / 255;
    return price;
}

typedef struct { int price, off, mlen, litlen; } hc_opt;   /* LZ4HC_optimal_t */

/* LZ4HC_FindLongerMatch (lz4hc.c:1255-1275): forward only, pattern analysis and
 * chain swap on.  Returns the length (0: none longer than min_len), *off set. */
static int hc_longer(hc_state *st, int ip, int ihigh, int min_len, int attempts, int *off) {
    int mpos = 0, spos = ip;
    int len = hc_wider(st, ip, ip, ihigh, min_len, &mpos, &spos, attempts, 1, 1);
    if (len <= min_len) return 0;
    *off = ip - mpos;
    return len;
}

/* LZ4HC_compress_optimal (lz4hc.c:1278-1538), limitedOutput */
static int hc_optimal(hc_state *st, const uint8_t *src, int n, uint8_t *dst, int dst_cap,
                      int attempts, int sufficient, int full) {
    hc_opt *opt = (hc_opt *)malloc(sizeof(hc_opt) * (HC_OPT_NUM + HC_TRAILING));
    if (!opt) return -1;
    const int mflimit = n - HC_MFLIMIT, matchlimit = n - HC_LASTLITERALS;
    int ip = 0, anchor = 0, op = 0;
    if (sufficient >= HC_OPT_NUM) sufficient = HC_OPT_NUM - 1;
    while (ip <= mflimit) {
        const int llen = ip - anchor;
        int best_mlen, best_off, cur, last_pos = 0, foff = 0;
        const int flen = hc_longer(st, ip, matchlimit, HC_MINMATCH - 1, attempts, &foff);
        if (flen == 0) { ip++; continue; }
        if (flen > sufficient) {       /* good enough: immediate encoding (:1318-1326) */
            if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, flen, ip - foff)) goto overflow;
            continue;
        }
        for (int r = 0; r < HC_MINMATCH; r++) {            /* :1329-1338 */
            opt[r].mlen = 1; opt[r].off = 0; opt[r].litlen = llen + r;
            opt[r].price = hc_lit_price(llen + r);
        }
        for (int ml = HC_MINMATCH; ml <= flen; ml++) {     /* :1340-1352 */
            opt[ml].mlen = ml; opt[ml].off = foff; opt[ml].litlen = llen;
            opt[ml].price = hc_seq_price(llen, ml);
        }
        last_pos = flen;
        for (int a = 1; a <= HC_TRAILING; a++) {           /* :1354-1362 */
            opt[last_pos + a].mlen = 1; opt[last_pos + a].off = 0; opt[last_pos + a].litlen = a;
            opt[last_pos + a].price = opt[last_pos].price + hc_lit_price(a);
        }
        for (cur = 1; cur < last_pos; cur++) {             /* :1365-1459 */
            const int cp = ip + cur;
            int noff = 0, nlen;
            if (cp > mflimit) break;
            if (full) {
                if (opt[cur + 1].price <= opt[cur].price &&
                    opt[cur + HC_MINMATCH].price < opt[cur].price + 3) continue;
            } else {
                if (opt[cur + 1].price <= opt[cur].price) continue;
            }
            if (full) nlen = hc_longer(st, cp, matchlimit, HC_MINMATCH - 1, attempts, &noff);
            else nlen = hc_longer(st, cp, matchlimit, last_pos - cur, attempts, &noff);
            if (!nlen) continue;
            if (nlen > sufficient || nlen + cur >= HC_OPT_NUM) {   /* :1391-1398 */
                best_mlen = nlen; best_off = noff; last_pos = cur + 1;
                goto encode;
            }
            {   const int base_ll = opt[cur].litlen;               /* :1401-1413 */
                for (int ll = 1; ll < HC_MINMATCH; ll++) {
                    const int price = opt[cur].price - hc_lit_price(base_ll) + hc_lit_price(base_ll + ll);
                    const int pos = cur + ll;
                    if (price < opt[pos].price) {
                        opt[pos].mlen = 1; opt[pos].off = 0; opt[pos].litlen = base_ll + ll;
                        opt[pos].price = price;
                    }
                }
            }
            for (int ml = HC_MINMATCH; ml <= nlen; ml++) {         /* :1416-1449 */
                const int pos = cur + ml;
                int price, ll;
                if (opt[cur].mlen == 1) {
                    ll = opt[cur].litlen;
                    price = (cur > ll ? opt[cur - ll].price : 0) + hc_seq_price(ll, ml);
                } else {
                    ll = 0;
                    price = opt[cur].price + hc_seq_price(0, ml);
                }
                if (pos > last_pos + HC_TRAILING || price <= opt[pos].price) {
                    if (ml == nlen && last_pos < pos) last_pos = pos;
                    opt[pos].mlen = ml; opt[pos].off = noff; opt[pos].litlen = ll;
                    opt[pos].price = price;
                }
            }
            for (int a = 1; a <= HC_TRAILING; a++) {               /* :1451-1458 */
                opt[last_pos + a].mlen = 1; opt[last_pos + a].off = 0; opt[last_pos + a].litlen = a;
                opt[last_pos + a].price = opt[last_pos].price + hc_lit_price(a);
            }
        }
        best_mlen = opt[last_pos].mlen;
        best_off = opt[last_pos].off;
        cur = last_pos - best_mlen;
    encode:                                                        /* :1466-1498 */
        {   int cand = cur, sel_ml = best_mlen, sel_off = best_off;
            for (;;) {                 /* reverse traversal */
                const int next_ml = opt[cand].mlen, next_off = opt[cand].off;
                opt[cand].mlen = sel_ml; opt[cand].off = sel_off;
                sel_ml = next_ml; sel_off = next_off;
                if (next_ml > cand) break;
                cand -= next_ml;
            }
        }
        {   int r = 0;
            while (r < last_pos) {
                const int ml = opt[r].mlen, off = opt[r].off;
                if (ml == 1) { ip++; r++; continue; }
                r += ml;
                if (hc_encode(src, dst, &op, dst_cap, &ip, &anchor, ml, ip - off)) goto overflow;
            }
        }
    }
    {   const int run = n - anchor;   /* :1501-1526 */
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
    free(opt);
    return op;
overflow:
    free(opt);
    return 0;
}

int or_lz4hc_compress_block(const uint8_t *src, int n, uint8_t *dst, int dst_cap, int level) {
    if (level > 12) level = 12;       /* MIN(LZ4HC_CLEVEL_MAX, cLevel), lz4hc.c:798 */
    const int attempts = or_lz4hc_attempts(level);
    const int pa = attempts > 128;    /* lz4hc.c:544 */
    hc_state *st = (hc_state *)malloc(sizeof *st);
    if (!st) return -1;
    for (int i = 0; i < (1 << HC_HASHLOG); i++) st->head[i] = HC_NONE;
    st->s = src;
    st->next = 0;
    if (level >= 10) {
        const int r = hc_optimal(st, src, n, dst, dst_cap, attempts,
                                 level == 10 ? 64 : level == 11 ? 128 : HC_OPT_NUM, level == 12);
        free(st);
        return r;
    }

    const int mflimit = n - HC_MFLIMIT, matchlimit = n - HC_LASTLITERALS;
    int ip = 0, anchor = 0, op = 0, unused = 0;
    int ml, ml0, ml2, ml3, start0, ref0, ref = 0, start2 = 0, ref2 = 0, start3 = 0, ref3 = 0;

    if (n < HC_MFLIMIT + 1) goto last;
    while (ip <= mflimit) {
        /* LZ4HC_InsertAndFindBestMatch (lz4hc.c:445-457) */
        ml = hc_wider(st, ip, ip, matchlimit, HC_MINMATCH - 1, &ref, &unused, attempts, pa, 0);
        if (ml < HC_MINMATCH) { ip++; continue; }
        start0 = ip; ref0 = ref; ml0 = ml;
    search2:
        if (ip + ml <= mflimit)
            ml2 = hc_wider(st, ip + ml - 2, ip, matchlimit, ml, &ref2, &start2, attempts, pa, 0);
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
            ml3 = hc_wider(st, start2 + ml2 - 3, start2, matchlimit, ml2, &ref3, &start3, attempts, pa, 0);
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
