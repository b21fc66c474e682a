/*
 * crc32c_oracle.c -- CPU restatement of src/crc32c.c (librdkafka v1.3.0).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restated, not copied: same polynomial, same table semantics, same chaining
 * contract (`crc` argument is the previous result, pre/post inversion applied
 * inside).  The reference file cannot be compiled here (rd.h:64 includes the
 * generated ../config.h), so this restatement is pinned by the reference's KAT
 * (crc32c.c:388-438) and by or_crc32c_bitwise().
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

#define CRC32C_POLY_REFLECTED 0x82f63b78u /* crc32c.c:63 */

/* tbl[k][b] = raw CRC (zero init, no inversion) of byte b followed by k zero
 * bytes; tbl[0] is the classic byte-wise table (crc32c.c:69-80), tbl[1..7]
 * the slicing-by-8 extension (crc32c.c:81-91). */
static uint32_t tbl[8][256];
static pthread_once_t tbl_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t r = b;
        for (int i = 0; i < 8; i++)
            r = (r >> 1) ^ ((r & 1u) ? CRC32C_POLY_REFLECTED : 0u);
        tbl[0][b] = r;
    }
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t r = tbl[0][b];
        for (int k = 1; k < 8; k++) {
            r = tbl[0][r & 0xffu] ^ (r >> 8);
            tbl[k][b] = r;
        }
    }
}

void or_crc32c_init(void) { pthread_once(&tbl_once, build_tables); }

/* crc32c_sw, crc32c.c:97-134: align to 8, then 8 bytes per step. */
uint32_t or_crc32c(uint32_t crc, const void *buf, size_t len) {
    const uint8_t *p = (const uint8_t *)buf;
    uint64_t c = (uint64_t)(crc ^ 0xffffffffu);
    or_crc32c_init();
    while (len && ((uintptr_t)p & 7u)) {
        c = tbl[0][(c ^ *p++) & 0xffu] ^ (c >> 8);
        len--;
    }
    while (len >= 8) {
        uint64_t w;
        memcpy(&w, p, 8); /* little-endian host */
        c ^= w;
        c = tbl[7][c & 0xff] ^ tbl[6][(c >> 8) & 0xff] ^
            tbl[5][(c >> 16) & 0xff] ^ tbl[4][(c >> 24) & 0xff] ^
            tbl[3][(c >> 32) & 0xff] ^ tbl[2][(c >> 40) & 0xff] ^
            tbl[1][(c >> 48) & 0xff] ^ tbl[0][c >> 56];
        p += 8;
        len -= 8;
    }
    while (len--) c = tbl[0][(c ^ *p++) & 0xffu] ^ (c >> 8);
    return (uint32_t)c ^ 0xffffffffu;
}

/* Definition of CRC-32C, one bit at a time (independent of the tables). */
uint32_t or_crc32c_bitwise(uint32_t crc, const void *buf, size_t len) {
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t c = ~crc;
    for (size_t i = 0; i < len; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++)
            c = (c >> 1) ^ (CRC32C_POLY_REFLECTED & (0u - (c & 1u)));
    }
    return ~c;
}

/* ---- GF(2) operators: crc32c.c:144-231 restated ------------------------- */

/* mat is 32 column vectors; returns mat * vec over GF(2) (crc32c.c:144). */
static uint32_t gf2_times(const uint32_t mat[32], uint32_t vec) {
    uint32_t s = 0;
    for (int i = 0; vec; i++, vec >>= 1)
        if (vec & 1u) s ^= mat[i];
    return s;
}

static void gf2_square(uint32_t dst[32], const uint32_t src[32]) {
    for (int i = 0; i < 32; i++) dst[i] = gf2_times(src, src[i]);
}

/* Operator that appends `nbytes` zero bytes to a raw CRC register
 * (crc32c_zeros_op, crc32c.c:173, generalised to any length by binary
 * decomposition instead of powers of two only). */
static void zeros_op(uint32_t op[32], size_t nbytes) {
    uint32_t one_bit[32], p[32], t[32];
    one_bit[0] = CRC32C_POLY_REFLECTED;
    for (int i = 1; i < 32; i++) one_bit[i] = 1u << (i - 1);
    gf2_square(t, one_bit);   /* 2 bits */
    gf2_square(p, t);         /* 4 bits */
    gf2_square(t, p);         /* 8 bits = 1 byte */
    memcpy(p, t, sizeof p);   /* p = operator for 1 byte */
    for (int i = 0; i < 32; i++) op[i] = 1u << i; /* identity */
    while (nbytes) {
        if (nbytes & 1u) {
            uint32_t r[32];
            for (int i = 0; i < 32; i++) r[i] = gf2_times(p, op[i]);
            memcpy(op, r, sizeof r);
        }
        nbytes >>= 1;
        if (!nbytes) break;
        gf2_square(t, p);
        memcpy(p, t, sizeof p);
    }
}

uint32_t or_crc32c_combine(uint32_t crcA, uint32_t crcB, size_t lenB) {
    uint32_t op[32];
    zeros_op(op, lenB);
    /* crc(A||B) = shift_lenB(crcA) ^ crcB: the pre/post inversions of the
     * two halves cancel exactly as in the 3-way merge at crc32c.c:290-291. */
    return gf2_times(op, crcA) ^ crcB;
}

/* ---- HW path (crc32c_hw, crc32c.c:236-338) ------------------------------- */
#if defined(__x86_64__)
#define HW_LONG 8192
#define HW_SHORT 256
static uint32_t shift_long[4][256], shift_short[4][256];
static int hw_ok = -1;
static pthread_once_t hw_once = PTHREAD_ONCE_INIT;

static void build_shift(uint32_t z[4][256], size_t n) {
    uint32_t op[32];
    zeros_op(op, n);
    for (uint32_t b = 0; b < 256; b++)
        for (int j = 0; j < 4; j++) z[j][b] = gf2_times(op, b << (8 * j));
}

static void hw_init(void) {
    unsigned a, b, c, d;
    hw_ok = 0;
    if (__get_cpuid(1, &a, &b, &c, &d) && ((c >> 20) & 1u)) hw_ok = 1;
    build_shift(shift_long, HW_LONG);
    build_shift(shift_short, HW_SHORT);
}

static inline uint32_t apply_shift(uint32_t z[4][256], uint32_t c) {
    return z[0][c & 0xff] ^ z[1][(c >> 8) & 0xff] ^ z[2][(c >> 16) & 0xff] ^
           z[3][c >> 24];
}

int or_crc32c_hw_available(void) {
    pthread_once(&hw_once, hw_init);
    return hw_ok;
}

__attribute__((target("sse4.2")))
uint32_t or_crc32c_hw(uint32_t crc, const void *buf, size_t len) {
    const uint8_t *p = (const uint8_t *)buf;
    uint64_t c0 = crc ^ 0xffffffffu, c1, c2;
    pthread_once(&hw_once, hw_init);
    while (len && ((uintptr_t)p & 7u)) { c0 = _mm_crc32_u8((uint32_t)c0, *p++); len--; }
    while (len >= 3 * HW_LONG) {
        const uint8_t *end = p + HW_LONG;
        c1 = c2 = 0;
        do {
            uint64_t a, b, e;
            memcpy(&a, p, 8); memcpy(&b, p + HW_LONG, 8); memcpy(&e, p + 2 * HW_LONG, 8);
            c0 = _mm_crc32_u64(c0, a); c1 = _mm_crc32_u64(c1, b); c2 = _mm_crc32_u64(c2, e);
            p += 8;
        } while (p < end);
        c0 = apply_shift(shift_long, (uint32_t)c0) ^ (uint32_t)c1;
        c0 = apply_shift(shift_long, (uint32_t)c0) ^ (uint32_t)c2;
        p += 2 * HW_LONG;
        len -= 3 * HW_LONG;
    }
    while (len >= 3 * HW_SHORT) {
        const uint8_t *end = p + HW_SHORT;
        c1 = c2 = 0;
        do {
            uint64_t a, b, e;
            memcpy(&a, p, 8); memcpy(&b, p + HW_SHORT, 8); memcpy(&e, p + 2 * HW_SHORT, 8);
            c0 = _mm_crc32_u64(c0, a); c1 = _mm_crc32_u64(c1, b); c2 = _mm_crc32_u64(c2, e);
            p += 8;
        } while (p < end);
        c0 = apply_shift(shift_short, (uint32_t)c0) ^ (uint32_t)c1;
        c0 = apply_shift(shift_short, (uint32_t)c0) ^ (uint32_t)c2;
        p += 2 * HW_SHORT;
        len -= 3 * HW_SHORT;
    }
    while (len >= 8) { uint64_t a; memcpy(&a, p, 8); c0 = _mm_crc32_u64(c0, a); p += 8; len -= 8; }
    while (len--) c0 = _mm_crc32_u8((uint32_t)c0, *p++);
    return (uint32_t)c0 ^ 0xffffffffu;
}
#else
int or_crc32c_hw_available(void) { return 0; }
uint32_t or_crc32c_hw(uint32_t crc, const void *buf, size_t len) {
    return or_crc32c(crc, buf, len);
}
#endif

/* ---- threaded batch driver (CPU baseline) -------------------------------- */
struct crc_job {
    const uint8_t *base; const uint64_t *offs; const uint32_t *lens;
    uint32_t *out; size_t lo, hi; int hw;
};

static void *crc_worker(void *arg) {
    struct crc_job *j = (struct crc_job *)arg;
    for (size_t i = j->lo; i < j->hi; i++)
        j->out[i] = j->hw ? or_crc32c_hw(0, j->base + j->offs[i], j->lens[i])
                          : or_crc32c(0, j->base + j->offs[i], j->lens[i]);
    return NULL;
}

void or_crc32c_batches_mt(const uint8_t *base, const uint64_t *offs,
                          const uint32_t *lens, uint32_t *out, size_t n,
                          int threads) {
    if (threads < 1) threads = 1;
    if (threads > 512) threads = 512;
    int hw = or_crc32c_hw_available();
    or_crc32c_init();
    pthread_t th[512];
    struct crc_job jobs[512];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (struct crc_job){base, offs, lens, out, n * t / threads,
                                   n * (t + 1) / threads, hw};
        pthread_create(&th[t], NULL, crc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
