/*
 * driver.c -- TEST FIXTURE: an "application" linked against libhostpath.so only.  It
 * builds a two-segment slice, calls the library's writer / reader call sites and prints
 * what came back, one `key value` per line.  Run plainly it reaches the host library's own
 * definitions; run with LD_PRELOAD=librdkafka_hip.so the same call sites reach the engine.
 *
 * Build: gcc -O1 -o driver driver.c -L. -lhostpath -Wl,-rpath,'$ORIGIN'
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct rd_segment_s {
    struct { struct rd_segment_s *tqe_next; struct rd_segment_s **tqe_prev; } seg_link;
    char *seg_p;
    size_t seg_of, seg_size, seg_absof;
    void (*seg_free)(void *p);
    int seg_flags;
} rd_segment_t;
typedef struct rd_slice_s {
    const void *buf;
    const rd_segment_t *seg;
    size_t rof, start, end;
} rd_slice_t;

uint32_t host_writer_calc_crc(rd_slice_t *slice);
int host_writer_compress(rd_slice_t *slice, void **out, size_t *outlen);
int host_reader_decompress(char *in, size_t inlen, void **out, size_t *outlen);
extern int host_calls_crc32c, host_calls_slice, host_calls_lz4c, host_calls_lz4d;

static void make_slice(rd_slice_t *sl, rd_segment_t seg[2], char *data, size_t n, size_t cut) {
    memset(seg, 0, 2 * sizeof seg[0]);
    seg[0].seg_p = data;        seg[0].seg_of = seg[0].seg_size = cut;     seg[0].seg_absof = 0;
    seg[1].seg_p = data + cut;  seg[1].seg_of = seg[1].seg_size = n - cut; seg[1].seg_absof = cut;
    seg[0].seg_link.tqe_next = &seg[1];
    memset(sl, 0, sizeof *sl);
    sl->seg = &seg[0];
    sl->end = n;
}

int main(int argc, char **argv) {
    size_t n = argc > 1 ? (size_t)atol(argv[1]) : 200000;
    char *data = malloc(n + 1);
    uint32_t s = 42;
    for (size_t i = 0; i < n; i++) { /* compressible text, LCG-driven */
        s = s * 1103515245u + 12345u;
        data[i] = "{\"id\":0,\"user\":\"u1\",\"event\":\"click\"}\n"[(i + ((s >> 16) % 3)) % 38];
    }
    rd_segment_t seg[2];
    rd_slice_t sl;
    make_slice(&sl, seg, data, n, 61);
    printf("crc %08x\n", host_writer_calc_crc(&sl));
    make_slice(&sl, seg, data, n, n / 3);
    void *frame = NULL;
    size_t flen = 0;
    int e = host_writer_compress(&sl, &frame, &flen);
    printf("compress_err %d\ncompress_len %zu\n", e, flen);
    if (e == 0) {
        void *back = NULL;
        size_t blen = 0;
        int e2 = host_reader_decompress(frame, flen, &back, &blen);
        printf("decompress_err %d\nroundtrip %d\n", e2,
               e2 == 0 && blen == n && memcmp(back, data, n) == 0);
        fwrite(frame, 1, flen, stderr); /* the frame itself, for the caller to check */
        free(back);
        free(frame);
    }
    printf("host_calls crc32c=%d slice=%d lz4c=%d lz4d=%d\n", host_calls_crc32c, host_calls_slice,
           host_calls_lz4c, host_calls_lz4d);
    FILE *f = fopen(argc > 2 ? argv[2] : "/dev/null", "wb");
    if (f) { fwrite(data, 1, n, f); fclose(f); }
    return 0;
}
