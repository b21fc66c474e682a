/*
 * hostlib.c -- TEST FIXTURE: a shared library shaped like the reference's CMake build of
 * librdkafka.so as far as symbol binding goes.  The internal functions of the hot path
 * (crc32c, rd_slice_crc32c, rd_kafka_lz4_compress, rd_kafka_lz4_decompress) are defined
 * here with default visibility and reached by their callers through the PLT, exactly as
 * an objdump of the reference's CMake build shows (`call crc32c@plt` from rd_slice_crc32c,
 * `call rd_slice_crc32c@plt` from the writer, ...).  The definitions here are deliberately
 * NOT the reference's code: crc32c is a bit-at-a-time loop and the LZ4 functions only
 * report that they ran.  The test preloads librdkafka_hip.so and checks that the CALLERS
 * in this library then reach the engine's definitions instead (ELF symbol interposition),
 * which is how the engine binds to the real library under LD_PRELOAD.
 *
 * Build: gcc -O1 -fPIC -shared -o libhostpath.so hostlib.c
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

/* src/rdbuf.h:63-115 layout (what the writer hands to these functions) */
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

#define HOST_SENTINEL_ERR (-12345) /* "the host library's own LZ4 stub ran" */

int host_calls_crc32c, host_calls_slice, host_calls_lz4c, host_calls_lz4d;

uint32_t crc32c(uint32_t crc, const void *buf, size_t len) {
    const uint8_t *p = buf;
    host_calls_crc32c++;
    crc = ~crc;
    while (len--) {
        crc ^= *p++;
        for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ ((crc & 1) ? 0x82f63b78u : 0);
    }
    return ~crc;
}

uint32_t rd_slice_crc32c(rd_slice_t *slice) {
    uint32_t crc = 0;
    host_calls_slice++;
    /* contiguous segments only: enough for the fixture */
    for (const rd_segment_t *s = slice->seg; s; s = s->seg_link.tqe_next)
        crc = crc32c(crc, s->seg_p, s->seg_of); /* call crc32c@plt */
    slice->seg = NULL;
    return crc;
}

int rd_kafka_lz4_compress(void *rkb, int proper_hc, int comp_level, rd_slice_t *slice,
                          void **outbuf, size_t *outlenp) {
    host_calls_lz4c++;
    *outbuf = NULL;
    *outlenp = 0;
    return HOST_SENTINEL_ERR;
}

int rd_kafka_lz4_decompress(void *rkb, int proper_hc, int64_t Offset, char *inbuf, size_t inlen,
                            void **outbuf, size_t *outlenp) {
    host_calls_lz4d++;
    *outbuf = NULL;
    *outlenp = 0;
    return HOST_SENTINEL_ERR;
}

/* ---- the callers: stand-ins for the two call sites of the MessageSet writer / reader */

/* rd_kafka_msgset_writer_calc_crc_v2 (rdkafka_msgset_writer.c:1229-1246) */
uint32_t host_writer_calc_crc(rd_slice_t *slice) { return rd_slice_crc32c(slice); }

/* rd_kafka_msgset_writer_compress_lz4 (rdkafka_msgset_writer.c:1089-1101) */
int host_writer_compress(rd_slice_t *slice, void **out, size_t *outlen) {
    return rd_kafka_lz4_compress(NULL, 1, 0, slice, out, outlen);
}

/* rd_kafka_msgset_reader_decompress, LZ4 case (rdkafka_msgset_reader.c:393-407) */
int host_reader_decompress(char *in, size_t inlen, void **out, size_t *outlen) {
    return rd_kafka_lz4_decompress(NULL, 1, 0, in, inlen, out, outlen);
}
