/*
 * librdkafka_hip.h -- C ABI of librdkafka_hip.so, the MI355X (gfx950) engine
 * for librdkafka's per-MessageSet data-parallel work: CRC32C over MsgVersion 2
 * record batches and LZ4F frame compression / decompression.
 *
 * Two layers:
 *
 *  1. DROP-IN symbols.  Exactly the internal librdkafka v1.3.0 functions the
 *     MessageSet writer/reader call through the PLT, with identical
 *     signatures, ownership and error contracts.  Preloading (or linking
 *     ahead of librdkafka.so) interposes them.
 *
 *  2. ENGINE batch API (rdk_hip_*).  Device-resident batches of many
 *     toppars' record batches, processed in one launch per stage on a caller
 *     stream.  Plain pointers and sizes only; `stream` is a hipStream_t
 *     passed as void* (NULL = the HIP null stream, as in the HIP API).
 *
 * Every function that touches the GPU fails loudly when no gfx950 device /
 * code object is available or a device call fails; there is no CPU path (the
 * only CPU work in the engine is frame-header bookkeeping):
 *   - rdk_hip_* return RDK_HIP_E_* and set rdk_hip_last_error();
 *   - rd_kafka_lz4_compress / _decompress return the reference's own codes
 *     (__CRIT_SYS_RESOURCE: no device or out of memory; __BAD_COMPRESSION: any
 *     other device failure) and report the first failure on stderr, so the
 *     writer sends the MessageSet uncompressed (rdkafka_msgset_writer.c:1175)
 *     and the reader raises a consumer error (rdkafka_msgset_reader.c:517-526);
 *   - crc32c / rd_slice_crc32c / rd_slice_crc32 return the checksum itself and
 *     have no error channel.  With no usable device the process is aborted with
 *     a message.  With a device, a failed call (allocation, copy, launch) is
 *     retried once; if that fails too, that one call's checksum is finished on
 *     the host from the bytes already staged, reported on stderr the first time
 *     and counted (rdk_hip_dropin_host_crcs), rather than handing back a wrong
 *     CRC or taking the producer down.
 */
#ifndef LIBRDKAFKA_HIP_H
#define LIBRDKAFKA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------
 * Boundary types (opaque / mirrored).
 * rd_slice_t is walked with the exact layout of src/rdbuf.h:63-115 (mirrored
 * privately in csrc/rdbuf_abi.h); the broker handle is never dereferenced.
 * ------------------------------------------------------------------------- */
typedef struct rd_slice_s rd_slice_t;
typedef struct rd_kafka_broker_s rd_kafka_broker_t;
typedef int rd_kafka_resp_err_t; /* enum in rdkafka.h:258-268 */

#define RDK_HIP_RESP_ERR_NO_ERROR 0
#define RDK_HIP_RESP_ERR__BAD_MSG (-199)            /* rdkafka.h:258 */
#define RDK_HIP_RESP_ERR__BAD_COMPRESSION (-198)    /* rdkafka.h:260 */
#define RDK_HIP_RESP_ERR__CRIT_SYS_RESOURCE (-194)  /* rdkafka.h:268 */

/* ------------------------------------------------------------------ drop-in */

/* Replaces crc32c() (src/crc32c.h:32, src/crc32c.c:360-368).  `crc` is the
 * previous result (0 to start): crc32c(crc32c(0,a),b) == crc32c(0,a||b). */
uint32_t crc32c(uint32_t crc, const void *buf, size_t len);

/* Replaces crc32c_global_init() (src/crc32c.c:378-386): idempotent; brings
 * up the device context and uploads the CRC tables. */
void crc32c_global_init(void);

/* Replaces rd_slice_crc32c() (src/rdbuf.c:1113-1122): CRC32C of the slice's
 * remaining segments, leaving the slice fully consumed exactly like the
 * rd_slice_reader() loop it replaces. */
uint32_t rd_slice_crc32c(rd_slice_t *slice);

/* Replaces rd_slice_crc32() (src/rdbuf.c:1093-1104): CRC-32 (zlib crc32(),
 * rdcrc32.h:93-131 under WITH_ZLIB) of the slice's remaining segments, leaving
 * the slice consumed.  The MsgVersion 0/1 reader's check.crcs site
 * (rdkafka_msgset_reader.c:606). */
uint32_t rd_slice_crc32(rd_slice_t *slice);

/* Replaces rd_kafka_lz4_compress() (src/rdkafka_lz4.c:329-442).  LZ4F frame
 * with prefs {blockIndependent, comp_level}, 64 KB blocks; *outbuf is
 * malloc()ed (caller frees with free()); slice is consumed.  comp_level < 3
 * runs LZ4_compress_generic's parse, 3..9 the LZ4HC hash-chain parse
 * (lz4frame.c:797-805, lz4hc.c:532) and 10..12 the LZ4HC optimal parse
 * (lz4hc.c:1278; higher levels clamp to 12, lz4hc.c:798), all byte-identical
 * to the reference's frames.  A device failure returns __BAD_COMPRESSION (the
 * writer then sends the MessageSet uncompressed, rdkafka_msgset_writer.c:1175).
 * No call is ever forwarded to another definition of the symbol. */
rd_kafka_resp_err_t rd_kafka_lz4_compress(rd_kafka_broker_t *rkb, int proper_hc,
                                          int comp_level, rd_slice_t *slice,
                                          void **outbuf, size_t *outlenp);

/* Replaces rd_kafka_lz4_decompress() (src/rdkafka_lz4.c:167-317).  *outbuf
 * is malloc()ed.  May modify inbuf only when !proper_hc.  The output buffer
 * is sized exactly from the frame's block table, so rkb_c.zbuf_grow is never
 * incremented (documented divergence; rkb is not dereferenced). */
rd_kafka_resp_err_t rd_kafka_lz4_decompress(rd_kafka_broker_t *rkb, int proper_hc,
                                            int64_t Offset, char *inbuf, size_t inlen,
                                            void **outbuf, size_t *outlenp);

/* How often each drop-in symbol above has been entered in this process, in the order
 * crc32c, rd_slice_crc32c, rd_slice_crc32, rd_kafka_lz4_compress, rd_kafka_lz4_decompress.
 * No counterpart in the reference: it lets an integration (a preload run, a relinked
 * library) verify that the writer's and reader's call sites bind to this library.  With
 * RDK_HIP_REPORT=1 in the environment the same counts are printed on stderr at exit. */
void rdk_hip_dropin_calls(uint64_t out[5]);
/* How many CRC drop-in calls finished on the host after the device path failed twice
 * (see the error contract at the top).  0 in a healthy process; the GPU tests assert it. */
uint64_t rdk_hip_dropin_host_crcs(void);
/* Concurrent calls of the symbols above from several threads (librdkafka's broker threads,
 * rdkafka_broker.c:5082) are served together: a thread that finds no batch in flight takes
 * every request queued so far to the device as one staging copy and one launch of each
 * batch kernel; a thread that is about to serve fewer requests than the previous batch held
 * waits at most RDK_HIP_COMBINE_WAIT_US microseconds (default 50; linger.ms is 500,
 * rdkafka_conf.c:1095) for the others; a lone caller never waits.  CRC and decompress
 * requests above 128 KiB go on their own thread's stream (their host copies dominate and
 * run in parallel that way).  RDK_HIP_COMBINE=0 turns
 * this off (every call on its own thread's stream).  out[0] = batches of two or more
 * requests so far, out[1] = requests served in them, out[2] = the largest batch, out[3] =
 * batches that fell back to one request at a time after a device error.  No counterpart
 * in the reference. */
void rdk_hip_dropin_combined(uint64_t out[4]);
/* Engine contexts created / destroyed so far.  Every calling thread gets one context (HIP
 * stream, pinned staging, device scratch) on its first call; it is released when the
 * thread exits, as librdkafka's broker threads do (rdkafka_broker.c:5082).  No
 * counterpart in the reference. */
void rdk_hip_ctx_counts(uint64_t out[2]);

/* ---- snappy drop-ins (src/snappy.h).  Same signatures, return values and ownership as
 * the reference's definitions in src/snappy.c; the writer reaches them from
 * rd_kafka_msgset_writer_compress_snappy (rdkafka_msgset_writer.c:1041-1083), the reader
 * from its snappy case (rdkafka_msgset_reader.c:299-390).  Streams are byte-identical to
 * compress_fragment's (snappy.c:957); the decoder returns 0 / -EIO under the conditions
 * of decompress_all_tags (snappy.c:1226) and writer_append* (:543, :572).  The
 * environment carries no state here (the hash table lives in LDS). */
struct snappy_env;
struct iovec;
int rd_kafka_snappy_init_env(struct snappy_env *env);                 /* snappy.c:1809 */
int rd_kafka_snappy_init_env_sg(struct snappy_env *env, bool sg);     /* snappy.c:1778 */
void rd_kafka_snappy_free_env(struct snappy_env *env);                /* snappy.c:1825 */
size_t rd_kafka_snappy_max_compressed_length(size_t source_len);      /* snappy.c:639 */
bool rd_kafka_snappy_uncompressed_length(const char *buf, size_t len, size_t *result); /* :751 */
int rd_kafka_snappy_compress_iov(struct snappy_env *env, const struct iovec *iov_in,
                                 size_t iov_in_cnt, size_t input_length,
                                 struct iovec *iov_out);              /* snappy.c:1488 */
int rd_kafka_snappy_compress(struct snappy_env *env, const char *input, size_t input_length,
                             char *compressed, size_t *compressed_length); /* snappy.c:1526 */
int rd_kafka_snappy_uncompress(const char *compressed, size_t n, char *uncompressed); /* :1572 */
char *rd_kafka_snappy_java_uncompress(const char *inbuf, size_t inlen, size_t *outlenp,
                                      char *errstr, size_t errstr_size);  /* snappy.c:1588 */
/* calls of the snappy drop-ins so far: [0] compress, [1] uncompress (bare or snappy-java);
 * no counterpart in the reference (see rdk_hip_dropin_calls) */
void rdk_hip_snappy_dropin_calls(uint64_t out[2]);

/* ------------------------------------------------------------- engine API */
#define RDK_HIP_OK 0
#define RDK_HIP_E_NODEV (-1)      /* no usable gfx950 device / code object */
#define RDK_HIP_E_HIP (-2)        /* HIP runtime error (launch, alloc, copy) */
#define RDK_HIP_E_INVAL (-3)      /* bad argument */
#define RDK_HIP_E_NOMEM (-4)

/* Bind the calling thread's engine context to `device` (default: device 0 or
 * $RDK_HIP_DEVICE).  Safe to call repeatedly. */
int rdk_hip_init(int device);
const char *rdk_hip_last_error(void);
/* Engine build/feature string (arch, kernel variants). */
const char *rdk_hip_version(void);

/* CRC32C of n independent byte ranges of device memory.
 *   d_base + d_offs[i], length d_lens[i]; init crc d_init[i] (NULL = 0);
 *   result -> d_out[i].  Same chaining semantics as crc32c(). */
int rdk_hip_crc32c_ranges(const void *d_base, const uint64_t *d_offs,
                          const uint32_t *d_lens, const uint32_t *d_init,
                          uint32_t *d_out, uint32_t n, void *stream);

/* Same for CRC-32 (zlib crc32(): MsgVersion 0/1, rdcrc32.h:93-131). */
int rdk_hip_crc32_ranges(const void *d_base, const uint64_t *d_offs,
                         const uint32_t *d_lens, const uint32_t *d_init,
                         uint32_t *d_out, uint32_t n, void *stream);

/* MsgVersion 0/1 MessageSets at d_base + d_set_offs[i], d_set_lens[i] bytes:
 * the reader's message walk and check.crcs (rd_kafka_msgset_reader_msg_v0_1,
 * rdkafka_msgset_reader.c:538-628) / the writer's per-message Crc
 * (rd_kafka_msgset_writer_write_msg_v0_1, rdkafka_msgset_writer.c:583-645).
 * Message k of set i goes to row d_row_offs[i] + k (at most d_row_caps[i]):
 *   d_msg_pos[row] = message start (its Offset field) from the set start
 *   d_msg_out[row] = CRC-32 of [16, 12+MessageSize) (mode COMPUTE / FINALIZE,
 *                    FINALIZE also stores it big-endian at the Crc field, +12)
 *                    or 0 / 1 = stored Crc matches / does not (mode VERIFY; the
 *                    reader skips such a message and continues, :612-627)
 *   d_count[i]     = number of whole messages (a partial message at the end
 *                    stops the walk, :599-600), or -(1+k) when message k fails
 *                    the header checks (MessageSize < hdrsize :590-597, or < 4)
 *                    or does not fit in the rows.
 * Modes are RDK_HIP_V2_CRC_COMPUTE / _FINALIZE / _VERIFY. */
int rdk_hip_msgset_v01_crc(void *d_base, const uint64_t *d_set_offs,
                           const uint32_t *d_set_lens, const uint64_t *d_row_offs,
                           const uint32_t *d_row_caps, uint32_t *d_msg_pos,
                           uint32_t *d_msg_out, int32_t *d_count, uint32_t n, int mode,
                           void *stream);

/* MsgVersion 2 record batches laid out at d_base + d_batch_offs[i].  The CRC
 * range is [21, 12+Length) read from each header (big-endian Length at 8),
 * as computed by rd_kafka_msgset_writer_calc_crc_v2
 * (rdkafka_msgset_writer.c:1229-1246) and verified by
 * rd_kafka_msgset_reader_v2 (rdkafka_msgset_reader.c:982-1015).
 *   mode RDK_HIP_V2_CRC_COMPUTE : d_out[i] = crc
 *   mode RDK_HIP_V2_CRC_FINALIZE: also store it big-endian at offset 17
 *   mode RDK_HIP_V2_CRC_VERIFY  : d_out[i] = (crc == stored) ? 0 : 1
 * Batches whose Length is < 9 or exceeds d_batch_caps[i]-12 get d_out = 2
 * (VERIFY) / are skipped. */
#define RDK_HIP_V2_CRC_COMPUTE 0
#define RDK_HIP_V2_CRC_FINALIZE 1
#define RDK_HIP_V2_CRC_VERIFY 2
int rdk_hip_msgset_v2_crc(void *d_base, const uint64_t *d_batch_offs,
                          const uint32_t *d_batch_caps, uint32_t *d_out,
                          uint32_t n, int mode, void *stream);

/* LZ4F compression of n independent inputs (rd_kafka_lz4_compress semantics
 * per input, prefs {blockIndependent, level}).  Frame i is written to
 * d_out + d_out_offs[i] (capacity rdk_hip_lz4f_compress_bound(len)); its
 * size goes to d_out_lens[i].  `level` as compression.level: < 3 the fast
 * parse, 3..9 the LZ4HC hash chain, 10..12 the LZ4HC optimal parser
 * (byte-identical frames at every level). */
size_t rdk_hip_lz4f_compress_bound(size_t len);
int rdk_hip_lz4f_compress(const void *d_in, const uint64_t *d_in_offs,
                          const uint32_t *d_in_lens, void *d_out,
                          const uint64_t *d_out_offs, uint32_t *d_out_lens,
                          uint32_t n, int level, void *stream);

/* snappy compression of n independent inputs (rd_kafka_snappy_compress_iov semantics per
 * input, snappy.c:1488): stream i = varint32 length + the 64 KiB fragments of
 * compress_fragment (snappy.c:957), byte-identical to the reference's, written to
 * d_out + d_out_offs[i] (capacity rdk_hip_snappy_max_compressed_length(len), which is
 * also used as staging room); its size goes to d_out_lens[i]. */
size_t rdk_hip_snappy_max_compressed_length(size_t len);
int rdk_hip_snappy_compress(const void *d_in, const uint64_t *d_in_offs,
                            const uint32_t *d_in_lens, void *d_out,
                            const uint64_t *d_out_offs, uint32_t *d_out_lens,
                            uint32_t n, void *stream);
/* snappy decompression of n streams (rd_kafka_snappy_uncompress semantics per stream,
 * snappy.c:1572): d_out_lens[i] = the length the preamble declares, d_status[i] = 0 or
 * RDK_HIP_SNAPPY_E_IO (-EIO, the reference's verdict), or RDK_HIP_SNAPPY_E_DSTSIZE when
 * d_out_caps[i] is below the declared length (the reader sizes its buffer from
 * rd_kafka_snappy_uncompressed_length first, rdkafka_msgset_reader.c:345-361).  The
 * chunks of a snappy-java frame (snappy.c:1588) are n streams of one call. */
#define RDK_HIP_SNAPPY_E_IO (-5)
#define RDK_HIP_SNAPPY_E_DSTSIZE (-1001)
int rdk_hip_snappy_uncompress(const void *d_in, const uint64_t *d_in_offs,
                              const uint32_t *d_in_lens, void *d_out,
                              const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                              uint32_t *d_out_lens, int32_t *d_status, uint32_t n,
                              void *stream);

/* Throughput-mode LZ4F compression: same arguments, frame format, prefs
 * ({blockIndependent}, 64 KB blocks, no checksums) and raw-block fallback
 * (lz4frame.c:739-761) as rdk_hip_lz4f_compress, but the match search is the
 * engine's own wavefront-parallel one (dense LZ4_hash4 table, 64 positions per
 * step), not an emulation of LZ4_compress_generic.  Frames decode with the
 * reference's rd_kafka_lz4_decompress (rdkafka_lz4.c:167) to the input;
 * they are not byte-identical to rd_kafka_lz4_compress's (rdkafka_lz4.c:329);
 * the compression ratio is within 5 % of it (tests/test_gpu_lz4.py). */
int rdk_hip_lz4f_compress_fast(const void *d_in, const uint64_t *d_in_offs,
                               const uint32_t *d_in_lens, void *d_out,
                               const uint64_t *d_out_offs, uint32_t *d_out_lens,
                               uint32_t n, void *stream);

/* The same contract as rdk_hip_lz4f_compress_fast on another engine: one 1024-thread
 * workgroup per 64 KB block with the block's source, the hash table and the output
 * staging in LDS, so a block's bytes are read from memory once and its output leaves in
 * aligned 16-byte stores (the one-wavefront-per-block engine behind _fast gathers its
 * candidates from memory).  Its output is defined by a sequential model
 * (tests/sim/lz4_units_sim.cpp) that it reproduces byte for byte.  No counterpart in the
 * reference.  RDK_HIP_LZ4_FAST_ENGINE=units in the environment makes _fast and the
 * producer's FAST mode run this engine. */
int rdk_hip_lz4f_compress_units(const void *d_in, const uint64_t *d_in_offs,
                                const uint32_t *d_in_lens, void *d_out,
                                const uint64_t *d_out_offs, uint32_t *d_out_lens,
                                uint32_t n, void *stream);

/* LZ4F decompression of n independent frames (rd_kafka_lz4_decompress
 * semantics per frame, proper HC).  Frame i decodes into
 * d_out + d_out_offs[i] with capacity d_out_caps[i]; d_out_lens[i] gets the
 * decoded size and d_status[i] the rd_kafka_resp_err_t (0, __BAD_MSG,
 * __BAD_COMPRESSION) or RDK_HIP_LZ4F_E_DSTSIZE when the capacity is short. */
#define RDK_HIP_LZ4F_E_DSTSIZE (-1000)
int rdk_hip_lz4f_decompress(const void *d_in, const uint64_t *d_in_offs,
                            const uint32_t *d_in_lens, void *d_out,
                            const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                            uint32_t *d_out_lens, int32_t *d_status, uint32_t n,
                            void *stream);

/* rdk_hip_lz4f_decompress for callers that cannot allocate (code under HIP
 * graph capture, tight serving loops, harnesses that forbid hipMalloc).  It has
 * no counterpart in the reference.  Same arguments and results; the frame and
 * block descriptor tables live in a fixed device array that is part of the
 * library (about 1.9 MB on every GPU the library is initialised on, held until
 * the process ends) instead of the per-thread scratch the plain entry point
 * grows on demand.  The call allocates and frees nothing and clears its work
 * counter with a kernel, not a memset.  rdk_hip_init(device) must have run for
 * the current device (it looks the array's address up); n is limited to
 * RDK_HIP_LZ4F_NOALLOC_MAX_FRAMES (RDK_HIP_E_INVAL beyond).  Every call on a GPU
 * shares that GPU's array: calls that overlap in time on one GPU race, so keep
 * them on one stream or order them yourself. */
#define RDK_HIP_LZ4F_NOALLOC_MAX_FRAMES 1024u
int rdk_hip_lz4f_decompress_noalloc(const void *d_in, const uint64_t *d_in_offs,
                                    const uint32_t *d_in_lens, void *d_out,
                                    const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                                    uint32_t *d_out_lens, int32_t *d_status, uint32_t n,
                                    void *stream);

/* ---------------------------------------------------------------------------
 * Producer batching front-end (pinned staging rings, copies overlapped with kernels).  One
 * producer per broker thread: a ring of `nslots` pinned host staging slots,
 * each with its own device buffers and HIP stream.  produce() gathers one
 * MsgVersion 2 batch -- the 61-byte header as the writer leaves it
 * (rdkafka_msgset_writer.c:352-403 / finalize_MessageSet_v2_header :1251-1295:
 * every field final except Length, the codec bits of Attributes and the CRC)
 * plus its uncompressed records -- into the filling slot.  A full slot (or
 * flush()) is launched as H2D -> LZ4F compress of every batch's records ->
 * header finalize (the frame is dropped when larger than the records,
 * rdkafka_msgset_writer.c:1179; Attributes |= LZ4 :1187; Length = size-12
 * :1265) -> CRC32C finalize (:1229-1246) -> D2H, on the slot's stream, so
 * the copies of one slot overlap the kernels of another.  poll() returns the
 * finished batches in submission order; `data` points into the producer's
 * pinned memory and stays valid until the next produce()/flush() call.
 * ------------------------------------------------------------------------- */
typedef struct rdk_hip_producer_s rdk_hip_producer_t;
typedef struct rdk_hip_batch_s {
  const void *data; /* finished v2 record batch (header + LZ4F or plain records) */
  uint32_t len;     /* bytes = 12 + Length */
  uint32_t crc;     /* the CRC32C stored big-endian at offset 17 */
  uint64_t cookie;  /* as passed to produce() */
} rdk_hip_batch_t;
#define RDK_HIP_PRODUCER_EXACT 0 /* frames byte-identical to rd_kafka_lz4_compress */
#define RDK_HIP_PRODUCER_FAST 1  /* rdk_hip_lz4f_compress_fast frames */
#define RDK_HIP_PRODUCER_SNAPPY 2 /* compression.codec=snappy: rdk_hip_snappy_compress streams */
#define RDK_HIP_E_BUSY (-5)      /* every slot is in flight: poll() first */
/* The writer's finalize (rd_kafka_msgset_writer_finalize, rdkafka_msgset_writer.c:1335:
 * rd_kafka_msgset_writer_compress :1128-1221 -> finalize_MessageSet_v2_header :1251-1295
 * -> calc_crc_v2 :1229-1246) for n device-resident MessageSets in one call.  Input i is
 * the 61-byte v2 header as the writer leaves it, immediately followed by the records at
 * d_in + d_rec_offs[i] (d_rec_lens[i] bytes; the header sits at d_rec_offs[i] - 61).
 * The finished batch is written to d_out + d_out_offs[i] (capacity d_out_caps[i] >=
 * 61 + rdk_hip_lz4f_compress_bound(len); offsets 16-byte aligned): header with Length
 * and the LZ4 codec bits set, the LZ4F frame (or the plain records when the frame would
 * be larger, :1179), CRC32C stored at offset 17.  d_frame_lens[i] = frame size,
 * d_batch_lens[i] = 12 + Length, d_crcs[i] = the CRC.  mode is RDK_HIP_PRODUCER_EXACT
 * (frames byte-identical to rd_kafka_lz4_compress at level 0), _FAST, or _SNAPPY (the
 * payload is the snappy stream of rd_kafka_snappy_compress_iov, the codec bits are 2 and
 * the slot capacity is 61 + rdk_hip_snappy_max_compressed_length(len)).  This is what
 * the producer front-end runs per staging slot. */
int rdk_hip_msgset_v2_finalize(const void *d_in, const uint64_t *d_rec_offs,
                               const uint32_t *d_rec_lens, void *d_out,
                               const uint64_t *d_out_offs, const uint32_t *d_out_caps,
                               uint32_t *d_frame_lens, uint32_t *d_batch_lens,
                               uint32_t *d_crcs, uint32_t n, int mode, void *stream);
rdk_hip_producer_t *rdk_hip_producer_new(int device, size_t slot_bytes, int nslots, int mode);
int rdk_hip_producer_produce(rdk_hip_producer_t *p, const void *hdr61, const void *records,
                             uint32_t len, uint64_t cookie);
int rdk_hip_producer_flush(rdk_hip_producer_t *p);
/* Up to `max` finished batches; block != 0 waits for the oldest slot.
 * Returns the number of batches, or an RDK_HIP_E_* code. */
int rdk_hip_producer_poll(rdk_hip_producer_t *p, rdk_hip_batch_t *out, int max, int block);
void rdk_hip_producer_destroy(rdk_hip_producer_t *p);

/* ---- MsgVersion 2 record serialisation ---------------------------------------
 * For device-resident messages, replaces
 *   rd_kafka_msgset_writer_write_MessageSet_v2_header  rdkafka_msgset_writer.c:352-403
 *   rd_kafka_msgset_writer_write_msg_v2                 rdkafka_msgset_writer.c:652-754
 *   rd_kafka_msgset_writer_finalize_MessageSet_v2_header rdkafka_msgset_writer.c:1251-1295
 * with write_msgq's batch semantics (:804-902): OffsetDelta = index in the batch,
 * TimestampDelta against the batch's first message, MaxTimestamp starting at 0.
 * Output: uncompressed batches (61-byte header + records), CRC optional. */
typedef struct rdk_hip_msgs_s {     /* all device pointers, one entry per message */
  const uint8_t *arena;             /* key / value / header bytes */
  const int64_t *timestamp;         /* rkm_timestamp */
  const uint64_t *key_off;
  const int32_t *key_len;           /* -1: null key (RD_KAFKAP_BYTES_LEN_NULL) */
  const uint64_t *value_off;
  const int32_t *value_len;         /* -1: null value */
  const uint64_t *headers_off;      /* headers already in wire form (:558-568) */
  const uint32_t *headers_len;
  const int32_t *header_count;      /* NULL: no message has headers */
} rdk_hip_msgs_t;
typedef struct rdk_hip_v2_batch_s { /* one MessageSet: messages [first_msg, +msg_count) */
  uint32_t first_msg, msg_count;
  int64_t producer_id;              /* msetw_pid.id (:392) */
  int32_t base_sequence;            /* msetw_batch->first_seq (:1289), -1 if none */
  int16_t producer_epoch;           /* (:395) */
  int16_t attributes;               /* codec bits etc. (:1271) */
} rdk_hip_v2_batch_t;
/* `batches` are HOST descriptors (copied to the device on `stream`).
 * Pass 1: d_rec_offs[m] = offset of message m's record from its batch start (header
 * included), d_batch_sizes[b] = 61 + records bytes, d_max_ts[b] = MaxTimestamp. */
int rdk_hip_msgset_v2_sizes(const rdk_hip_msgs_t *msgs, const rdk_hip_v2_batch_t *batches,
                            uint32_t n_batches, uint32_t *d_rec_offs, uint32_t *d_batch_sizes,
                            int64_t *d_max_ts, void *stream);
/* Pass 2: batch b written at d_out + d_out_offs[b] (d_batch_sizes[b] bytes); with d_crc
 * the CRC32C is stored at offset 17 as calc_crc_v2 does (:1229-1246) and in d_crc[b]. */
int rdk_hip_msgset_v2_write(const rdk_hip_msgs_t *msgs, const rdk_hip_v2_batch_t *batches,
                            uint32_t n_batches, const uint32_t *d_rec_offs,
                            const uint32_t *d_batch_sizes, const int64_t *d_max_ts,
                            const uint64_t *d_out_offs, uint8_t *d_out, uint32_t *d_crc,
                            void *stream);

/* ---- MsgVersion 2 record index -------------------------------------------------
 * rd_kafka_msgset_reader_msg_v2 (rdkafka_msgset_reader.c:715-927) for every record of
 * n batches, on the device: batch i's header (BaseOffset, BaseTimestamp) at
 * d_hdr_base + d_hdr_offs[i], its (uncompressed / decompressed) records at
 * d_rec_base + d_rec_offs[i], d_rec_lens[i] bytes.  Row j of batch i goes to
 * index d_row_offs[i] + j of every rows array (at most d_row_caps[i] rows):
 *   offset = BaseOffset + OffsetDelta (:742), timestamp = BaseTimestamp +
 *   TimestampDelta (:911-912, CreateTime), key/value offset (from the records start)
 *   and length (-1 = null), headers = HeaderCount varint + headers (binhdrs, :876-878).
 * d_count[i] = number of records, or -(1+j) when record j fails to parse (the
 * reader's rd_kafka_buf_parse_fail / underflow; fields overrunning the record's Length
 * fail; varints longer than 10 bytes fail).  Control batches, aborted transactions and
 * offsets below the fetch offset are the caller's (record-level filters of :744-865). */
typedef struct rdk_hip_v2_rows_s {  /* device arrays */
  int64_t *offset;
  int64_t *timestamp;
  uint32_t *key_off;
  int32_t *key_len;
  uint32_t *value_off;
  int32_t *value_len;
  uint32_t *headers_off;
  uint32_t *headers_len;
} rdk_hip_v2_rows_t;
int rdk_hip_msgset_v2_index(const void *d_hdr_base, const uint64_t *d_hdr_offs,
                            const void *d_rec_base, const uint64_t *d_rec_offs,
                            const uint32_t *d_rec_lens, const uint64_t *d_row_offs,
                            const uint32_t *d_row_caps, const rdk_hip_v2_rows_t *rows,
                            int32_t *d_count, uint32_t n_batches, void *stream);

/* Deterministic synthetic workloads generated on the device (bench/tests).
 * v2 batches: n batches of `batch_size` bytes at i*batch_size: a valid 61-byte
 * v2 header (Magic 2, Length = batch_size-12, RecordCount) followed by
 * splitmix64(seed) bytes; CRC field left 0. */
int rdk_hip_gen_v2_batches(void *d_base, uint32_t n, uint32_t batch_size,
                           uint64_t seed, void *stream);

/* Host-side JSON-like record stream: exactly `len`
 * bytes of `{"id":..,"user":"u.....","ts":..,"event":"..","value":..}\n`
 * records from the LCG s = s*1103515245+12345 seeded with `seed`. */
void rdk_hip_gen_json(uint8_t *dst, size_t len, uint32_t seed);

#ifdef __cplusplus
}
#endif
#endif /* LIBRDKAFKA_HIP_H */
