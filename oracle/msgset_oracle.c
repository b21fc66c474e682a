/*
 * msgset_oracle.c -- CPU restatement of the MsgVersion 2 record writer and
 * record parser.  TEST INFRASTRUCTURE ONLY.
 *
 * Reference (bluelichen19/librdkafka v1.3.0):
 *   varints     src/rdvarint.h:48-75 (encode), :114-141 (decode)
 *   batch head  src/rdkafka_msgset_writer.c:352-403 (write_MessageSet_v2_header)
 *   record      src/rdkafka_msgset_writer.c:652-754 (write_msg_v2)
 *   finalize    src/rdkafka_msgset_writer.c:1251-1295 (finalize_MessageSet_v2_header)
 *               + :1229-1246 (calc_crc_v2)
 *   batch loop  src/rdkafka_msgset_writer.c:804-902 (write_msgq: OffsetDelta = msgcnt,
 *               BaseTimestamp = first message, MaxTimestamp from 0)
 *   parser      src/rdkafka_msgset_reader.c:715-927 (reader_msg_v2)
 *
 * Parity pinning: rdvarint.h includes rd.h, which needs the generated config.h,
 * so the reference cannot be compiled here.  The varint
 * codec is pinned by the reference's own known answers (rdvarint.c:
 * unittest_rdvarint, tests/golden/varint_kat.json); the record layout is a
 * field-by-field restatement of the lines above ("parity unpinned" beyond the
 * varint vectors).
 */
#include <stdint.h>
#include <string.h>
#include <zlib.h>

#include "oracle.h"

/* rdvarint.h:48-63 -- unsigned LEB128 */
static size_t enc_u64(uint8_t *dst, uint64_t num) {
  size_t of = 0;
  do {
    dst[of++] = (uint8_t)((num & 0x7f) | (num > 0x7f ? 0x80 : 0));
    num >>= 7;
  } while (num);
  return of;
}

/* rdvarint.h:67-70 -- zig-zag then LEB128 */
size_t or_varint_enc_i64(uint8_t *dst, int64_t num) {
  return enc_u64(dst, ((uint64_t)num << 1) ^ (uint64_t)(num >> 63));
}

/* rdvarint.h:114-141 -- returns bytes read, 0 on failure (truncated / > 10 bytes) */
size_t or_varint_dec_i64(const uint8_t *src, size_t srcsize, int64_t *nump) {
  uint64_t num = 0;
  int shift = 0;
  size_t of = 0;
  do {
    if (of >= srcsize || shift > 63) return 0;
    num |= (uint64_t)(src[of] & 0x7f) << shift;
    shift += 7;
  } while (src[of++] & 0x80);
  *nump = (int64_t)(num >> 1) ^ -(int64_t)(num & 1);
  return of;
}

static void be16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static void be64(uint8_t *p, uint64_t v) { be32(p, (uint32_t)(v >> 32)); be32(p + 4, (uint32_t)v); }

/* Serialise messages [first, first+cnt) as one MsgVersion 2 batch into out
 * (uncompressed records); returns the batch size (61 + records). */
size_t or_msgset_v2_write(const uint8_t *arena, const int64_t *ts, const uint64_t *key_off,
                          const int32_t *key_len, const uint64_t *val_off, const int32_t *val_len,
                          const uint64_t *hdr_off, const uint32_t *hdr_len, const int32_t *hdr_cnt,
                          uint32_t first, uint32_t cnt, int64_t producer_id, int16_t producer_epoch,
                          int32_t base_sequence, int16_t attributes, uint8_t *out) {
  size_t pos = 61;  /* RD_KAFKAP_MSGSET_V2_SIZE */
  const int64_t base_ts = ts[first];   /* write_msgq :826 */
  int64_t max_ts = 0;                  /* write_msgq :813, :891 */
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t m = first + k;
    uint8_t vT[10], vO[10], vK[5], vV[5], vH[5], vL[10];
    const int32_t kl = key_len[m], vl = val_len[m];
    const int32_t hc = hdr_cnt ? hdr_cnt[m] : 0;
    const uint32_t hl = hdr_len ? hdr_len[m] : 0;
    if (max_ts < ts[m]) max_ts = ts[m];
    const size_t sT = or_varint_enc_i64(vT, ts[m] - base_ts);          /* :684 */
    const size_t sO = or_varint_enc_i64(vO, (int64_t)k);               /* :687 */
    const size_t sK = or_varint_enc_i64(vK, kl);                        /* :689 */
    const size_t sV = or_varint_enc_i64(vV, vl);                        /* :693 */
    const size_t sH = or_varint_enc_i64(vH, hc);                        /* :697 */
    const size_t kb = kl > 0 ? (size_t)kl : 0, vb = vl > 0 ? (size_t)vl : 0;
    const size_t msz = 1 + sT + sO + sK + kb + sV + vb + sH + hl;       /* :703 */
    const size_t sL = or_varint_enc_i64(vL, (int64_t)msz);             /* :715 */
    uint8_t *p = out + pos;
    memcpy(p, vL, sL); p += sL;
    *p++ = 0;                                                           /* :722 */
    memcpy(p, vT, sT); p += sT;
    memcpy(p, vO, sO); p += sO;
    memcpy(p, vK, sK); p += sK;
    if (kb) { memcpy(p, arena + key_off[m], kb); p += kb; }
    memcpy(p, vV, sV); p += sV;
    if (vb) { memcpy(p, arena + val_off[m], vb); p += vb; }
    memcpy(p, vH, sH); p += sH;
    if (hl) { memcpy(p, arena + hdr_off[m], hl); p += hl; }
    pos += sL + msz;
  }
  /* header: write_MessageSet_v2_header :362-401, finalize :1265-1292 */
  memset(out, 0, 61);
  be64(out + 0, 0);                        /* BaseOffset */
  be32(out + 8, (uint32_t)(pos - 12));     /* Length */
  be32(out + 12, 0);                       /* PartitionLeaderEpoch */
  out[16] = 2;                             /* Magic */
  be16(out + 21, (uint16_t)attributes);    /* Attributes (|= CREATE_TIME = 0) */
  be32(out + 23, cnt - 1);                 /* LastOffsetDelta */
  be64(out + 27, (uint64_t)base_ts);       /* BaseTimestamp */
  be64(out + 35, (uint64_t)max_ts);        /* MaxTimestamp */
  be64(out + 43, (uint64_t)producer_id);   /* ProducerId */
  be16(out + 51, (uint16_t)producer_epoch);
  be32(out + 53, (uint32_t)base_sequence); /* BaseSequence */
  be32(out + 57, cnt);                     /* RecordCount */
  be32(out + 17, or_crc32c(0, out + 21, pos - 21)); /* calc_crc_v2 :1235-1245 */
  return pos;
}

/* reader_msg_v2 :736-878 for every record of the batch records [rec, rec+len):
 * fills one index row per record; returns the number of records, or -(1 + i)
 * when record i fails to parse (rd_kafka_buf_parse_fail / underflow). */
long or_msgset_v2_index(const uint8_t *rec, size_t len, int64_t base_offset, int64_t base_ts,
                        int64_t *offset, int64_t *timestamp, uint32_t *key_off, int32_t *key_len,
                        uint32_t *val_off, int32_t *val_len, uint32_t *hdr_off, uint32_t *hdr_len,
                        long max_rows) {
  size_t pos = 0;
  long i = 0;
  while (pos < len) {
    int64_t L, tsd, od, kl, vl;
    size_t r;
    int8_t attr;
    if (i >= max_rows) return -(1 + i);
    if (!(r = or_varint_dec_i64(rec + pos, len - pos, &L))) return -(1 + i);  /* :736 */
    pos += r;
    if (L < 0 || (size_t)L > len - pos) return -(1 + i);
    const size_t end = pos + (size_t)L;                                       /* :737 */
    if (pos + 1 > end) return -(1 + i);
    attr = (int8_t)rec[pos++];                                                /* :738 */
    (void)attr;
    if (!(r = or_varint_dec_i64(rec + pos, end - pos, &tsd))) return -(1 + i);  /* :740 */
    pos += r;
    if (!(r = or_varint_dec_i64(rec + pos, end - pos, &od))) return -(1 + i);   /* :741 */
    pos += r;
    if (!(r = or_varint_dec_i64(rec + pos, end - pos, &kl))) return -(1 + i);   /* :871 */
    pos += r;
    if (kl < -1 || (kl > 0 && (size_t)kl > end - pos)) return -(1 + i);
    key_off[i] = (uint32_t)pos;
    key_len[i] = (int32_t)kl;
    if (kl > 0) pos += (size_t)kl;
    if (!(r = or_varint_dec_i64(rec + pos, end - pos, &vl))) return -(1 + i);   /* :872 */
    pos += r;
    if (vl < -1 || (vl > 0 && (size_t)vl > end - pos)) return -(1 + i);
    val_off[i] = (uint32_t)pos;
    val_len[i] = (int32_t)vl;
    if (vl > 0) pos += (size_t)vl;
    hdr_off[i] = (uint32_t)pos;                                               /* :876-878 */
    hdr_len[i] = (uint32_t)(end - pos);
    offset[i] = base_offset + od;                                             /* :742 */
    timestamp[i] = base_ts + tsd;                                             /* :910-912 */
    pos = end;
    ++i;
  }
  return i;
}

/* ======================================================================
 * MsgVersion 0/1 MessageSets and their per-message CRC-32.
 *
 *   CRC-32     rdcrc32.h:93-131; the reference is configured WITH_ZLIB, so this is zlib's
 *              crc32() (reflected 0xedb88320, ~0 in and out, chainable).  Restated here as
 *              the table-driven form of rdcrc32.h:108-117 / rdcrc32.c (crc_table).  Pinned
 *              by the standard check value and by the system zlib (the library the
 *              reference links) in tests/test_oracle_legacy.py.
 *   writer     rd_kafka_msgset_writer_write_msg_v0_1 rdkafka_msgset_writer.c:583-645
 *   reader     rd_kafka_msgset_reader_msg_v0_1 rdkafka_msgset_reader.c:538-628 (header reads,
 *              hdrsize check, partial-message check, check.crcs)
 * ====================================================================== */
static uint32_t crc32_tab[256];
static int crc32_tab_ok;

static void crc32_tab_init(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t r = b;
    for (int i = 0; i < 8; ++i) r = (r >> 1) ^ ((r & 1u) ? 0xedb88320u : 0u);
    crc32_tab[b] = r;
  }
  crc32_tab_ok = 1;
}

/* zlib crc32(crc, buf, len) */
uint32_t or_crc32(uint32_t crc, const void *buf, size_t len) {
  const uint8_t *p = (const uint8_t *)buf;
  if (!crc32_tab_ok) crc32_tab_init();
  crc = ~crc;
  while (len--) crc = crc32_tab[(crc ^ *p++) & 0xffu] ^ (crc >> 8);
  return ~crc;
}

static uint32_t rd_be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* Messages [first, first+cnt) as one uncompressed MsgVersion `magic` (0 or 1) MessageSet;
 * Offset = base_offset + k (write_msg(..., msgcnt, ...)).  Returns the set size. */
size_t or_msgset_v01_write(const uint8_t *arena, const int64_t *ts, const uint64_t *key_off,
                           const int32_t *key_len, const uint64_t *val_off,
                           const int32_t *val_len, uint32_t first, uint32_t cnt, int magic,
                           int64_t base_offset, int8_t attributes, uint8_t *out) {
  size_t pos = 0;
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t m = first + k;
    const int32_t kl = key_len[m], vl = val_len[m];
    const uint32_t kb = kl > 0 ? (uint32_t)kl : 0, vb = vl > 0 ? (uint32_t)vl : 0;
    const uint32_t size = 4 + 1 + 1 + 4 + kb + 4 + vb + (magic == 1 ? 8 : 0); /* :598-604 */
    uint8_t *p = out + pos;
    be64(p, (uint64_t)(base_offset + k));                 /* Offset :594 */
    be32(p + 8, size);                                    /* MessageSize :606 */
    uint8_t *q = p + 16;
    *q++ = (uint8_t)magic;                                /* MagicByte :620 */
    *q++ = (uint8_t)attributes;                           /* Attributes :623 */
    if (magic == 1) { be64(q, (uint64_t)ts[m]); q += 8; } /* Timestamp :626-627 */
    be32(q, (uint32_t)(kl >= 0 ? kl : -1)); q += 4;       /* Key :630 */
    if (kb) { memcpy(q, arena + key_off[m], kb); q += kb; }
    be32(q, (uint32_t)(vl >= 0 ? vl : -1)); q += 4;       /* Value :633-637 */
    if (vb) { memcpy(q, arena + val_off[m], vb); q += vb; }
    be32(p + 12, or_crc32(0, p + 16, size - 4));          /* Crc :613-616, :639-641 */
    pos += 12 + size;
  }
  return pos;
}

/* The reader's message walk + check.crcs over one MessageSet [0, len):
 *   mode 0 COMPUTE : out[k] = CRC-32 of message k's [16, 12+MessageSize)
 *   mode 1 FINALIZE: also stores it big-endian at the message's Crc field
 *   mode 2 VERIFY  : out[k] = (stored == computed) ? 0 : 1 (the reader continues)
 * pos[k] = message start.  Returns the number of whole messages (a partial message at
 * the end stops the walk, :599-600 / UNDERFLOW), or -(1+k) when message k fails the
 * header checks (MessageSize < hdrsize :590-597; MessageSize < 4, where the reference's
 * rd_slice_narrow_copy asserts) or does not fit in max_rows. */
typedef uint32_t (*crc_fn)(uint32_t, const void *, size_t);

static long v01_walk(uint8_t *set, size_t len, int mode, uint32_t *pos, uint32_t *out,
                     long max_rows, crc_fn crcf) {
  size_t p = 0;
  long k = 0;
  while (p < len) {
    const size_t R = len - p;
    if (R < 16) return k;                          /* Offset, MessageSize, Crc :566-570 */
    const int32_t S = (int32_t)rd_be32(set + p + 8);
    if (S < 4) return -(1 + k);
    if ((size_t)(S - 4) > R - 16) return k;        /* narrow_copy + check_len :571-573 */
    if (R < 18) return k;                          /* MagicByte, Attributes :575-576 */
    size_t hdr = 6;
    if (set[p + 16] == 1) {                        /* Timestamp :578-580 */
      if (R < 26) return k;
      hdr = 14;
    }
    if ((size_t)S < hdr) return -(1 + k);          /* :590-597 */
    if (k >= max_rows) return -(1 + k);
    const uint32_t crc = crcf(0, set + p + 16, (size_t)S - 4);
    pos[k] = (uint32_t)p;
    if (mode == 2) {
      out[k] = rd_be32(set + p + 12) == crc ? 0u : 1u;   /* :602-628 */
    } else {
      out[k] = crc;
      if (mode == 1) be32(set + p + 12, crc);
    }
    p += 12 + (size_t)S;
    ++k;
  }
  return k;
}

long or_msgset_v01_crc(uint8_t *set, size_t len, int mode, uint32_t *pos, uint32_t *out,
                       long max_rows) {
  return v01_walk(set, len, mode, pos, out, max_rows, or_crc32);
}

/* The same walk with the system zlib's crc32() -- the function the reference itself calls
 * (rdcrc32.h WITH_ZLIB): bench.py's CPU baseline ("kind": "reference" for the CRC). */
static uint32_t zlib_crc(uint32_t c, const void *p, size_t n) {
  return (uint32_t)crc32(c, (const Bytef *)p, (uInt)n);
}

long or_msgset_v01_crc_zlib(uint8_t *set, size_t len, int mode, uint32_t *pos, uint32_t *out,
                            long max_rows) {
  return v01_walk(set, len, mode, pos, out, max_rows, zlib_crc);
}
