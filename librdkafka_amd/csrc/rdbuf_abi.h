// rdbuf_abi.h -- binary layout of librdkafka's segmented buffer types, as
// declared in src/rdbuf.h:63-115 (v1.3.0) with TAILQ from <sys/queue.h>
// (src/rdsysqueue.h).  Only the fields the drop-in symbols read are used:
// the slice reader walk of rd_slice_reader0 (src/rdbuf.c:750-779).
#pragma once

#include <cstddef>

extern "C" {

struct rd_segment_s {
  struct {
    struct rd_segment_s *tqe_next;
    struct rd_segment_s **tqe_prev;
  } seg_link;               // TAILQ_ENTRY(rd_segment_s)
  char *seg_p;              // backing store
  size_t seg_of;            // payload length (write position)
  size_t seg_size;
  size_t seg_absof;         // absolute offset of segment start in the buffer
  void (*seg_free)(void *p);
  int seg_flags;
};
typedef struct rd_segment_s rd_segment_t;

struct rd_buf_s;  // never dereferenced by the shim

struct rd_slice_s {
  const struct rd_buf_s *buf;
  const rd_segment_t *seg;  // current read segment, NULL at end
  size_t rof;               // relative read offset in seg
  size_t start;
  size_t end;
};
}

namespace rdk {

// rd_slice_abs_offset / rd_slice_remains (src/rdbuf.h:229, 255-260)
inline size_t slice_abs_offset(const rd_slice_s *s) {
  return s->seg ? s->seg->seg_absof + s->rof : s->end;
}
inline size_t slice_remains(const rd_slice_s *s) { return s->end - slice_abs_offset(s); }

// rd_slice_reader (src/rdbuf.c:750-795): next contiguous run, advancing.
inline size_t slice_reader(rd_slice_s *slice, const void **p) {
  size_t rof = slice->rof;
  const rd_segment_t *seg;
  for (seg = slice->seg; seg && seg->seg_absof + rof < slice->end && seg->seg_of == rof;
       seg = seg->seg_link.tqe_next)
    rof = 0;
  if (!seg || seg->seg_absof + rof >= slice->end) return 0;
  *p = seg->seg_p + rof;
  size_t avail = seg->seg_of - rof, rem = slice_remains(slice);
  size_t rlen = avail < rem ? avail : rem;
  if (slice->seg != seg) {
    slice->seg = seg;
    slice->rof = rlen;
  } else {
    slice->rof += rlen;
  }
  return rlen;
}

}  // namespace rdk
