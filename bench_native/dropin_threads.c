/* dropin_threads.c -- BENCH/TEST INFRASTRUCTURE: N pthreads calling one drop-in symbol in a
 * loop, as librdkafka's broker threads do (rdkafka_broker.c:5082).  The symbol comes in as a
 * function pointer, so this file links against nothing but libc/pthread.  Python threads
 * cannot stand in for it: the interpreter lock serialises the call overhead at the
 * microsecond scale that is being measured.
 *
 * which: 0 crc32c(0, buf, len)            1 rd_slice_crc32c(slice over buf)
 *        2 rd_kafka_lz4_compress(slice)   3 rd_kafka_lz4_decompress(buf = a frame)
 * Returns microseconds of wall time per call (all threads' calls counted), < 0 on a wrong
 * result: every CRC is compared with `expect_crc`, every LZ4 output length with `expect_len`. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

struct seg { /* rd_segment_t, src/rdbuf.h:63-79 */
  struct { struct seg *next; struct seg **prev; } link;
  char *p; size_t of, size, absof; void (*free_cb)(void *); int flags;
};
struct slice { /* rd_slice_t, src/rdbuf.h:107-115 */
  const void *buf; const struct seg *seg; size_t rof, start, end;
};

typedef uint32_t (*crc_fn)(uint32_t, const void *, size_t);
typedef uint32_t (*slice_crc_fn)(struct slice *);
typedef int (*lz4c_fn)(void *, int, int, struct slice *, void **, size_t *);
typedef int (*lz4d_fn)(void *, int, int64_t, char *, size_t, void **, size_t *);

struct job {
  int which; void *fn; char *buf; size_t len; double seconds;
  uint32_t expect_crc; size_t expect_len;
  volatile int *go; uint64_t calls; int bad;
};

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void one(struct job *j, struct seg *sg, struct slice *sl) {
  void *out = NULL;
  size_t outlen = 0;
  sl->seg = sg; sl->rof = 0;
  switch (j->which) {
    case 0: if (((crc_fn)j->fn)(0, j->buf, j->len) != j->expect_crc) j->bad = 1; break;
    case 1: if (((slice_crc_fn)j->fn)(sl) != j->expect_crc) j->bad = 1; break;
    case 2:
      if (((lz4c_fn)j->fn)(NULL, 1, 0, sl, &out, &outlen) || outlen != j->expect_len) j->bad = 1;
      free(out);
      break;
    default:
      if (((lz4d_fn)j->fn)(NULL, 1, 0, j->buf, j->len, &out, &outlen) || outlen != j->expect_len) j->bad = 1;
      free(out);
      break;
  }
}

static void *run(void *arg) {
  struct job *j = arg;
  struct seg sg;
  struct slice sl;
  memset(&sg, 0, sizeof sg);
  sg.p = j->buf; sg.of = sg.size = j->len;
  sl.buf = NULL; sl.start = 0; sl.end = j->len;
  one(j, &sg, &sl); /* the thread's context, staging and first-touch costs: untimed */
  __sync_fetch_and_add(j->go, 1);
  while (*j->go >= 0) { /* start together: go turns negative */
  }
  const double until = now() + j->seconds;
  do {
    one(j, &sg, &sl);
    j->calls++;
  } while (!j->bad && now() < until);
  return NULL;
}

double dropin_threads_run(int which, void *fn, char *buf, size_t len, uint32_t expect_crc, size_t expect_len,
                          int threads, double seconds) {
  pthread_t th[64];
  struct job jobs[64];
  volatile int go = 0;
  if (threads < 1 || threads > 64) return -2.0;
  for (int t = 0; t < threads; ++t) {
    struct job j = {which, fn, buf, len, seconds, expect_crc, expect_len, &go, 0, 0};
    jobs[t] = j;
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  while (go < threads) {
  }
  const double t0 = now();
  go = -1;
  uint64_t calls = 0;
  int bad = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    calls += jobs[t].calls;
    bad |= jobs[t].bad;
  }
  const double el = now() - t0;
  if (bad || !calls) return -1.0;
  return el * 1e6 / (double)calls;
}
