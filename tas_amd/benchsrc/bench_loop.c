/*
 * bench_loop.c -- launch loops for bench.py (libtasx_bench.so; measurement
 * plumbing, not part of the product library).
 *
 * bench.py's timed region issues K back-to-back launches of one libtasx entry
 * point over R rotating batches.  From Python each launch is a ctypes call
 * (~5-8 us of host time), and the first launch of a timed region then reaches
 * the GPU late.  These loops make the K calls from C, through libtasx's public
 * C ABI exactly as a TAS integration would call it: same entry point, same
 * arguments, one call per step.
 */
#include <stdint.h>
#include <time.h>

#include "tasx_xsum.h"

/* tasx_tcp4_cksum_batch_dev_room / tasx_tcp4_verify_batch_dev_room arguments
 * of one batch */
typedef struct tasxb_tcp4 {
  void *base;
  const uint64_t *off;
  uint64_t stride;
  const uint32_t *flen;
  uint32_t flen0;
  uint32_t room;
  uint32_t n;
  uint32_t ip_off;
  uint32_t l4_off;
  uint32_t flags;
  void *out; /* uint16_t results (TX) or uint8_t flags (verify) */
} tasxb_tcp4;

/* entry-point selector for tasxb_tcp4_loop */
enum { TASXB_DEV = 0, TASXB_HINT = 1, TASXB_ROOM = 2, TASXB_VERIFY = 3 };

static int tcp4_call(int which, const tasxb_tcp4 *a, void *stream)
{
  switch (which) {
  case TASXB_DEV:
    return tasx_tcp4_cksum_batch_dev(a->base, a->off, a->stride, a->n, a->ip_off, a->l4_off,
        (uint16_t *) a->out, a->flags, stream);
  case TASXB_HINT:
    return tasx_tcp4_cksum_batch_dev_hint(a->base, a->off, a->stride, a->flen, a->flen0, a->n,
        a->ip_off, a->l4_off, (uint16_t *) a->out, a->flags, stream);
  case TASXB_ROOM:
    return tasx_tcp4_cksum_batch_dev_room(a->base, a->off, a->stride, a->flen, a->flen0, a->room,
        a->n, a->ip_off, a->l4_off, (uint16_t *) a->out, a->flags, stream);
  default:
    return tasx_tcp4_verify_batch_dev_room(a->base, a->off, a->stride, a->flen, a->flen0, a->room,
        a->n, a->ip_off, a->l4_off, (uint8_t *) a->out, stream);
  }
}

/* launch batches a[(first + k) % R] for k < K, batch k on streams[(first + k)
 * % S] (S fast-path contexts with a stream each); 0 or the first error */
int tasxb_tcp4_loop(int which, const tasxb_tcp4 *a, int R, int first, int K, void *const *streams, int S)
{
  for (int k = 0; k < K; k++) {
    int rc = tcp4_call(which, &a[(first + k) % R], streams[(first + k) % S]);
    if (rc)
      return rc;
  }
  return 0;
}

typedef struct tasxb_raw {
  const void *base;
  const uint64_t *off;
  uint64_t stride;
  const uint32_t *len;
  uint32_t len0;
  uint32_t n;
  uint16_t *out;
} tasxb_raw;

int tasxb_raw_loop(const tasxb_raw *a, int R, int first, int K, void *const *streams, int S)
{
  for (int k = 0; k < K; k++) {
    const tasxb_raw *b = &a[(first + k) % R];
    int rc = tasx_raw_cksum_batch_dev(b->base, b->off, b->stride, b->len, b->len0, b->n, b->out, streams[(first + k) % S]);
    if (rc)
      return rc;
  }
  return 0;
}

typedef struct tasxb_txseg {
  const void *shm;
  uint64_t shm_len;
  void *frames;
  const tasx_tx_seg *segs;
  uint32_t n;
  uint32_t ip_off;
  uint32_t l4_off;
  uint32_t *out;
} tasxb_txseg;

int tasxb_txseg_loop(const tasxb_txseg *a, int R, int first, int K, void *const *streams, int S)
{
  for (int k = 0; k < K; k++) {
    const tasxb_txseg *b = &a[(first + k) % R];
    int rc = tasx_tx_segment_batch_dev(b->shm, b->shm_len, b->frames, b->segs, b->n, b->ip_off,
        b->l4_off, b->out, streams[(first + k) % S]);
    if (rc)
      return rc;
  }
  return 0;
}

typedef struct tasxb_flow {
  const void *base;
  const uint64_t *off;
  uint64_t stride;
  uint32_t n;
  uint32_t ip_off;
  uint32_t l4_off;
  const void *flowht;
  uint32_t ht_entries;
  const void *flowst;
  uint32_t fs_num;
  uint32_t fs_stride;
  uint32_t fs_key_off;
  uint32_t *hash_out;
  uint32_t *fid_out;
} tasxb_flow;

int tasxb_flow_loop(const tasxb_flow *a, int R, int first, int K, void *const *streams, int S)
{
  for (int k = 0; k < K; k++) {
    const tasxb_flow *b = &a[(first + k) % R];
    int rc = tasx_flow_lookup_batch_dev(b->base, b->off, b->stride, b->n, b->ip_off, b->l4_off,
        b->flowht, b->ht_entries, b->flowst, b->fs_num, b->fs_stride, b->fs_key_off, b->hash_out,
        b->fid_out, streams[(first + k) % S]);
    if (rc)
      return rc;
  }
  return 0;
}

/* one RX pass: tasx_rx_batch_dev (which = 0), or the two calls it replaces in
 * turn, tasx_tcp4_verify_batch_dev_room then tasx_flow_lookup_batch_dev
 * (which = 1), over the same frames and outputs */
typedef struct tasxb_rx {
  tasxb_tcp4 v;     /* verify arguments (out = uint8_t flags) */
  tasxb_flow f;     /* lookup arguments (base/off/stride/n/ip_off/l4_off as v's) */
} tasxb_rx;

int tasxb_rx_loop(int which, const tasxb_rx *a, int R, int first, int K, void *const *streams, int S)
{
  for (int k = 0; k < K; k++) {
    const tasxb_rx *b = &a[(first + k) % R];
    void *s = streams[(first + k) % S];
    const tasxb_tcp4 *v = &b->v;
    const tasxb_flow *f = &b->f;
    int rc;
    if (which == 0) {
      rc = tasx_rx_batch_dev(v->base, v->off, v->stride, v->flen, v->flen0, v->room, v->n, v->ip_off,
          v->l4_off, (uint8_t *) v->out, f->flowht, f->ht_entries, f->flowst, f->fs_num, f->fs_stride,
          f->fs_key_off, f->hash_out, f->fid_out, s);
    } else {
      rc = tcp4_call(TASXB_VERIFY, v, s);
      if (!rc)
        rc = tasx_flow_lookup_batch_dev(f->base, f->off, f->stride, f->n, f->ip_off, f->l4_off, f->flowht,
            f->ht_entries, f->flowst, f->fs_num, f->fs_stride, f->fs_key_off, f->hash_out, f->fid_out, s);
    }
    if (rc)
      return rc;
  }
  return 0;
}

/* tx_flush at TAS's batch size from C (the fast-path core's view): `iters`
 * synchronous flushes of the n frames at base + i * stride -- n x
 * tasx_defer_tcp4 (the deferred tcp_checksums), tasx_flush_submit,
 * tasx_flush_wait -- on context ctx, whatever it is attached to (nothing: its
 * own launches; the feeder; the flush server).  us[k] = record + submit + wait
 * of flush k (CLOCK_MONOTONIC).  0 or the first error. */
static double tasxb_now_us(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

int tasxb_flush_loop(unsigned ctx, uint8_t *base, uint64_t stride, uint32_t n, int iters, double *us)
{
  for (int k = 0; k < iters; k++) {
    const double t0 = tasxb_now_us();
    for (uint32_t i = 0; i < n; i++) {
      int rc = tasx_defer_tcp4(ctx, base + (uint64_t) i * stride, TASX_TAS_IP_OFF, TASX_TAS_L4_OFF);
      if (rc)
        return rc;
    }
    uint32_t t;
    int rc = tasx_flush_submit(ctx, &t);
    if (rc == 0)
      rc = tasx_flush_wait(ctx, t);
    if (rc)
      return rc;
    us[k] = tasxb_now_us() - t0;
  }
  return 0;
}
