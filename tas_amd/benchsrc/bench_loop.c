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
#define _GNU_SOURCE
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

/* ---------------------------------------------------------------------- */
/* Several fast-path threads at TAS's batch size (bench.py's `fastpath_mt`
 * line; the same loop as tools/feeder_bench.c, without its oracle check):
 * thread k binds context ctx0 + k (initialised here), owns a pinned mempool of
 * slots of 32 frames at a 2 KiB stride (half 1514-B data segments, half 66-B
 * ACKs), and runs the INTEGRATION.md section 4b loop: record 32 frames with
 * tasx_tcp_checksums, tasx_flush_submit, poll the oldest tickets, wait for
 * the oldest when `inflight` are out (a slot is reused only after its flush
 * completed).  mode 0: each context launches its own flushes; 1: the shared
 * feeder; 2: the persistent flush server.
 *   out[0] frames/s over all threads (wall time from a common start)
 *   out[1] median latency, submit returned -> completion seen (us)
 *   out[2] median latency from the submit call's start (us)
 *   out[3] median core time per flush: record + submit + polls (us)
 * keep (optional, keep_bytes): thread 0's mempool after the run, for the
 * caller's check against the device kernel. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MT_BATCH 32u
#define MT_STRIDE 2048u
#define MT_MAXQ 8u
#define MT_MAXT 16

struct mt_thr {
  unsigned ctx, nslot, inflight;
  const tasx_tx_seg *segs; /* TX segment mode: MT_BATCH descriptors per slot */
  int inited; /* tasx_ctx_init succeeded: destroyed at the end */
  uint8_t *pool;
  int flushes, n, err;
  double *lat, *lat2, *core;
  const int *go; /* 1: start, 2: leave at once */
};

static void mt_frame(uint8_t *f, unsigned k, uint64_t *rng)
{
  const unsigned payload = (k & 1) ? 0 : 1448, tl = 52 + payload;
  for (unsigned i = 0; i < 66 + payload; i++) {
    *rng = *rng * 6364136223846793005ull + 1442695040888963407ull;
    f[i] = (uint8_t) (*rng >> 56);
  }
  f[12] = 0x08, f[13] = 0x00, f[14] = 0x45, f[15] = 0;
  f[16] = (uint8_t) (tl >> 8), f[17] = (uint8_t) tl;
  f[22] = 0xff, f[23] = 6;
  f[34 + 12] = 0x80, f[34 + 13] = 0x18;
}

static void *mt_worker(void *arg)
{
  struct mt_thr *T = arg;
  uint32_t q[MT_MAXQ];
  double qt[MT_MAXQ], qs[MT_MAXQ];
  unsigned qh = 0, qn = 0;
  if (tasx_set_thread_ctx(T->ctx) != 0)
    T->err = 1;
  int g;
  while ((g = __atomic_load_n(T->go, __ATOMIC_ACQUIRE)) == 0)
    ;
  if (g != 1)
    T->err = 7;
  for (int b = 0; b < T->flushes && !T->err; b++) {
    uint8_t *slot = T->pool + (size_t) (b % T->nslot) * MT_BATCH * MT_STRIDE;
    if (qn >= T->inflight) {
      if (tasx_flush_wait(TASX_CTX_SELF, q[qh % MT_MAXQ]) != 0) {
        T->err = 2;
        break;
      }
      const double w1 = tasxb_now_us();
      T->lat2[T->n] = w1 - qs[qh % MT_MAXQ];
      T->lat[T->n++] = w1 - qt[qh % MT_MAXQ];
      qh++, qn--;
    }
    const double t0 = tasxb_now_us();
    uint32_t tk;
    double tsub;
    if (T->segs) { /* the whole batch's build (payload copy + checksums) to the server */
      tsub = t0;
      if (tasx_server_tx_segments(TASX_CTX_SELF, T->segs + (size_t) (b % T->nslot) * MT_BATCH, MT_BATCH, &tk) != 0) {
        T->err = 8;
        break;
      }
    } else {
      for (unsigned i = 0; i < MT_BATCH && !T->err; i++)
        if (tasx_tcp_checksums(TASX_CTX_SELF, NULL, slot + (size_t) i * MT_STRIDE, 0, 0, 0) != 0)
          T->err = 3;
      tsub = tasxb_now_us();
      if (T->err || tasx_flush_submit(TASX_CTX_SELF, &tk) != 0) {
        T->err = T->err ? T->err : 4;
        break;
      }
    }
    const double ts = tasxb_now_us();
    q[(qh + qn) % MT_MAXQ] = tk, qt[(qh + qn) % MT_MAXQ] = ts, qs[(qh + qn) % MT_MAXQ] = tsub, qn++;
    while (qn > 0) {
      const int r = tasx_flush_poll(TASX_CTX_SELF, q[qh % MT_MAXQ]);
      if (r < 0)
        T->err = 5;
      if (r <= 0)
        break;
      const double tc = tasxb_now_us();
      T->lat2[T->n] = tc - qs[qh % MT_MAXQ];
      T->lat[T->n++] = tc - qt[qh % MT_MAXQ];
      qh++, qn--;
    }
    T->core[b] = tasxb_now_us() - t0;
  }
  while (qn > 0 && !T->err) {
    if (tasx_flush_wait(TASX_CTX_SELF, q[qh % MT_MAXQ]) != 0) {
      T->err = 6;
      break;
    }
    const double tc = tasxb_now_us();
    T->lat2[T->n] = tc - qs[qh % MT_MAXQ];
    T->lat[T->n++] = tc - qt[qh % MT_MAXQ];
    qh++, qn--;
  }
  tasx_set_thread_ctx(TASX_CTX_SELF);
  return NULL;
}

static int mt_cmp(const void *a, const void *b)
{
  const double x = *(const double *) a, y = *(const double *) b;
  return (x > y) - (x < y);
}

static double mt_median(double *v, size_t n)
{
  if (n == 0)
    return 0.0;
  qsort(v, n, sizeof(double), mt_cmp);
  return v[n / 2];
}

int tasxb_fastpath_mt(int device, unsigned ctx0, int threads, unsigned inflight, int flushes, int mode,
                      double *out, uint8_t *keep, size_t keep_bytes)
{
  if (threads < 1 || threads > MT_MAXT || inflight < 1 || inflight > MT_MAXQ - 1 || flushes < 1 || mode < 0 ||
      mode > 2 || ctx0 + (unsigned) threads > TASX_MAX_CTX)
    return -22; /* -EINVAL */
  struct mt_thr T[MT_MAXT];
  pthread_t th[MT_MAXT];
  int go = 0;
  const unsigned nslot = inflight + 1;
  const size_t pool_bytes = (size_t) nslot * MT_BATCH * MT_STRIDE;
  int rc = 0, started = 0;
  memset(T, 0, sizeof(T));
  for (int k = 0; k < threads && !rc; k++) {
    T[k].ctx = ctx0 + (unsigned) k, T[k].nslot = nslot, T[k].inflight = inflight, T[k].flushes = flushes;
    T[k].pool = tasx_host_alloc(pool_bytes);
    T[k].lat = malloc(sizeof(double) * (size_t) flushes);
    T[k].lat2 = malloc(sizeof(double) * (size_t) flushes);
    T[k].core = malloc(sizeof(double) * (size_t) flushes);
    if (!T[k].pool || !T[k].lat || !T[k].lat2 || !T[k].core) {
      rc = -12; /* -ENOMEM */
      break;
    }
    uint64_t r = 100 + (uint64_t) k;
    memset(T[k].pool, 0, pool_bytes);
    for (unsigned i = 0; i < nslot * MT_BATCH; i++)
      mt_frame(T[k].pool + (size_t) i * MT_STRIDE, i, &r);
    if ((rc = tasx_ctx_init(T[k].ctx, device, 4u << 20)) != 0)
      break;
    T[k].inited = 1;
    if ((rc = tasx_ctx_register_frames(T[k].ctx, T[k].pool, pool_bytes)) != 0)
      break;
  }
  if (!rc && mode == 1 && (rc = tasx_feeder_start(device)) == 0)
    started = 1;
  if (!rc && mode == 2 && (rc = tasx_server_start(device)) == 0)
    started = 2;
  for (int k = 0; k < threads && !rc; k++)
    rc = mode == 1 ? tasx_ctx_use_feeder(T[k].ctx, 1) : mode == 2 ? tasx_ctx_use_server(T[k].ctx, 1) : 0;
  double wall = 0.0;
  if (!rc) {
    int k;
    for (k = 0; k < threads; k++) {
      T[k].go = &go;
      if (pthread_create(&th[k], NULL, mt_worker, &T[k]) != 0)
        break;
    }
    const double t0 = tasxb_now_us();
    __atomic_store_n(&go, k == threads ? 1 : 2, __ATOMIC_RELEASE); /* 2: the created ones leave */
    for (int j = 0; j < k; j++)
      pthread_join(th[j], NULL);
    wall = tasxb_now_us() - t0;
    if (k < threads)
      rc = -11; /* -EAGAIN */
  }
  for (int k = 0; k < threads && !rc; k++)
    if (T[k].err)
      rc = -1000 - T[k].err;
  if (!rc) {
    size_t total = 0;
    for (int k = 0; k < threads; k++)
      total += (size_t) T[k].n;
    double *all = malloc(sizeof(double) * total), *all2 = malloc(sizeof(double) * total),
           *core = malloc(sizeof(double) * (size_t) threads * (size_t) flushes);
    if (all && all2 && core) {
      size_t o = 0;
      for (int k = 0; k < threads; k++) {
        memcpy(all + o, T[k].lat, sizeof(double) * (size_t) T[k].n);
        memcpy(all2 + o, T[k].lat2, sizeof(double) * (size_t) T[k].n);
        memcpy(core + (size_t) k * flushes, T[k].core, sizeof(double) * (size_t) flushes);
        o += (size_t) T[k].n;
      }
      out[0] = (double) threads * flushes * MT_BATCH / (wall * 1e-6);
      out[1] = mt_median(all, total);
      out[2] = mt_median(all2, total);
      out[3] = mt_median(core, (size_t) threads * (size_t) flushes);
    } else {
      rc = -12;
    }
    free(all);
    free(all2);
    free(core);
    if (keep && T[0].pool)
      memcpy(keep, T[0].pool, keep_bytes < pool_bytes ? keep_bytes : pool_bytes);
  }
  for (int k = 0; k < threads; k++) {
    if (mode == 1 && T[k].inited)
      tasx_ctx_use_feeder(T[k].ctx, 0);
    if (mode == 2 && T[k].inited)
      tasx_ctx_use_server(T[k].ctx, 0);
  }
  if (started == 1)
    tasx_feeder_stop(device);
  if (started == 2)
    tasx_server_stop(device);
  for (int k = 0; k < threads; k++) { /* only what this call set up */
    if (T[k].inited)
      tasx_ctx_destroy(T[k].ctx);
    if (T[k].pool)
      tasx_host_free(T[k].pool);
    free(T[k].lat);
    free(T[k].lat2);
    free(T[k].core);
  }
  return rc;
}

/* The fused TX segment build through the flush server from several fast-path
 * threads (bench.py's `txseg_server_mt`): thread k on context ctx0 + k, a
 * pinned mbuf pool of slots of 32 frames (headers filled: 1514-B data
 * segments) and a pinned shared-memory region of 32 flows' 16 KiB circular TX
 * buffers; per flush tasx_server_tx_segments(32 descriptors) -- payload copy
 * and both checksums on the GPU over PCIe -- then the polls and waits of the
 * loop above.  out[] as tasxb_fastpath_mt (out[0] in segments/s, out[2] =
 * out[1]: the submit call is the whole hand-over). */
#define MT_FLOWS 32u
#define MT_TXLEN 16384u

int tasxb_txseg_server_mt(int device, unsigned ctx0, int threads, unsigned inflight, int flushes, double *out)
{
  if (threads < 1 || threads > MT_MAXT || inflight < 1 || inflight > MT_MAXQ - 1 || flushes < 1 ||
      ctx0 + (unsigned) threads > TASX_MAX_CTX)
    return -22;
  struct mt_thr T[MT_MAXT];
  uint8_t *shm[MT_MAXT];
  tasx_tx_seg *segs[MT_MAXT];
  pthread_t th[MT_MAXT];
  int go = 0, rc = 0, started = 0;
  const unsigned nslot = inflight + 1;
  const size_t pool_bytes = (size_t) nslot * MT_BATCH * MT_STRIDE, shm_bytes = (size_t) MT_FLOWS * MT_TXLEN;
  memset(T, 0, sizeof(T));
  memset(shm, 0, sizeof(shm));
  memset(segs, 0, sizeof(segs));
  for (int k = 0; k < threads && !rc; k++) {
    T[k].ctx = ctx0 + (unsigned) k, T[k].nslot = nslot, T[k].inflight = inflight, T[k].flushes = flushes;
    T[k].pool = tasx_host_alloc(pool_bytes);
    shm[k] = tasx_host_alloc(shm_bytes);
    segs[k] = malloc(sizeof(tasx_tx_seg) * nslot * MT_BATCH);
    T[k].lat = malloc(sizeof(double) * (size_t) flushes);
    T[k].lat2 = malloc(sizeof(double) * (size_t) flushes);
    T[k].core = malloc(sizeof(double) * (size_t) flushes);
    if (!T[k].pool || !shm[k] || !segs[k] || !T[k].lat || !T[k].lat2 || !T[k].core) {
      rc = -12;
      break;
    }
    uint64_t r = 300 + (uint64_t) k;
    memset(T[k].pool, 0, pool_bytes);
    for (unsigned i = 0; i < nslot * MT_BATCH; i++) /* headers (the payload bytes are the build's) */
      mt_frame(T[k].pool + (size_t) i * MT_STRIDE, 0, &r);
    for (size_t i = 0; i < shm_bytes; i++) {
      r = r * 6364136223846793005ull + 1442695040888963407ull;
      shm[k][i] = (uint8_t) (r >> 56);
    }
    for (unsigned i = 0; i < nslot * MT_BATCH; i++) {
      tasx_tx_seg *g = &segs[k][i];
      g->frame_off = (uint64_t) i * MT_STRIDE;
      g->tx_base = (uint64_t) (i % MT_FLOWS) * MT_TXLEN;
      g->tx_len = MT_TXLEN;
      g->pos = (i * 1448u + 77u * (i / MT_FLOWS)) % MT_TXLEN; /* wraps included */
      g->payload = 1448;
      g->hdrs_len = 66;
      g->room = MT_STRIDE;
    }
    T[k].segs = segs[k];
    if ((rc = tasx_ctx_init(T[k].ctx, device, 4u << 20)) != 0)
      break;
    T[k].inited = 1;
    if ((rc = tasx_ctx_register_frames(T[k].ctx, T[k].pool, pool_bytes)) != 0 ||
        (rc = tasx_ctx_register_shm(T[k].ctx, shm[k], shm_bytes)) != 0)
      break;
  }
  if (!rc && (rc = tasx_server_start(device)) == 0)
    started = 1;
  for (int k = 0; k < threads && !rc; k++)
    rc = tasx_ctx_use_server(T[k].ctx, 1);
  double wall = 0.0;
  if (!rc) {
    int k;
    for (k = 0; k < threads; k++) {
      T[k].go = &go;
      if (pthread_create(&th[k], NULL, mt_worker, &T[k]) != 0)
        break;
    }
    const double t0 = tasxb_now_us();
    __atomic_store_n(&go, k == threads ? 1 : 2, __ATOMIC_RELEASE);
    for (int j = 0; j < k; j++)
      pthread_join(th[j], NULL);
    wall = tasxb_now_us() - t0;
    if (k < threads)
      rc = -11;
  }
  for (int k = 0; k < threads && !rc; k++)
    if (T[k].err)
      rc = -1000 - T[k].err;
  if (!rc) {
    size_t total = 0;
    for (int k = 0; k < threads; k++)
      total += (size_t) T[k].n;
    double *all = malloc(sizeof(double) * total), *core = malloc(sizeof(double) * (size_t) threads * flushes);
    if (all && core) {
      size_t o = 0;
      for (int k = 0; k < threads; k++) {
        memcpy(all + o, T[k].lat, sizeof(double) * (size_t) T[k].n);
        memcpy(core + (size_t) k * flushes, T[k].core, sizeof(double) * (size_t) flushes);
        o += (size_t) T[k].n;
      }
      out[0] = (double) threads * flushes * MT_BATCH / (wall * 1e-6);
      out[1] = out[2] = mt_median(all, total);
      out[3] = mt_median(core, (size_t) threads * (size_t) flushes);
    } else {
      rc = -12;
    }
    free(all);
    free(core);
  }
  for (int k = 0; k < threads; k++)
    if (T[k].inited)
      tasx_ctx_use_server(T[k].ctx, 0);
  if (started)
    tasx_server_stop(device);
  for (int k = 0; k < threads; k++) {
    if (T[k].inited)
      tasx_ctx_destroy(T[k].ctx);
    if (T[k].pool)
      tasx_host_free(T[k].pool);
    if (shm[k])
      tasx_host_free(shm[k]);
    free(segs[k]);
    free(T[k].lat);
    free(T[k].lat2);
    free(T[k].core);
  }
  return rc;
}
