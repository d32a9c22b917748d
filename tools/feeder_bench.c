/*
 * feeder_bench.c -- tx_flush at TAS's batch size from several fast-path
 * threads, with and without the shared feeder (not a product file; links the
 * C oracle only for the CPU per-frame baseline and the final check).
 *
 * Each thread binds its own context (TASX_CTX_SELF), owns a registered pinned
 * "mempool" of D batch slots of 32 frames (TXBUF_SIZE; half data segments,
 * half pure ACKs), and runs the INTEGRATION.md section 4b loop: record 32
 * frames with tasx_tcp_checksums, tasx_flush_submit, poll the oldest tickets,
 * wait for the oldest only when 3 are in flight (a slot is reused only after
 * its flush completed).  Per mode and thread count, one JSON line:
 *   core_us_per_flush   time inside record + submit + polls per flush (what
 *                       the fast-path core spends), median over flushes
 *   stall_us_per_flush  time blocked in tasx_flush_wait per flush (mean)
 *   latency_us          submit returned -> completion seen by a poll (median)
 *   latency_from_submit_us  the same from the submit call's start (a launch
 *                       per flush pays its launch inside the call)
 *   frames_per_s        all threads' frames / wall time
 *   cpu_core_us_per_flush  the same 32 frames through oracle_tcp_checksums
 *                       on the calling core (TAS's own path)
 *
 *   gcc -O2 -std=gnu99 -pthread -Iinclude -Ioracle tools/feeder_bench.c \
 *       -o tools/bin/feeder_bench -Ltas_amd/_lib -ltasx -Loracle/build -loracle \
 *       -Wl,-rpath,/root/repo/tas_amd/_lib -Wl,-rpath,/root/repo/oracle/build
 *   FB_BATCH=n: n frames per flush (1..32, default 32); FB_MALLOC=1: plain pages
 *   tools/bin/feeder_bench [flushes_per_thread] [in_flight (1..7, default 3)]
 *                          [modes: bit 0 per-context, 1 feeder, 2 server; default 7]
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "tasx_xsum.h"
#include "tasx_oracle.h"

#define STRIDE 2048u
#define BATCH 32u
#define MAXQ 8u   /* in-flight depth limit (the feeder queues 8 batches per context) */
#define MAXT 8

static double now_us(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b)
{
  double x = *(const double *) a, y = *(const double *) b;
  return (x > y) - (x < y);
}

static double median(double *v, int n)
{
  qsort(v, (size_t) n, sizeof(double), cmp_d);
  return v[n / 2];
}

/* frame k of a thread: a data segment (1448 B) or a pure ACK (ip.len 52) */
static void make_frame(uint8_t *f, unsigned k, uint64_t *rng)
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

static unsigned INFLIGHT = 3, DSLOT = 4; /* batch slots: in flight + 1 being recorded */
static unsigned NB = BATCH;              /* frames recorded per flush (FB_BATCH, 1..32) */

struct thr {
  int id, flushes, use_feeder;
  uint8_t *pool;
  double *core, *lat, *lat2;
  double stall;
  int nlat, err;
};

static void *run(void *arg)
{
  struct thr *T = arg;
  uint32_t q[MAXQ];
  double qt[MAXQ], qs[MAXQ];
  unsigned qh = 0, qn = 0;
  if (tasx_set_thread_ctx((unsigned) T->id) != 0) {
    T->err = 1;
    return NULL;
  }
  for (int b = 0; b < T->flushes; b++) {
    uint8_t *slot = T->pool + (size_t) (b % DSLOT) * BATCH * STRIDE;
    /* the slot's previous flush (b - DSLOT) is complete: at most INFLIGHT in flight */
    if (qn >= INFLIGHT) {
      const double w0 = now_us();
      if (tasx_flush_wait(TASX_CTX_SELF, q[qh % MAXQ]) != 0) {
        T->err = 2;
        return NULL;
      }
      const double w1 = now_us();
      T->stall += w1 - w0;
      T->lat2[T->nlat] = w1 - qs[qh % MAXQ];
      T->lat[T->nlat++] = w1 - qt[qh % MAXQ];
      qh++, qn--;
    }
    const double t0 = now_us();
    for (unsigned i = 0; i < NB; i++) {
      uint8_t *f = slot + (size_t) i * STRIDE;
      if (tasx_tcp_checksums(TASX_CTX_SELF, NULL, f, 0, 0, 0) != 0) {
        T->err = 3;
        return NULL;
      }
    }
    uint32_t tk;
    const double tsub = now_us();
    if (tasx_flush_submit(TASX_CTX_SELF, &tk) != 0) {
      T->err = 4;
      return NULL;
    }
    const double ts = now_us();
    q[(qh + qn) % MAXQ] = tk, qt[(qh + qn) % MAXQ] = ts, qs[(qh + qn) % MAXQ] = tsub, qn++;
    while (qn > 0) { /* completions the loop notices without blocking */
      const int r = tasx_flush_poll(TASX_CTX_SELF, q[qh % MAXQ]);
      if (r < 0) {
        T->err = 5;
        return NULL;
      }
      if (r == 0)
        break;
      const double tc = now_us();
      T->lat2[T->nlat] = tc - qs[qh % MAXQ];
      T->lat[T->nlat++] = tc - qt[qh % MAXQ];
      qh++, qn--;
    }
    T->core[b] = now_us() - t0;
  }
  while (qn > 0) {
    if (tasx_flush_wait(TASX_CTX_SELF, q[qh % MAXQ]) != 0) {
      T->err = 6;
      return NULL;
    }
    const double tc = now_us();
    T->lat2[T->nlat] = tc - qs[qh % MAXQ];
    T->lat[T->nlat++] = tc - qt[qh % MAXQ];
    qh++, qn--;
  }
  tasx_set_thread_ctx(TASX_CTX_SELF);
  return NULL;
}

int main(int argc, char **argv)
{
  const int flushes = argc > 1 ? atoi(argv[1]) : 4000;
  INFLIGHT = argc > 2 ? (unsigned) atoi(argv[2]) : 3u;
  if (INFLIGHT < 1 || INFLIGHT > MAXQ - 1)
    INFLIGHT = 3;
  DSLOT = INFLIGHT + 1;
  if (getenv("FB_BATCH")) {
    NB = (unsigned) atoi(getenv("FB_BATCH"));
    if (NB < 1 || NB > BATCH)
      NB = BATCH;
  }
  const int modes = argc > 3 ? atoi(argv[3]) : 7;
  const int nthreads[] = {1, 2, 4, 8};
  const size_t pool_bytes = (size_t) DSLOT * BATCH * STRIDE;
  struct thr T[MAXT];
  uint8_t *ref = malloc(pool_bytes);
  uint64_t rng = 7;
  int bad = 0;

  /* the CPU path: the same 32 frames through TAS's per-frame calls */
  {
    uint8_t *fr = malloc(BATCH * STRIDE);
    double v[2000];
    for (unsigned i = 0; i < BATCH; i++)
      make_frame(fr + (size_t) i * STRIDE, i, &rng);
    for (int r = 0; r < 2000; r++) {
      const double t0 = now_us();
      for (unsigned i = 0; i < BATCH; i++)
        oracle_tcp_checksums(fr + (size_t) i * STRIDE + 14, fr + (size_t) i * STRIDE + 34);
      v[r] = now_us() - t0;
    }
    printf("{\"mode\": \"cpu\", \"cpu_core_us_per_flush\": %.3f, \"frames\": %u}\n", median(v, 2000), BATCH);
    free(fr);
  }

  for (int k = 0; k < MAXT; k++) {
    memset(&T[k], 0, sizeof(T[k]));
    T[k].id = k;
    /* FB_MALLOC=1: plain malloc'd pages, pinned by tasx_ctx_register_frames
     * (hipHostRegister, as TAS's hugepage mempools would be) */
    T[k].pool = getenv("FB_MALLOC") ? aligned_alloc(4096, (pool_bytes + 4095) & ~(size_t) 4095)
                                    : tasx_host_alloc(pool_bytes);
    T[k].core = malloc(sizeof(double) * (size_t) flushes);
    T[k].lat = malloc(sizeof(double) * (size_t) flushes);
    T[k].lat2 = malloc(sizeof(double) * (size_t) flushes);
    uint64_t r2 = 100 + (uint64_t) k;
    for (unsigned i = 0; i < DSLOT * BATCH; i++)
      make_frame(T[k].pool + (size_t) i * STRIDE, i, &r2);
    if (!T[k].pool || tasx_ctx_init((unsigned) k, 0, 4u << 20) != 0 ||
        tasx_ctx_register_frames((unsigned) k, T[k].pool, pool_bytes) != 0) {
      fprintf(stderr, "setup: %s\n", tasx_last_error());
      return 1;
    }
  }
  if (tasx_feeder_start(0) != 0) {
    fprintf(stderr, "feeder: %s\n", tasx_last_error());
    return 1;
  }
  static const char *const mname[3] = {"per_context", "feeder", "server"};
  for (int mode = 0; mode < 3; mode++) {
    if (!(modes & (1 << mode)))
      continue;
    if (mode == 2 && tasx_server_start(0) != 0) {
      fprintf(stderr, "server: %s\n", tasx_last_error());
      return 1;
    }
    for (unsigned ni = 0; ni < sizeof(nthreads) / sizeof(nthreads[0]); ni++) {
      const int n = nthreads[ni];
      pthread_t th[MAXT];
      uint64_t sw0 = 0, sw1 = 0, fr0, fr1;
      for (int k = 0; k < n; k++) {
        T[k].flushes = flushes, T[k].use_feeder = mode, T[k].stall = 0, T[k].nlat = 0, T[k].err = 0;
        if (tasx_ctx_use_feeder((unsigned) k, mode == 1) != 0 || tasx_ctx_use_server((unsigned) k, mode == 2) != 0) {
          fprintf(stderr, "use_feeder / use_server: %s\n", tasx_last_error());
          return 1;
        }
      }
      if (mode == 2)
        tasx_server_stats(0, &sw0, &fr0);
      else
        tasx_feeder_stats(0, &sw0, &fr0);
      const double t0 = now_us();
      for (int k = 0; k < n; k++)
        pthread_create(&th[k], NULL, run, &T[k]);
      for (int k = 0; k < n; k++)
        pthread_join(th[k], NULL);
      const double wall = now_us() - t0;
      if (mode == 2)
        tasx_server_stats(0, &sw1, &fr1);
      else
        tasx_feeder_stats(0, &sw1, &fr1);
      double core_all[MAXT], stall = 0, lat_all[MAXT], lat2_all[MAXT];
      for (int k = 0; k < n; k++) {
        if (T[k].err) {
          fprintf(stderr, "thread %d failed (%d): %s\n", k, T[k].err, tasx_last_error());
          return 1;
        }
        core_all[k] = median(T[k].core, flushes);
        lat_all[k] = median(T[k].lat, T[k].nlat);
        lat2_all[k] = median(T[k].lat2, T[k].nlat);
        stall += T[k].stall / flushes;
      }
      printf("{\"mode\": \"%s\", \"threads\": %d, \"in_flight\": %u, \"flushes_per_thread\": %d, \"frames_per_flush\": %u, "
             "\"core_us_per_flush\": %.3f, \"stall_us_per_flush\": %.3f, \"latency_us\": %.2f, \"latency_from_submit_us\": %.2f, "
             "\"frames_per_s\": %.0f, \"sweeps\": %llu, \"frames_per_sweep\": %.1f}\n",
             mname[mode], n, INFLIGHT, flushes, NB, median(core_all, n), stall / n, median(lat_all, n), median(lat2_all, n),
             (double) n * flushes * NB / (wall * 1e-6), (unsigned long long) (sw1 - sw0),
             sw1 > sw0 ? (double) (fr1 - fr0) / (double) (sw1 - sw0) : 0.0);
      fflush(stdout);
    }
    if (mode == 2) {
      for (int k = 0; k < MAXT; k++)
        tasx_ctx_use_server((unsigned) k, 0);
      if (tasx_server_stop(0) != 0) {
        fprintf(stderr, "server stop: %s\n", tasx_last_error());
        return 1;
      }
    }
  }
  /* every thread's last batches against the oracle */
  for (int k = 0; k < MAXT; k++) {
    memcpy(ref, T[k].pool, pool_bytes);
    for (unsigned i = 0; i < DSLOT * BATCH; i++)
      oracle_tcp_checksums(ref + (size_t) i * STRIDE + 14, ref + (size_t) i * STRIDE + 34);
    if (memcmp(ref, T[k].pool, pool_bytes) != 0)
      bad++;
    tasx_ctx_use_feeder((unsigned) k, 0);
    tasx_ctx_destroy((unsigned) k);
  }
  tasx_feeder_stop(0);
  printf("{\"check\": \"%s\"}\n", bad ? "MISMATCH" : "bit-exact");
  return bad ? 1 : 0;
}
