/*
 * flush_bench.c -- latency of TAS's deferred surface through the C ABI
 * (tasx_tcp_checksums x n + tasx_flush), staged and zero-copy, against the
 * reference per-frame CPU path (the oracle's tcp_checksums restatement) for
 * the same frames.  Measurement tool only: it links the oracle to time the CPU
 * baseline, the product library never does.
 *
 *   gcc -O2 -std=gnu99 -Iinclude -Ioracle tools/flush_bench.c -o tools/bin/flush_bench \
 *       -Ltas_amd/_lib -ltasx -Loracle/build -loracle -Wl,-rpath,$PWD/tas_amd/_lib \
 *       -Wl,-rpath,$PWD/oracle/build
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "tasx_xsum.h"
#include "tasx_oracle.h"

#define STRIDE 2048u

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

/* a TAS data segment (flow_tx_segment layout) with `payload` random bytes */
static void make_frame(uint8_t *f, unsigned payload, uint64_t *rng)
{
  unsigned i, tl = 52 + payload;
  for (i = 0; i < 66 + payload; i++) {
    *rng = *rng * 6364136223846793005ull + 1442695040888963407ull;
    f[i] = (uint8_t) (*rng >> 56);
  }
  f[12] = 0x08; f[13] = 0x00;
  f[14] = 0x45; f[15] = 0;
  f[16] = (uint8_t) (tl >> 8); f[17] = (uint8_t) tl;
  f[22] = 0xff; f[23] = 6;
  f[34 + 12] = 0x80; f[34 + 13] = 0x18;
}

static double median(double *v, int n)
{
  qsort(v, (size_t) n, sizeof(double), cmp_d);
  return v[n / 2];
}

int main(int argc, char **argv)
{
  const unsigned sizes[] = {1, 8, 32, 128, 512, 2048, 8192};
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const unsigned maxn = 8192;
  uint64_t rng = 12345;
  uint8_t *pool = tasx_host_alloc((size_t) maxn * STRIDE);   /* "mempool" */
  uint8_t *plain = malloc((size_t) maxn * STRIDE);
  uint8_t *ref = malloc((size_t) maxn * STRIDE);
  double *t = malloc(sizeof(double) * (size_t) reps);
  unsigned s, i;
  int r;

  if (!pool || !plain || !ref || tasx_ctx_init(0, 0, 32u << 20) || tasx_ctx_init(1, 0, 32u << 20) ||
      tasx_ctx_register_frames(1, pool, (size_t) maxn * STRIDE)) {
    fprintf(stderr, "setup: %s\n", tasx_last_error());
    return 1;
  }
  for (i = 0; i < maxn; i++)
    make_frame(plain + (size_t) i * STRIDE, 1448, &rng);
  memcpy(pool, plain, (size_t) maxn * STRIDE);
  memcpy(ref, plain, (size_t) maxn * STRIDE);
  for (i = 0; i < maxn; i++)
    oracle_tcp_checksums(ref + (size_t) i * STRIDE + 14, ref + (size_t) i * STRIDE + 34);

  for (s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++) {
    const unsigned n = sizes[s];
    double staged, zc, cpu;
    /* staged flush (frames in ordinary memory) */
    for (r = 0; r < reps; r++) {
      double t0 = now_us();
      for (i = 0; i < n; i++)
        tasx_tcp_checksums(0, NULL, plain + (size_t) i * STRIDE, 0, 0, 0);
      if (tasx_flush(0)) {
        fprintf(stderr, "flush: %s\n", tasx_last_error());
        return 1;
      }
      t[r] = now_us() - t0;
    }
    staged = median(t, reps);
    /* zero-copy flush (frames in the registered pool) */
    for (r = 0; r < reps; r++) {
      double t0 = now_us();
      for (i = 0; i < n; i++)
        tasx_tcp_checksums(1, NULL, pool + (size_t) i * STRIDE, 0, 0, 0);
      if (tasx_flush(1)) {
        fprintf(stderr, "flush: %s\n", tasx_last_error());
        return 1;
      }
      t[r] = now_us() - t0;
    }
    zc = median(t, reps);
    /* pipelined: tasx_flush_submit per batch (up to 3 in flight, the 4th
     * submit completes the oldest), one wait at the end -- a core that keeps
     * polling while its batches are on the GPU */
    double pipe;
    {
      const int nb = 64;
      uint32_t tk = 0;
      double t0 = now_us();
      for (r = 0; r < nb; r++) {
        for (i = 0; i < n; i++)
          tasx_tcp_checksums(1, NULL, pool + (size_t) i * STRIDE, 0, 0, 0);
        if (tasx_flush_submit(1, &tk)) {
          fprintf(stderr, "submit: %s\n", tasx_last_error());
          return 1;
        }
      }
      if (tasx_flush_wait(1, tk)) {
        fprintf(stderr, "wait: %s\n", tasx_last_error());
        return 1;
      }
      pipe = (now_us() - t0) / nb;
    }
    /* the reference path on one core: tcp_checksums per frame */
    for (r = 0; r < reps; r++) {
      double t0 = now_us();
      for (i = 0; i < n; i++)
        oracle_tcp_checksums(plain + (size_t) i * STRIDE + 14, plain + (size_t) i * STRIDE + 34);
      t[r] = now_us() - t0;
    }
    cpu = median(t, reps);
    if (memcmp(plain, ref, (size_t) n * STRIDE) || memcmp(pool, ref, (size_t) n * STRIDE)) {
      fprintf(stderr, "MISMATCH at n=%u\n", n);
      return 2;
    }
    printf("{\"frames\": %u, \"staged_flush_us\": %.2f, \"zero_copy_flush_us\": %.2f, "
           "\"zero_copy_pipelined_us_per_flush\": %.2f, \"cpu_1core_us\": %.2f, \"bytes_per_frame\": 1504}\n",
           n, staged, zc, pipe, cpu);
    fflush(stdout);
  }
  {
    uint32_t z = 0, st = 0;
    tasx_ctx_stats(1, &z, &st);
    fprintf(stderr, "zero-copy flushes %u, staged %u\n", z, st);
  }
  tasx_ctx_destroy(0);
  tasx_ctx_destroy(1);
  tasx_host_free(pool);
  return 0;
}
