/*
 * tasx_oracle.c -- TEST INFRASTRUCTURE ONLY (see tasx_oracle.h for the rules
 * and the parity status).  CPU restatement of:
 *   - DPDK 19.11 lib/librte_net/rte_ip.h: __rte_raw_cksum, __rte_raw_cksum_reduce,
 *     rte_raw_cksum, rte_ipv4_cksum, rte_ipv4_phdr_cksum, rte_ipv4_udptcp_cksum
 *     (third-party, not vendored in the reference; restated from the published
 *     algorithm);
 *   - TAS tcp_checksums() flag-off branch, tas/fast/fast_flows.c:1058-1069;
 *   - TAS network_ip_phdr_xsum(), tas/fast/network.h:157-173.
 * Compiled with the reference's flags (-std=gnu99 -O3 -march=native,
 * /root/reference/Makefile:8).  Host is little-endian x86: every "u16 word" is
 * a native LE load of two consecutive bytes counted from the buffer start.
 */
#define _GNU_SOURCE
#include "tasx_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static inline uint16_t ld16(const uint8_t *p)
{
  uint16_t v;
  memcpy(&v, p, 2); /* the may_alias u16 load of rte_ip.h */
  return v;
}

/* a1: __rte_raw_cksum.  4-word unrolled loop, 1-word loop, odd tail byte
 * added as the low byte of a zero-padded LE word.  32-bit accumulator. */
uint32_t oracle_raw_cksum_acc(const void *buf, size_t len, uint32_t sum)
{
  const uint8_t *b = (const uint8_t *) buf;

  while (len >= 8) {
    sum += ld16(b);
    sum += ld16(b + 2);
    sum += ld16(b + 4);
    sum += ld16(b + 6);
    len -= 8;
    b += 8;
  }
  while (len >= 2) {
    sum += ld16(b);
    len -= 2;
    b += 2;
  }
  if (len == 1)
    sum += *b;
  return sum;
}

/* __rte_raw_cksum_reduce: two end-around folds, no inversion. */
uint16_t oracle_raw_cksum_reduce(uint32_t sum)
{
  sum = ((sum & 0xffff0000u) >> 16) + (sum & 0xffffu);
  sum = ((sum & 0xffff0000u) >> 16) + (sum & 0xffffu);
  return (uint16_t) sum;
}

/* a2: rte_raw_cksum */
uint16_t oracle_raw_cksum(const void *buf, size_t len)
{
  return oracle_raw_cksum_reduce(oracle_raw_cksum_acc(buf, len, 0));
}

/* a3: rte_ipv4_cksum -- fixed 20-byte header, 0xffff kept, else inverted. */
uint16_t oracle_ipv4_cksum(const void *ip_hdr)
{
  uint16_t c = oracle_raw_cksum(ip_hdr, 20);
  return (c == 0xffff) ? c : (uint16_t) ~c;
}

/* a4: rte_ipv4_phdr_cksum.  12-byte pseudo header {src, dst, 0, proto,
 * htons(total_length - 20)}; length 0 under PKT_TX_TCP_SEG. */
uint16_t oracle_ipv4_phdr_cksum(const void *ip_hdr, uint64_t ol_flags)
{
  const uint8_t *ip = (const uint8_t *) ip_hdr;
  uint8_t psd[12];
  uint16_t tl = (uint16_t) ((ip[2] << 8) | ip[3]);
  uint16_t l4 = (uint16_t) (tl - 20);

  memcpy(psd, ip + 12, 4);      /* src_addr */
  memcpy(psd + 4, ip + 16, 4);  /* dst_addr */
  psd[8] = 0;                   /* zero */
  psd[9] = ip[9];               /* proto (next_proto_id) */
  if (ol_flags & ORACLE_PKT_TX_TCP_SEG) {
    psd[10] = 0;
    psd[11] = 0;
  } else {
    psd[10] = (uint8_t) (l4 >> 8); /* rte_cpu_to_be_16 */
    psd[11] = (uint8_t) l4;
  }
  return oracle_raw_cksum(psd, sizeof(psd));
}

/* a5: rte_ipv4_udptcp_cksum, DPDK 19.11 semantics: l3 < 20 -> 0; L4 length
 * from ip.total_length; one fold; invert; 0 -> 0xffff. */
uint16_t oracle_ipv4_udptcp_cksum(const void *ip_hdr, const void *l4_hdr)
{
  const uint8_t *ip = (const uint8_t *) ip_hdr;
  uint32_t l3_len = (uint32_t) ((ip[2] << 8) | ip[3]);
  uint32_t cksum;

  if (l3_len < 20)
    return 0;
  cksum = oracle_raw_cksum(l4_hdr, l3_len - 20);
  cksum += oracle_ipv4_phdr_cksum(ip_hdr, 0);
  cksum = ((cksum & 0xffff0000u) >> 16) + (cksum & 0xffffu);
  cksum = (~cksum) & 0xffffu;
  if (cksum == 0)
    cksum = 0xffff;
  return (uint16_t) cksum;
}

/* a6: tcp_checksums(), fp_xsumoffload == 0 branch (fast_flows.c:1061-1067).
 * Order as in the reference: ip.chksum = 0; tcp.chksum = 0; ip.chksum =
 * a3(ip); tcp.chksum = a5(ip, tcp).  Stores are native (LE) u16. */
void oracle_tcp_checksums(void *ip_hdr, void *l4_hdr)
{
  uint8_t *ip = (uint8_t *) ip_hdr;
  uint8_t *tcp = (uint8_t *) l4_hdr;
  uint16_t v;

  memset(ip + 10, 0, 2);
  memset(tcp + 16, 0, 2);
  v = oracle_ipv4_cksum(ip);
  memcpy(ip + 10, &v, 2);
  v = oracle_ipv4_udptcp_cksum(ip, tcp);
  memcpy(tcp + 16, &v, 2);
}

/* a8: network_ip_phdr_xsum (offload branch's pseudo-header fold).  The
 * beui32 .x fields hold network-order bytes read as a native LE u32. */
uint16_t oracle_ip_phdr_xsum(uint32_t ip_src_be, uint32_t ip_dst_be,
    uint8_t proto, uint16_t l3_paylen)
{
  uint32_t sum = 0;
  sum += ip_src_be & 0xffff;
  sum += (ip_src_be >> 16) & 0xffff;
  sum += ip_dst_be & 0xffff;
  sum += (ip_dst_be >> 16) & 0xffff;
  sum += ((uint16_t) proto) << 8;
  sum += (uint16_t) __builtin_bswap16(l3_paylen); /* t_beui16(l3_paylen).x */
  sum = ((sum & 0xffff0000u) >> 16) + (sum & 0xffffu);
  sum = ((sum & 0xffff0000u) >> 16) + (sum & 0xffffu);
  return (uint16_t) sum;
}

/* Receive-side verification (new behaviour; see tasx_oracle.h). */
int oracle_ipv4_hdr_verify(const void *ip_hdr)
{
  return oracle_raw_cksum(ip_hdr, 20) == 0xffff;
}

int oracle_ipv4_udptcp_cksum_verify(const void *ip_hdr, const void *l4_hdr)
{
  const uint8_t *ip = (const uint8_t *) ip_hdr;
  uint32_t l3_len = (uint32_t) ((ip[2] << 8) | ip[3]);
  uint32_t cksum;
  if (l3_len < 20)
    return 0; /* __rte_ipv4_udptcp_cksum returns 0, which is not 0xffff */
  cksum = oracle_raw_cksum(l4_hdr, l3_len - 20);
  cksum += oracle_ipv4_phdr_cksum(ip_hdr, 0);
  cksum = ((cksum & 0xffff0000u) >> 16) + (cksum & 0xffffu);
  return (uint16_t) cksum == 0xffff;
}

/* ---------------------------------------------------------------------- */
/* Batch drivers (one reference-style call per packet). */

static inline uint64_t pkt_off(const uint64_t *off, uint64_t stride, size_t i)
{
  return off ? off[i] : (uint64_t) i * stride;
}

void oracle_raw_batch(const uint8_t *base, const uint64_t *off,
    const uint32_t *len, uint64_t stride, uint32_t len0, size_t n,
    uint16_t *out)
{
  size_t i;
  for (i = 0; i < n; i++)
    out[i] = oracle_raw_cksum(base + pkt_off(off, stride, i),
        len ? len[i] : len0);
}

void oracle_tcp4_batch(uint8_t *base, const uint64_t *off, uint64_t stride,
    size_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out, int inplace)
{
  size_t i;
  for (i = 0; i < n; i++) {
    uint8_t *f = base + pkt_off(off, stride, i);
    uint8_t save_ip[2], save_tcp[2];
    if (!inplace) {
      memcpy(save_ip, f + ip_off + 10, 2);
      memcpy(save_tcp, f + l4_off + 16, 2);
    }
    oracle_tcp_checksums(f + ip_off, f + l4_off);
    memcpy(&out[2 * i], f + ip_off + 10, 2);
    memcpy(&out[2 * i + 1], f + l4_off + 16, 2);
    if (!inplace) {
      memcpy(f + ip_off + 10, save_ip, 2);
      memcpy(f + l4_off + 16, save_tcp, 2);
    }
  }
}

void oracle_tcp4_verify_batch(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off, uint8_t *flags)
{
  size_t i;
  for (i = 0; i < n; i++) {
    const uint8_t *f = base + pkt_off(off, stride, i);
    uint8_t v = 0;
    if (oracle_ipv4_hdr_verify(f + ip_off))
      v |= 1;
    if (oracle_ipv4_udptcp_cksum_verify(f + ip_off, f + l4_off))
      v |= 2;
    if ((f[ip_off] & 0x0f) != 5)
      v |= 4;
    flags[i] = v;
  }
}

/* The same, with a per-frame read bound (bytes from the frame start: the
 * received length, room or stride slot; bound == NULL -> bound0, 0 = none):
 * a datagram whose L4 part reaches past the bound fails the L4 check without
 * being read (libtasx's receive-side contract, include/tasx_xsum.h). */
void oracle_tcp4_verify_batch_bounded(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off,
    const uint32_t *bound, uint32_t bound0, uint8_t *flags)
{
  size_t i;
  for (i = 0; i < n; i++) {
    const uint8_t *f = base + pkt_off(off, stride, i);
    const uint32_t b = bound ? bound[i] : bound0;
    const uint32_t tl = (uint32_t) ((f[ip_off + 2] << 8) | f[ip_off + 3]);
    const uint32_t len = tl >= 20 ? tl - 20 : 0;
    const uint32_t have = b > l4_off ? b - l4_off : 0;
    uint8_t v = 0;
    if (oracle_ipv4_hdr_verify(f + ip_off))
      v |= 1;
    if ((b == 0 || len <= have) && oracle_ipv4_udptcp_cksum_verify(f + ip_off, f + l4_off))
      v |= 2;
    if ((f[ip_off] & 0x0f) != 5)
      v |= 4;
    flags[i] = v;
  }
}

/* ---------------------------------------------------------------------- */
/* TX segment build. */

/* flow_tx_read(), tas/fast/fast_flows.c:833-846: read len bytes at circular
 * position pos of the flow's TX buffer; dma_read() (tas/fast/dma.h:39-53) is a
 * bounds-asserted rte_memcpy from the shared-memory region. */
static void oracle_flow_tx_read(const uint8_t *shm, uint64_t tx_base,
    uint32_t tx_len, uint32_t pos, uint16_t len, uint8_t *dst)
{
  uint32_t part;
  if (pos + len <= tx_len) {
    memcpy(dst, shm + tx_base + pos, len);
  } else {
    part = tx_len - pos;
    memcpy(dst, shm + tx_base + pos, part);
    memcpy(dst + part, shm + tx_base, len - part);
  }
}

/* the descriptor checks that stand in for dma_read()'s assertions */
static int oracle_tx_seg_ok(const struct oracle_tx_seg *d, uint64_t shm_len,
    uint32_t l4_off)
{
  return (d->payload == 0 || d->pos < d->tx_len) && d->payload <= d->tx_len &&
      d->tx_base <= shm_len && d->tx_len <= shm_len - d->tx_base &&
      d->hdrs_len >= l4_off + 20;
}

void oracle_tx_segment_batch(const uint8_t *shm, uint64_t shm_len,
    uint8_t *frames, const struct oracle_tx_seg *segs, size_t n,
    uint32_t ip_off, uint32_t l4_off, uint32_t *out)
{
  size_t i;
  for (i = 0; i < n; i++) {
    const struct oracle_tx_seg *d = &segs[i];
    uint8_t *f = frames + d->frame_off;
    uint16_t ipc, tcpc;
    if (!oracle_tx_seg_ok(d, shm_len, l4_off)) {
      if (out)
        out[i] = 0;
      continue;
    }
    /* flow_tx_segment(): payload at hdrs_len (:930-933), then the checksums
     * over the finished frame (:936 -> tcp_checksums, :1058-1069) */
    if (d->payload > 0)
      oracle_flow_tx_read(shm, d->tx_base, d->tx_len, d->pos, d->payload,
          f + d->hdrs_len);
    oracle_tcp_checksums(f + ip_off, f + l4_off);
    memcpy(&ipc, f + ip_off + 10, 2);
    memcpy(&tcpc, f + l4_off + 16, 2);
    if (out)
      out[i] = (uint32_t) ipc | ((uint32_t) tcpc << 16);
  }
}

/* ---------------------------------------------------------------------- */
/* RX flow lookup. */

/* CRC32C (Castagnoli, reflected polynomial 0x82F63B78) as the SSE4.2 crc32
 * instruction computes it: no pre/post inversion, the data operand consumed
 * least-significant byte first.  DPDK's crc32c_sse42_u32 / _u64
 * (rte_hash_crc.h, third-party, not vendored) wrap exactly that instruction;
 * TAS's flow_hash() (tas/fast/fast_flows.c:1078-1082) and the slow path's
 * rte_hash_crc() over the same 12 bytes (tas/slow/nicif.c:588-600) agree. */
static uint32_t crc_table[256];
static int crc_table_ready;

static void crc_init(void)
{
  uint32_t i, k, c;
  for (i = 0; i < 256; i++) {
    c = i;
    for (k = 0; k < 8; k++)
      c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : c >> 1;
    crc_table[i] = c;
  }
  crc_table_ready = 1;
}

static uint32_t crc_bytes(uint32_t crc, uint64_t data, int nbytes)
{
  int b;
  if (!crc_table_ready)
    crc_init();
  for (b = 0; b < nbytes; b++)
    crc = crc_table[(crc ^ (uint32_t) (data >> (8 * b))) & 0xff] ^ (crc >> 8);
  return crc;
}

uint32_t oracle_crc32c_u32(uint32_t data, uint32_t init)
{
  return crc_bytes(init, data, 4);
}

uint32_t oracle_crc32c_u64(uint64_t data, uint32_t init)
{
  return crc_bytes(init, data, 8);
}

/* flow_hash() of the key fast_flows_packet_fss() builds from a received
 * frame (:1097-1101): local = destination, remote = source. */
uint32_t oracle_flow_hash(const void *ip_hdr, const void *l4_hdr)
{
  const uint8_t *ip = (const uint8_t *) ip_hdr, *l4 = (const uint8_t *) l4_hdr;
  uint32_t lip, rip;
  uint16_t lp, rp;
  memcpy(&lip, ip + 16, 4); /* ip.dest */
  memcpy(&rip, ip + 12, 4); /* ip.src */
  memcpy(&lp, l4 + 2, 2);   /* tcp.dest */
  memcpy(&rp, l4, 2);       /* tcp.src */
  return oracle_crc32c_u32((uint32_t) lp | ((uint32_t) rp << 16),
      oracle_crc32c_u64((uint64_t) lip | ((uint64_t) rip << 32), 0));
}

void oracle_flow_lookup_batch(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off,
    const uint32_t *flowht, uint32_t ht_entries, const uint8_t *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *hash_out, uint32_t *fid_out)
{
  size_t i;
  uint32_t j;
  for (i = 0; i < n; i++) {
    const uint8_t *f = base + pkt_off(off, stride, i);
    const uint8_t *ip = f + ip_off, *l4 = f + l4_off;
    const uint32_t h = oracle_flow_hash(ip, l4);
    uint32_t res = 0xffffffffu;
    /* the last loop of fast_flows_packet_fss() (:1127-1162); the two before
     * it only prefetch */
    for (j = 0; j < 4; j++) {
      const uint32_t k = (h + j) % ht_entries;
      const uint32_t ffid = flowht[2 * k], eh = flowht[2 * k + 1];
      const uint32_t fid = ffid & ((1u << 29) - 1);
      const uint8_t *fs;
      if ((ffid & 0x80000000u) == 0 || eh != h)
        continue;
      if (fid >= fs_num) /* the reference would read past flowst[] */
        continue;
      fs = flowst + (uint64_t) fid * fs_stride + fs_key_off;
      if (memcmp(fs, ip + 16, 4) == 0 && memcmp(fs + 4, ip + 12, 4) == 0 &&
          memcmp(fs + 8, l4 + 2, 2) == 0 && memcmp(fs + 10, l4, 2) == 0) {
        res = fid;
        break;
      }
    }
    fid_out[i] = res;
    if (hash_out)
      hash_out[i] = h;
  }
}

/* ---------------------------------------------------------------------- */
/* CPU baseline timing. */

struct bench_arg {
  int mode, cpu;
  uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride;
  uint32_t len0, ip_off, l4_off;
  size_t lo, hi;
  uint16_t *out;
  const uint8_t *shm;
  uint64_t shm_len;
  const struct oracle_tx_seg *segs;
  const uint32_t *flowht;
  const uint8_t *flowst;
  uint32_t ht_entries, fs_num, fs_stride, fs_key_off;
  uint32_t *fid_out;
  pthread_barrier_t *bar;
  double t0, t1;
};

static double now_s(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static void *bench_worker(void *p)
{
  struct bench_arg *a = (struct bench_arg *) p;
  size_t i;
  if (a->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(a->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  pthread_barrier_wait(a->bar);
  a->t0 = now_s();
  if (a->mode == 0) {
    for (i = a->lo; i < a->hi; i++)
      a->out[i] = oracle_raw_cksum(a->base + pkt_off(a->off, a->stride, i),
          a->len ? a->len[i] : a->len0);
  } else if (a->mode == 3) {
    /* fast_flows_packet_fss() per RX burst */
    oracle_flow_lookup_batch(a->off ? a->base : a->base + a->lo * a->stride,
        a->off ? a->off + a->lo : NULL, a->stride,
        a->hi - a->lo, a->ip_off, a->l4_off, a->flowht, a->ht_entries,
        a->flowst, a->fs_num, a->fs_stride, a->fs_key_off, NULL,
        a->fid_out + a->lo);
  } else if (a->mode == 2) {
    /* flow_tx_segment()'s payload copy + tcp_checksums(), per segment */
    oracle_tx_segment_batch(a->shm, a->shm_len, a->base, a->segs + a->lo,
        a->hi - a->lo, a->ip_off, a->l4_off, NULL);
  } else {
    /* in place, exactly what tcp_checksums() does to each TX frame */
    for (i = a->lo; i < a->hi; i++) {
      uint8_t *f = a->base + pkt_off(a->off, a->stride, i);
      oracle_tcp_checksums(f + a->ip_off, f + a->l4_off);
    }
  }
  a->t1 = now_s();
  return NULL;
}

static int cmp_d(const void *x, const void *y)
{
  double a = *(const double *) x, b = *(const double *) y;
  return (a > b) - (a < b);
}

static double bench_run(const struct bench_arg *proto, size_t n, int threads,
    int reps)
{
  pthread_t *th;
  struct bench_arg *args;
  pthread_barrier_t bar;
  double *times, med;
  cpu_set_t avail;
  int t, r, ncpu_avail = 0, cpus[1024];

  if (threads < 1)
    threads = 1;
  if (reps < 1)
    reps = 1;
  /* pin to the cpus this process may run on, in order */
  CPU_ZERO(&avail);
  if (sched_getaffinity(0, sizeof(avail), &avail) == 0) {
    for (t = 0; t < CPU_SETSIZE && ncpu_avail < 1024; t++)
      if (CPU_ISSET(t, &avail))
        cpus[ncpu_avail++] = t;
  }
  th = calloc((size_t) threads, sizeof(*th));
  args = calloc((size_t) threads, sizeof(*args));
  times = calloc((size_t) reps, sizeof(*times));
  for (r = 0; r < reps; r++) {
    double t0 = 1e300, t1 = 0;
    pthread_barrier_init(&bar, NULL, (unsigned) threads);
    for (t = 0; t < threads; t++) {
      struct bench_arg *a = &args[t];
      *a = *proto;
      a->cpu = ncpu_avail ? cpus[t % ncpu_avail] : -1;
      a->lo = n * (size_t) t / (size_t) threads;
      a->hi = n * (size_t) (t + 1) / (size_t) threads;
      a->bar = &bar;
      pthread_create(&th[t], NULL, bench_worker, a);
    }
    for (t = 0; t < threads; t++) {
      pthread_join(th[t], NULL);
      if (args[t].t0 < t0)
        t0 = args[t].t0;
      if (args[t].t1 > t1)
        t1 = args[t].t1;
    }
    pthread_barrier_destroy(&bar);
    times[r] = t1 - t0;
  }
  qsort(times, (size_t) reps, sizeof(double), cmp_d);
  med = times[reps / 2];
  free(th);
  free(args);
  free(times);
  return med;
}

double oracle_bench(int mode, uint8_t *base, const uint64_t *off,
    const uint32_t *len, uint64_t stride, uint32_t len0, size_t n,
    uint32_t ip_off, uint32_t l4_off, uint16_t *out, int threads, int reps)
{
  struct bench_arg a;
  memset(&a, 0, sizeof(a));
  a.mode = mode;
  a.base = base;
  a.off = off;
  a.len = len;
  a.stride = stride;
  a.len0 = len0;
  a.ip_off = ip_off;
  a.l4_off = l4_off;
  a.out = out;
  return bench_run(&a, n, threads, reps);
}

double oracle_bench_tx_segment(const uint8_t *shm, uint64_t shm_len,
    uint8_t *frames, const struct oracle_tx_seg *segs, size_t n,
    uint32_t ip_off, uint32_t l4_off, int threads, int reps)
{
  struct bench_arg a;
  memset(&a, 0, sizeof(a));
  a.mode = 2;
  a.base = frames;
  a.shm = shm;
  a.shm_len = shm_len;
  a.segs = segs;
  a.ip_off = ip_off;
  a.l4_off = l4_off;
  return bench_run(&a, n, threads, reps);
}

double oracle_bench_flow_lookup(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off,
    const uint32_t *flowht, uint32_t ht_entries, const uint8_t *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *fid_out, int threads, int reps)
{
  struct bench_arg a;
  memset(&a, 0, sizeof(a));
  a.mode = 3;
  a.base = (uint8_t *) base;
  a.off = off;
  a.stride = stride;
  a.ip_off = ip_off;
  a.l4_off = l4_off;
  a.flowht = flowht;
  a.ht_entries = ht_entries;
  a.flowst = flowst;
  a.fs_num = fs_num;
  a.fs_stride = fs_stride;
  a.fs_key_off = fs_key_off;
  a.fid_out = fid_out;
  return bench_run(&a, n, threads, reps);
}
