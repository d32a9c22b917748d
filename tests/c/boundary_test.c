/*
 * boundary_test.c -- libtasx at the C boundary, in TAS's own terms (runs on the
 * GPU box; links libtasx.so only, no oracle).
 *
 * A fake-mbuf harness modelled on the reference unit test
 * (tests/tas_unit/fastpath.c:92-99: calloc'd mbufs, data_off 256, buf_addr
 * after the header) drives the glue of INTEGRATION.md sections 3-4
 * (tests/c/tas_glue.h: tcp_checksums() / fast_flows_kernelxsums() with the
 * reference's own struct pkt_tcp and beui32_t, compiled against
 * /root/reference/include in the build container) over the frames
 * tests/c/gen_ref_frames.c built with the reference's header code, then the
 * tx_flush checksum step, and checks every frame against the committed
 * expectations: the unit-test frame's a3 bb / cf d7 and a 32-frame
 * TXBUF_SIZE batch, staged, zero-copy (mbufs in a registered pool) and through
 * the shared feeder, with
 * the thread-bound context (TASX_CTX_SELF) as the only context plumbing.
 * Then the error contract (ABI 8): a flush server whose
 * kernel is aborted with the batch queued fails the flush; the glue takes the
 * unfinished frames back, finishes them with TAS's CPU path (the test's DPDK
 * stand-in, tests/c/rte_standin.h) and goes on, and the next flush runs on the
 * GPU again -- every frame bit-exact against the fixture.
 *
 *   usage: boundary_test tests/golden/ref_frames.bin
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <packet_defs.h>

/* what TAS provides around the glue (tas/include/config.h:118-119,
 * tas/fast/network.h:37, tas/fast/fastemu.h:97-102) */
struct network_buf_handle;
static struct {
  uint8_t fp_xsumoffload;
} config; /* zero-initialised like the unit test's `struct configuration config;` (fastpath.c:38) */

static inline uint16_t tx_xsum_enable(struct network_buf_handle *nbh, struct ip_hdr *iph, beui32_t ip_s,
    beui32_t ip_d, uint16_t l3_paylen)
{
  (void) nbh, (void) iph, (void) ip_s, (void) ip_d, (void) l3_paylen;
  abort(); /* the offload branch is not under test */
}

/* TAS links DPDK for its CPU checksums; the test links this stand-in */
#include "rte_standin.h"
#include "tas_glue.h"

/* the unit test's dummy mbuf: buf_addr points data_off bytes past the header */
struct fake_mbuf {
  uint8_t *buf_addr;
  uint16_t data_off;
  uint16_t data_len;
  uint32_t buf_len;
};

static struct fake_mbuf *mbuf_at(uint8_t *mem)
{
  struct fake_mbuf *m = (struct fake_mbuf *) mem;
  memset(m, 0, 4096);
  m->data_off = 256;
  m->buf_addr = (uint8_t *) (m + 1) + m->data_off;
  m->buf_len = 4096 - sizeof(*m);
  return m;
}

struct rec {
  uint32_t len;
  uint16_t ip, tcp;
  uint32_t kind;
};

static int fails;
#define CHECK(c, ...) do { if (!(c)) { fails++; fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
                                       fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); } } while (0)

/* record every frame through the glue as its caller would (flow_tx_segment /
 * flow_tx_ack pass the l3 payload length; inject_tcp_ts goes through
 * fast_flows_kernelxsums), flush, check */
static void run_batch(const char *what, struct fake_mbuf **mb, const uint8_t *frames, const struct rec *r,
    uint32_t first, uint32_t n, uint32_t room)
{
  for (uint32_t i = 0; i < n; i++) {
    struct fake_mbuf *m = mb[i];
    memcpy(m->buf_addr, frames + (size_t) (first + i) * room, room);
    m->data_len = (uint16_t) r[first + i].len;
    struct pkt_tcp *p = (struct pkt_tcp *) m->buf_addr;
    struct network_buf_handle *nbh = (struct network_buf_handle *) m;
    if (r[first + i].kind == 2)
      fast_flows_kernelxsums(nbh, p);
    else
      tcp_checksums(nbh, p, p->ip.src, p->ip.dest, f_beui16(p->ip.len) - sizeof(p->ip));
    CHECK(p->ip.chksum == 0 && p->tcp.chksum == 0, "%s frame %u: fields not zeroed by tcp_checksums", what, i);
  }
  CHECK(tasx_pending(TASX_CTX_SELF) == (int) n, "%s: %d pending, expected %u", what, tasx_pending(TASX_CTX_SELF), n);
  tx_flush_checksums();
  CHECK(tasx_pending(TASX_CTX_SELF) == 0, "%s: frames left pending after the flush", what);
  for (uint32_t i = 0; i < n; i++) {
    const struct pkt_tcp *p = (const struct pkt_tcp *) mb[i]->buf_addr;
    const uint8_t *want = frames + (size_t) (first + i) * room;
    CHECK(p->ip.chksum == r[first + i].ip, "%s frame %u: ip.chksum %04x, expected %04x", what, first + i,
          p->ip.chksum, r[first + i].ip);
    CHECK(p->tcp.chksum == r[first + i].tcp, "%s frame %u: tcp.chksum %04x, expected %04x", what, first + i,
          p->tcp.chksum, r[first + i].tcp);
    /* nothing else in the frame changed */
    uint8_t a[4096], b[4096];
    memcpy(a, p, room);
    memcpy(b, want, room);
    memset(a + 24, 0, 2), memset(b + 24, 0, 2), memset(a + 50, 0, 2), memset(b + 50, 0, 2);
    CHECK(memcmp(a, b, room) == 0, "%s frame %u: bytes besides the checksum fields changed", what, first + i);
  }
}

int main(int argc, char **argv)
{
  char magic[8];
  uint32_t n, room;
  FILE *f;
  if (argc != 2 || !(f = fopen(argv[1], "rb"))) {
    fprintf(stderr, "usage: %s ref_frames.bin\n", argv[0]);
    return 2;
  }
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "TASXRF01", 8) || fread(&n, 4, 1, f) != 1 ||
      fread(&room, 4, 1, f) != 1 || n < 2 || n > 64 || room != 2048) {
    fprintf(stderr, "bad fixture %s\n", argv[1]);
    return 2;
  }
  struct rec *r = calloc(n, sizeof(*r));
  uint8_t *frames = malloc((size_t) n * room);
  for (uint32_t i = 0; i < n; i++)
    if (fread(&r[i].len, 4, 1, f) != 1 || fread(&r[i].ip, 2, 1, f) != 1 || fread(&r[i].tcp, 2, 1, f) != 1 ||
        fread(&r[i].kind, 4, 1, f) != 1)
      return 2;
  if (fread(frames, room, n, f) != n)
    return 2;
  fclose(f);

  /* dataplane_init: one context per fast-path core; dataplane_loop binds it */
  if (tasx_ctx_init(0, 0, 4u << 20) != 0 || tasx_set_thread_ctx(0) != 0) {
    fprintf(stderr, "context: %s\n", tasx_last_error());
    return 1;
  }
  CHECK(tasx_thread_ctx() == 0, "thread context not bound");

  /* staged flushes: calloc'd mbufs, as fastpath.c:92-99 */
  struct fake_mbuf *mb[64];
  uint8_t *heap[64];
  for (uint32_t i = 0; i < n; i++)
    mb[i] = mbuf_at(heap[i] = calloc(1, 4096));
  run_batch("kat", mb, frames, r, 0, 1, room);
  {
    const uint8_t *ip = mb[0]->buf_addr + 14;
    CHECK(ip[10] == 0xa3 && ip[11] == 0xbb && ip[36] == 0xcf && ip[37] == 0xd7,
          "unit-test frame: %02x %02x / %02x %02x, expected a3 bb / cf d7", ip[10], ip[11], ip[36], ip[37]);
  }
  run_batch("staged", mb, frames, r, 1, n - 1, room);

  /* zero-copy flushes: the mbufs live in one pool registered as the
   * context's frame region (TAS: the per-core mempool, network.c:320-330) */
  uint8_t *pool = NULL;
  if (posix_memalign((void **) &pool, 4096, (size_t) n * 4096) != 0 || tasx_ctx_register_frames(TASX_CTX_SELF, pool, (size_t) n * 4096) != 0) {
    fprintf(stderr, "register frames: %s\n", tasx_last_error());
    return 1;
  }
  struct fake_mbuf *pm[64];
  for (uint32_t i = 0; i < n; i++)
    pm[i] = mbuf_at(pool + (size_t) i * 4096);
  uint32_t zc0, st0, zc1, st1;
  tasx_ctx_stats(TASX_CTX_SELF, &zc0, &st0);
  run_batch("zero-copy", pm, frames, r, 0, n, room);
  tasx_ctx_stats(TASX_CTX_SELF, &zc1, &st1);
  CHECK(zc1 == zc0 + 1 && st1 == st0, "zero-copy flush not taken (%u/%u -> %u/%u)", zc0, st0, zc1, st1);

  /* the same batch through the GPU's shared feeder */
  uint32_t ff = 0;
  if (tasx_feeder_start(0) != 0 || tasx_ctx_use_feeder(TASX_CTX_SELF, 1) != 0) {
    fprintf(stderr, "feeder: %s\n", tasx_last_error());
    return 1;
  }
  run_batch("feeder", pm, frames, r, 0, n, room);
  tasx_ctx_feeder_flushes(TASX_CTX_SELF, &ff);
  CHECK(ff == 1, "feeder flush not taken (%u)", ff);
  CHECK(tasx_feeder_stop(0) != 0, "feeder stopped while a context is attached");
  if (tasx_ctx_use_feeder(TASX_CTX_SELF, 0) != 0 || tasx_feeder_stop(0) != 0) {
    fprintf(stderr, "feeder: %s\n", tasx_last_error());
    return 1;
  }

  /* the flush server (ABI 6), and a pause (ABI 9): HIP frees wait for the
   * running kernel, so libtasx refuses its own (-EBUSY); paused, with the
   * context still attached, they go through, and the resumed kernel takes the
   * next flush */
  if (tasx_server_start(0) != 0 || tasx_ctx_use_server(TASX_CTX_SELF, 1) != 0) {
    fprintf(stderr, "server: %s\n", tasx_last_error());
    return 1;
  }
  {
    uint32_t sf0 = 0, sf1 = 0;
    void *scratch = tasx_host_alloc(1u << 20);
    CHECK(scratch != NULL, "tasx_host_alloc: %s", tasx_last_error());
    CHECK(tasx_host_free(scratch) == -EBUSY, "a free went through beside the running server");
    CHECK(tasx_server_pause(0) == 0, "server pause: %s", tasx_last_error());
    CHECK(tasx_host_free(scratch) == 0, "free while paused: %s", tasx_last_error());
    CHECK(tasx_server_resume(0) == 0, "server resume: %s", tasx_last_error());
    tasx_ctx_server_flushes(TASX_CTX_SELF, &sf0);
    run_batch("server-after-resume", pm, frames, r, 0, n, room);
    tasx_ctx_server_flushes(TASX_CTX_SELF, &sf1);
    CHECK(sf1 == sf0 + 1, "the flush after the resume did not go through the server (%u -> %u)", sf0, sf1);
  }
  /* a failed flush: the flush server's kernel aborted while the context is
   * attached, then a batch recorded and flushed.  tx_flush_checksums sees the
   * error and finishes every frame on the CPU; TAS keeps running. */
  CHECK(tasx_server_abort(0) == 0, "server abort: %s", tasx_last_error());
  unsigned recovered = 0;
  {
    for (uint32_t i = 0; i < n; i++) { /* record as run_batch does */
      struct fake_mbuf *m = pm[i];
      memcpy(m->buf_addr, frames + (size_t) i * room, room);
      m->data_len = (uint16_t) r[i].len;
      struct pkt_tcp *p = (struct pkt_tcp *) m->buf_addr;
      if (r[i].kind == 2)
        fast_flows_kernelxsums((struct network_buf_handle *) m, p);
      else
        tcp_checksums((struct network_buf_handle *) m, p, p->ip.src, p->ip.dest, f_beui16(p->ip.len) - sizeof(p->ip));
    }
    CHECK(tasx_flush(TASX_CTX_SELF) != 0, "a flush through an aborted server succeeded");
    recovered = tasx_finish_unfinished();
    CHECK(recovered == n, "%u frames handed back, expected %u", recovered, n);
    CHECK(tasx_pending(TASX_CTX_SELF) == 0, "frames left pending after the recovery");
    for (uint32_t i = 0; i < n; i++) {
      const struct pkt_tcp *p = (const struct pkt_tcp *) pm[i]->buf_addr;
      CHECK(p->ip.chksum == r[i].ip && p->tcp.chksum == r[i].tcp, "recovered frame %u: %04x/%04x, expected %04x/%04x",
            i, p->ip.chksum, p->tcp.chksum, r[i].ip, r[i].tcp);
    }
  }
  /* the context detached from the gone kernel; the next flush is the GPU's again */
  CHECK(tasx_server_stop(0) == 0, "server stop after the recovery: %s", tasx_last_error());
  tasx_ctx_stats(TASX_CTX_SELF, &zc0, &st0);
  run_batch("after-recovery", pm, frames, r, 0, n, room);
  tasx_ctx_stats(TASX_CTX_SELF, &zc1, &st1);
  CHECK(zc1 == zc0 + 1, "the flush after the recovery did not run on the GPU");

  tasx_ctx_destroy(TASX_CTX_SELF);
  tasx_set_thread_ctx(TASX_CTX_SELF);
  CHECK(tasx_thread_ctx() < 0, "thread context still bound");
  printf("boundary_test: %u frames (unit-test KAT + %u-frame tx_flush batch), staged, zero-copy and feeder: %s\n", n,
         n - 1, fails ? "FAILED" : "OK");
  printf("boundary_test: aborted flush server, %u frames finished by the glue's CPU path, then the GPU again: %s\n",
         recovered, fails ? "FAILED" : "OK");
  return fails ? 1 : 0;
}
