/*
 * tas_glue.h -- the TAS-side glue of INTEGRATION.md sections 3 and 4, as code:
 * tests/c/boundary_test.c compiles exactly this text against the reference's
 * own wire types (/root/reference/include/packet_defs.h, include/utils.h:
 * struct pkt_tcp, beui32_t, f_beui16), the way tas/fast/fast_flows.c would.
 *
 * The including file provides what TAS provides there: `config`
 * (tas/include/config.h:118-119, fp_xsumoffload), tx_xsum_enable()
 * (tas/fast/fastemu.h:97-102, the offload branch, untouched) and the opaque
 * struct network_buf_handle (tas/fast/network.h:37).
 *
 * Context plumbing: tcp_checksums() and fast_flows_kernelxsums() carry no
 * dataplane_context (fast_flows.c:1058,1071), but each fast-path thread runs
 * exactly one context (dataplane_loop, tas/fast/fastemu.c:142), so the thread
 * binds its context once -- tasx_set_thread_ctx(ctx->id) at the top of
 * dataplane_loop -- and the per-frame calls pass TASX_CTX_SELF.
 */
#ifndef TAS_GLUE_H_
#define TAS_GLUE_H_

#include <stdio.h>
#include <stdlib.h>

#include <packet_defs.h>

#include "tasx_xsum.h"

/* tas/fast/fast_flows.c:1058-1069: the flag-off branch records the frame on
 * the calling thread's libtasx context (no device work under fs_lock) */
static inline void tcp_checksums(struct network_buf_handle *nbh,
    struct pkt_tcp *p, beui32_t ip_s, beui32_t ip_d, uint16_t l3_paylen)
{
  p->ip.chksum = 0;
  if (config.fp_xsumoffload) {
    p->tcp.chksum = tx_xsum_enable(nbh, &p->ip, ip_s, ip_d, l3_paylen);
  } else {
    p->tcp.chksum = 0;
    if (tasx_tcp_checksums(TASX_CTX_SELF, nbh, p, ip_s.x, ip_d.x, l3_paylen) != 0) {
      fprintf(stderr, "tcp_checksums: %s\n", tasx_last_error());
      abort(); /* as tx_send on a full TX buffer, fastemu.h:86-89 */
    }
  }
}

/* tas/fast/fast_flows.c:1071-1076, unchanged: it reaches libtasx through
 * tcp_checksums() */
static inline void fast_flows_kernelxsums(struct network_buf_handle *nbh,
    struct pkt_tcp *p)
{
  tcp_checksums(nbh, p, p->ip.src, p->ip.dest,
      f_beui16(p->ip.len) - sizeof(p->ip));
}

/* the checksum part of tx_flush (tas/fast/fastemu.c:544-566), before
 * network_send(): every recorded frame gets both fields */
static inline void tx_flush_checksums(void)
{
  if (!config.fp_xsumoffload && tasx_pending(TASX_CTX_SELF) > 0 &&
      tasx_flush(TASX_CTX_SELF) != 0) {
    fprintf(stderr, "tx_flush: tasx_flush: %s\n", tasx_last_error());
    abort();
  }
}

#endif
