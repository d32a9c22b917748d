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
 * It also provides the CPU checksum functions TAS's own build links from DPDK
 * (rte_ipv4_cksum, rte_ipv4_udptcp_cksum; here tests/c/rte_standin.h): the
 * glue's error recovery finishes the frames libtasx hands back with them.
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
      /* not recorded (the context's pending capacity): this frame takes
       * TAS's own CPU path, the reference's #else branch */
      p->ip.chksum = rte_ipv4_cksum((void *) &p->ip);
      p->tcp.chksum = rte_ipv4_udptcp_cksum((void *) &p->ip, (void *) &p->tcp);
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

/* Error recovery (ABI 8): after any failed libtasx call the frames the GPU
 * did not finish come back from tasx_take_unfinished and take TAS's own CPU
 * path (fast_flows.c:1065-1067); returns how many did */
static inline unsigned tasx_finish_unfinished(void)
{
  tasx_frame_ref fr[64];
  unsigned done = 0;
  int k;
  while ((k = tasx_take_unfinished(TASX_CTX_SELF, fr, 64)) > 0) {
    for (int i = 0; i < k; i++) {
      struct ip_hdr *ip = (struct ip_hdr *) fr[i].ip;
      struct tcp_hdr *tcp = (struct tcp_hdr *) fr[i].l4;
      ip->chksum = 0;
      tcp->chksum = 0;
      ip->chksum = rte_ipv4_cksum((void *) ip);
      tcp->chksum = rte_ipv4_udptcp_cksum((void *) ip, (void *) tcp);
    }
    done += (unsigned) k;
  }
  return done;
}

/* the checksum part of tx_flush (tas/fast/fastemu.c:544-566), before
 * network_send(): every recorded frame gets both fields -- from the GPU, or,
 * when its flush fails, from the CPU path above; TAS keeps running */
static inline void tx_flush_checksums(void)
{
  if (!config.fp_xsumoffload && tasx_pending(TASX_CTX_SELF) > 0 &&
      tasx_flush(TASX_CTX_SELF) != 0) {
    fprintf(stderr, "tx_flush: tasx_flush: %s; finishing on the CPU\n", tasx_last_error());
    tasx_finish_unfinished();
  }
}

#endif
