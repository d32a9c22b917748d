/*
 * gen_ref_frames.c -- golden TX frames built with the reference's own wire
 * types and header macros (test infrastructure; runs in the build container,
 * where /root/reference exists, never on the GPU box).
 *
 *   gcc -std=gnu99 -O2 -I/root/reference/include -Iinclude \
 *       tests/c/gen_ref_frames.c oracle/tasx_oracle.c -o gen && ./gen out.bin
 *
 * The frames are what TAS hands to tcp_checksums(): flow_tx_segment's header
 * fill (tas/fast/fast_flows.c:886-933: IPH_VHL_SET, t_beui16/t_beui32,
 * TCPH_HDRLEN_FLAGS_SET, the 10-byte timestamp option padded to 12) and
 * flow_tx_ack's in-place rewrite of a received segment (:976-1008, checksum
 * fields left as received).  Frame 0 is the reference unit test's frame
 * (tests/tas_unit/fastpath.c:68-89,187-207: fast_flows_bump ->
 * flow_tx_segment, payload 0), whose checksums are the hand-derived KAT
 * a3 bb / cf d7; frames 1..32 are a TXBUF_SIZE (32,
 * tas/include/fastpath.h:38) tx_flush batch of data segments, window updates,
 * FIN, ECN-capable segments and ACKs.  Expected checksums come from the CPU
 * oracle (oracle/tasx_oracle.c, the DPDK 19.11 restatement).
 *
 * Output (little endian): "TASXRF01", u32 n, u32 room, n x {u32 frame_len
 * (the tx_send length), u16 ip.chksum, u16 tcp.chksum, u32 kind (0 segment,
 * 1 ack, 2 kernelxsums)}, then n x room bytes of frames.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <packet_defs.h>

#include "../../oracle/tasx_oracle.h"

/* the layout the kernels assume (include/tasx_xsum.h TASX_TAS_IP_OFF/L4_OFF) */
_Static_assert(sizeof(struct pkt_tcp) == 54, "struct pkt_tcp is 54 bytes");
_Static_assert(offsetof(struct pkt_tcp, ip) == 14, "ip at frame offset 14");
_Static_assert(offsetof(struct pkt_tcp, tcp) == 34, "tcp at frame offset 34");
_Static_assert(sizeof(struct ip_hdr) == 20 && sizeof(struct tcp_hdr) == 20, "20-byte IPv4 / TCP headers");
_Static_assert(offsetof(struct ip_hdr, chksum) == 10, "ip.chksum at ip + 10");
_Static_assert(offsetof(struct tcp_hdr, chksum) == 16, "tcp.chksum at tcp + 16");
_Static_assert(sizeof(struct tcp_timestamp_opt) == 10, "10-byte timestamp option");

#define ROOM 2048 /* BUFFER_SIZE, tas/fast/internal.h:34 */
#define NFRAMES 33
#define TEST_IP 0x0a010203 /* tests/tas_unit/fastpath.c:18-22 */
#define TEST_PORT 12345
#define TEST_LIP 0x0a010201
#define TEST_LPORT 23456

struct flow {
  struct eth_addr remote_mac;
  beui32_t local_ip, remote_ip;
  beui16_t local_port, remote_port;
  int ecn;
};

static const struct eth_addr eth_addr; /* the unit test's (zero) local MAC */

/* flow_tx_segment()'s frame, fast_flows.c:886-933; returns hdrs_len + payload */
static uint16_t segment(uint8_t *buf, const struct flow *fs, uint32_t seq, uint32_t ack, uint32_t rxwnd,
    uint16_t payload, const uint8_t *data, uint32_t ts_echo, uint32_t ts_my, int fin)
{
  struct pkt_tcp *p = (struct pkt_tcp *) buf;
  struct tcp_timestamp_opt *opt_ts;
  const uint16_t optlen = (sizeof(*opt_ts) + 3) & ~3;
  const uint16_t hdrs_len = sizeof(*p) + optlen;

  p->eth.dest = fs->remote_mac;
  memcpy(&p->eth.src, &eth_addr, ETH_ADDR_LEN);
  p->eth.type = t_beui16(ETH_TYPE_IP);
  IPH_VHL_SET(&p->ip, 4, 5);
  p->ip._tos = 0;
  p->ip.len = t_beui16(hdrs_len - offsetof(struct pkt_tcp, ip) + payload);
  p->ip.id = t_beui16(3);
  p->ip.offset = t_beui16(0);
  p->ip.ttl = 0xff;
  p->ip.proto = IP_PROTO_TCP;
  p->ip.chksum = 0;
  p->ip.src = fs->local_ip;
  p->ip.dest = fs->remote_ip;
  if (fs->ecn)
    IPH_ECN_SET(&p->ip, IP_ECN_ECT0);
  p->tcp.src = fs->local_port;
  p->tcp.dest = fs->remote_port;
  p->tcp.seqno = t_beui32(seq);
  p->tcp.ackno = t_beui32(ack);
  TCPH_HDRLEN_FLAGS_SET(&p->tcp, 5 + optlen / 4, TCP_PSH | TCP_ACK | (fin ? TCP_FIN : 0));
  p->tcp.wnd = t_beui16(MIN(0xFFFF, rxwnd));
  p->tcp.chksum = 0;
  p->tcp.urgp = t_beui16(0);
  memset(p + 1, 0, optlen);
  opt_ts = (struct tcp_timestamp_opt *) (p + 1);
  opt_ts->kind = TCP_OPT_TIMESTAMP;
  opt_ts->length = sizeof(*opt_ts);
  opt_ts->ts_val = t_beui32(ts_my);
  opt_ts->ts_ecr = t_beui32(ts_echo);
  if (payload > 0)
    memcpy(buf + hdrs_len, data, payload);
  return hdrs_len + payload;
}

/* flow_tx_ack()'s in-place rewrite of a received segment, fast_flows.c:976-1008
 * (checksum fields stay as received: tcp_checksums() zeroes them); returns hdrlen */
static uint16_t ack_in_place(uint8_t *buf, uint32_t seq, uint32_t ack, uint32_t rxwnd, uint32_t echots,
    uint32_t myts)
{
  struct pkt_tcp *p = (struct pkt_tcp *) buf;
  struct tcp_timestamp_opt *ts_opt = (struct tcp_timestamp_opt *) (p + 1);
  struct eth_addr eth = p->eth.src;
  ip_addr_t ip = p->ip.src;
  beui16_t port = p->tcp.src;
  uint16_t ecn_flags = 0, hdrlen;

  p->eth.src = p->eth.dest;
  p->eth.dest = eth;
  p->ip.src = p->ip.dest;
  p->ip.dest = ip;
  p->tcp.src = p->tcp.dest;
  p->tcp.dest = port;
  hdrlen = sizeof(*p) + (TCPH_HDRLEN(&p->tcp) - 5) * 4;
  if (IPH_ECN(&p->ip) == IP_ECN_CE)
    ecn_flags = TCP_ECE;
  IPH_ECN_SET(&p->ip, IP_ECN_NONE);
  p->tcp.seqno = t_beui32(seq);
  p->tcp.ackno = t_beui32(ack);
  TCPH_HDRLEN_FLAGS_SET(&p->tcp, TCPH_HDRLEN(&p->tcp), TCP_ACK | ecn_flags);
  p->tcp.wnd = t_beui16(MIN(0xFFFF, rxwnd));
  p->tcp.urgp = t_beui16(0);
  ts_opt->ts_val = t_beui32(myts);
  ts_opt->ts_ecr = t_beui32(echots);
  p->ip.len = t_beui16(hdrlen - offsetof(struct pkt_tcp, ip));
  p->ip.ttl = 0xff;
  return hdrlen;
}

static uint32_t lcg(uint32_t *s)
{
  *s = *s * 1664525u + 1013904223u;
  return *s >> 8;
}

int main(int argc, char **argv)
{
  static uint8_t frames[NFRAMES][ROOM];
  static uint8_t data[ROOM];
  uint32_t len[NFRAMES], kind[NFRAMES];
  uint16_t eip[NFRAMES], etcp[NFRAMES];
  uint32_t s = 0x7a5c5eed;
  FILE *f;

  if (argc != 2) {
    fprintf(stderr, "usage: %s out.bin\n", argv[0]);
    return 2;
  }
  memset(frames, 0, sizeof(frames));
  for (int i = 0; i < ROOM; i++)
    data[i] = (uint8_t) lcg(&s);

  /* frame 0: the unit test's flow (flow_init, fastpath.c:68-89) after
   * test_rxbump_fc_reopen_notx's bump: seq 0, ack 0, window 1024, no payload */
  struct flow t0;
  memset(&t0, 0, sizeof(t0));
  t0.local_ip = t_beui32(TEST_LIP);
  t0.remote_ip = t_beui32(TEST_IP);
  t0.local_port = t_beui16(TEST_LPORT);
  t0.remote_port = t_beui16(TEST_PORT);
  len[0] = segment(frames[0], &t0, 0, 0, 1024, 0, NULL, 0, 0, 0);
  kind[0] = 0;

  /* frames 1..32: one tx_flush batch over 5 flows */
  struct flow fl[5];
  for (int k = 0; k < 5; k++) {
    memset(&fl[k], 0, sizeof(fl[k]));
    for (int b = 0; b < ETH_ADDR_LEN; b++)
      fl[k].remote_mac.addr[b] = (uint8_t) lcg(&s);
    fl[k].local_ip = t_beui32(0x0a000001u + (uint32_t) k);
    fl[k].remote_ip = t_beui32(0xc0a80000u | (lcg(&s) & 0xffff));
    fl[k].local_port = t_beui16((uint16_t) (1024 + lcg(&s) % 60000));
    fl[k].remote_port = t_beui16((uint16_t) (1 + lcg(&s) % 65535));
    fl[k].ecn = k == 3;
  }
  static const uint16_t pays[] = {1448, 1448, 1448, 0, 1, 2, 3, 536, 1447, 100, 1448, 0, 1000, 1448, 17, 1448,
                                  1448, 1448, 64, 1448};
  int i = 1;
  for (int k = 0; k < 20; k++, i++) {
    const struct flow *fs = &fl[k % 5];
    const uint16_t pay = pays[k];
    len[i] = segment(frames[i], fs, lcg(&s), lcg(&s), lcg(&s) % 200000, pay, data + (k * 37) % 512,
        lcg(&s), lcg(&s), k == 9 || k == 17);
    kind[i] = k % 7 == 6 ? 2 : 0; /* some through fast_flows_kernelxsums (inject_tcp_ts) */
  }
  for (int k = 0; k < 12; k++, i++) {
    /* a received segment of the peer (addresses the other way round, random
     * checksum fields, CE marked on some), turned into the ACK in place */
    struct flow peer = fl[k % 5];
    peer.local_ip = fl[k % 5].remote_ip;
    peer.remote_ip = fl[k % 5].local_ip;
    peer.local_port = fl[k % 5].remote_port;
    peer.remote_port = fl[k % 5].local_port;
    segment(frames[i], &peer, lcg(&s), lcg(&s), 4096, (uint16_t) (k * 113 % 1449), data, lcg(&s), lcg(&s), 0);
    struct pkt_tcp *p = (struct pkt_tcp *) frames[i];
    p->ip.chksum = (uint16_t) lcg(&s);
    p->tcp.chksum = (uint16_t) lcg(&s);
    if (k % 4 == 1)
      IPH_ECN_SET(&p->ip, IP_ECN_CE);
    len[i] = ack_in_place(frames[i], lcg(&s), lcg(&s), lcg(&s) % 70000, lcg(&s), lcg(&s));
    kind[i] = 1;
  }

  /* expected: tcp_checksums()' flag-off branch on a copy of each frame */
  for (i = 0; i < NFRAMES; i++) {
    uint8_t tmp[ROOM];
    memcpy(tmp, frames[i], ROOM);
    oracle_tcp_checksums(tmp + 14, tmp + 34);
    memcpy(&eip[i], tmp + 24, 2);
    memcpy(&etcp[i], tmp + 50, 2);
  }
  if (!(eip[0] == 0xbba3 && etcp[0] == 0xd7cf)) { /* bytes a3 bb / cf d7 */
    fprintf(stderr, "KAT frame: ip %04x tcp %04x, expected a3bb / cfd7 (as bytes)\n", eip[0], etcp[0]);
    return 1;
  }

  if (!(f = fopen(argv[1], "wb")))
    return 1;
  const uint32_t n = NFRAMES, room = ROOM;
  fwrite("TASXRF01", 1, 8, f);
  fwrite(&n, 4, 1, f);
  fwrite(&room, 4, 1, f);
  for (i = 0; i < NFRAMES; i++) {
    fwrite(&len[i], 4, 1, f);
    fwrite(&eip[i], 2, 1, f);
    fwrite(&etcp[i], 2, 1, f);
    fwrite(&kind[i], 4, 1, f);
  }
  fwrite(frames, ROOM, NFRAMES, f);
  fclose(f);
  printf("%d frames (KAT a3bb/cfd7 + a %d-frame tx_flush batch) -> %s\n", NFRAMES, NFRAMES - 1, argv[1]);
  return 0;
}
