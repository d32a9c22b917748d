/*
 * tasx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's software checksum path (TAS run with
 * --fp-no-xsumoffload).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may link or call this code, and only as the checker /
 * reported baseline.  The product library (tas_amd/csrc -> libtasx.so) never
 * links it and has no CPU fallback.
 *
 * Parity status: the arithmetic lives in DPDK's header-only rte_ip.h, which
 * is a third-party dependency absent from /root/reference (TAS CI pins DPDK
 * 17.11.9 / 18.11.5 / 19.11, .travis.yml:7-9).  It is restated here from the
 * published DPDK 19.11 lib/librte_net/rte_ip.h algorithm.  The reference's own
 * tests pin NO checksum value (tests/tas_unit/fastpath.c:206,258 "TODO: check
 * ack packet"), so the oracle is pinned by (1) the published RFC 1071 section 3
 * vector, (2) a known-answer frame built exactly as the reference unit test
 * scenario builds it (tests/tas_unit/fastpath.c:187-207 ->
 * tas/fast/fast_flows.c:877-955), hand-derived, (3) the Linux TCP/IP stack
 * -- the check the reference's own end-to-end test relies on
 * (tests/full/fulltest.c:103: TAS with --fp-no-xsumoffload against Linux,
 * which drops bad checksums): 51 frames Linux checksummed and 41 frames this
 * oracle checksummed that Linux accepted (tests/golden/gen_linux_frames.py,
 * tests/test_linux_frames.py), and (4) an independent numpy restatement
 * (oracle/xsum_ref.py) over committed random fixtures.  No output of the
 * reference itself exists for this path (it cannot be built here; see
 * DESIGN.md section 4).
 */
#ifndef TASX_ORACLE_H_
#define TASX_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* a1: DPDK __rte_raw_cksum(buf, len, sum) */
uint32_t oracle_raw_cksum_acc(const void *buf, size_t len, uint32_t sum);
/* DPDK __rte_raw_cksum_reduce(sum) */
uint16_t oracle_raw_cksum_reduce(uint32_t sum);
/* a2: DPDK rte_raw_cksum(buf, len) -- folded, NOT inverted */
uint16_t oracle_raw_cksum(const void *buf, size_t len);
/* a3: DPDK rte_ipv4_cksum(ip) (20 B, IHL ignored) */
uint16_t oracle_ipv4_cksum(const void *ip_hdr);
/* a4: DPDK rte_ipv4_phdr_cksum(ip, ol_flags) */
uint16_t oracle_ipv4_phdr_cksum(const void *ip_hdr, uint64_t ol_flags);
/* a5: DPDK 19.11 rte_ipv4_udptcp_cksum(ip, l4) */
uint16_t oracle_ipv4_udptcp_cksum(const void *ip_hdr, const void *l4_hdr);
/* a6 (flag-off branch) of tas/fast/fast_flows.c:1058-1069 tcp_checksums():
 * zero ip.chksum and tcp.chksum, then store rte_ipv4_cksum / udptcp_cksum. */
void oracle_tcp_checksums(void *ip_hdr, void *l4_hdr);
/* a8: tas/fast/network.h:157-173 network_ip_phdr_xsum (offload side) */
uint16_t oracle_ip_phdr_xsum(uint32_t ip_src_be, uint32_t ip_dst_be,
    uint8_t proto, uint16_t l3_paylen);

/* Receive-side verification (new behaviour).
 * hdr: rte_raw_cksum of the 20-byte header (checksum included) == 0xffff.
 * l4: DPDK 21.11 rte_ipv4_udptcp_cksum_verify for IHL 5 (published algorithm,
 * third-party): l3 < 20 fails; fold1(rte_raw_cksum(l4, l3-20) +
 * rte_ipv4_phdr_cksum(ip, 0)) == 0xffff. */
int oracle_ipv4_hdr_verify(const void *ip_hdr);
int oracle_ipv4_udptcp_cksum_verify(const void *ip_hdr, const void *l4_hdr);
/* flags[i] = hdr_ok | l4_ok << 1 | (IHL != 5) << 2 */
void oracle_tcp4_verify_batch(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off, uint8_t *flags);
/* with a per-frame read bound (bound[i], or bound0; 0 = none): L4 fails when
 * the datagram's L4 part reaches past it (libtasx's RX contract) */
void oracle_tcp4_verify_batch_bounded(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off,
    const uint32_t *bound, uint32_t bound0, uint8_t *flags);

/* TX segment build: flow_tx_segment()'s payload
 * copy, flow_tx_read() (tas/fast/fast_flows.c:833-846, :930-933), then
 * tcp_checksums() over the frame (:936).  Same 32-byte descriptor as
 * tasx_tx_seg (include/tasx_xsum.h).  Rejected descriptors: out[i] = 0, frame
 * untouched.  out may be NULL. */
struct oracle_tx_seg {
  uint64_t frame_off, tx_base;
  uint32_t tx_len, pos;
  uint16_t payload, hdrs_len;
  uint32_t room;     /* ignored: the oracle writes exactly the frame's bytes */
};
void oracle_tx_segment_batch(const uint8_t *shm, uint64_t shm_len,
    uint8_t *frames, const struct oracle_tx_seg *segs, size_t n,
    uint32_t ip_off, uint32_t l4_off, uint32_t *out);

/* RX flow lookup: fast_flows_packet_fss(),
 * tas/fast/fast_flows.c:1084-1163, and its CRC32C flow_hash (:1078-1082). */
uint32_t oracle_crc32c_u32(uint32_t data, uint32_t init);
uint32_t oracle_crc32c_u64(uint64_t data, uint32_t init);
uint32_t oracle_flow_hash(const void *ip_hdr, const void *l4_hdr);
void oracle_flow_lookup_batch(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off,
    const uint32_t *flowht, uint32_t ht_entries, const uint8_t *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *hash_out, uint32_t *fid_out);

/* PKT_TX_TCP_SEG bit of DPDK 19.11 rte_mbuf_core.h (1ULL << 50) */
#define ORACLE_PKT_TX_TCP_SEG (1ULL << 50)

/* Batch drivers: one per-packet call each, the way TAS calls per frame. */
void oracle_raw_batch(const uint8_t *base, const uint64_t *off,
    const uint32_t *len, uint64_t stride, uint32_t len0, size_t n,
    uint16_t *out);
/* TCP4 frames: frame i at base + off[i] (or i*stride when off == NULL);
 * out[2i] = ip.chksum, out[2i+1] = tcp.chksum as tcp_checksums() stores them.
 * inplace != 0: leave the results in the frames (as TAS does); otherwise the
 * 4 checksum bytes of each frame are restored afterwards. */
void oracle_tcp4_batch(uint8_t *base, const uint64_t *off, uint64_t stride,
    size_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out, int inplace);

/* CPU baseline timing (bench.py cpu_baseline leg): run the per-packet loop over
 * contiguous shards on `threads` pinned pthreads, `reps` times; returns the
 * median wall seconds of one pass over all n packets. mode 0 = RAW, 1 = TCP4. */
double oracle_bench(int mode, uint8_t *base, const uint64_t *off,
    const uint32_t *len, uint64_t stride, uint32_t len0, size_t n,
    uint32_t ip_off, uint32_t l4_off, uint16_t *out, int threads, int reps);
/* same for the RX flow lookup (mode 3) */
double oracle_bench_flow_lookup(const uint8_t *base, const uint64_t *off,
    uint64_t stride, size_t n, uint32_t ip_off, uint32_t l4_off,
    const uint32_t *flowht, uint32_t ht_entries, const uint8_t *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *fid_out, int threads, int reps);
/* same for the TX segment build (copy + checksums per segment) */
double oracle_bench_tx_segment(const uint8_t *shm, uint64_t shm_len,
    uint8_t *frames, const struct oracle_tx_seg *segs, size_t n,
    uint32_t ip_off, uint32_t l4_off, int threads, int reps);

#ifdef __cplusplus
}
#endif
#endif
