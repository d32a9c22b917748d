/*
 * tasx_xsum.h -- C ABI of libtasx, the MI355X (gfx950) implementation of TAS's
 * software TCP/IP checksum path (TAS run with --fp-no-xsumoffload).
 *
 * What it replaces in the reference (/root/reference):
 *   - tcp_checksums(nbh, p, ip_s, ip_d, l3_paylen), flag-off branch,
 *     tas/fast/fast_flows.c:1058-1069 (decl :75-76)      -> tasx_tcp_checksums
 *   - fast_flows_kernelxsums(nbh, p), tas/fast/fast_flows.c:1071-1076,
 *     declared tas/fast/fastemu.h:70-71                   -> tasx_fast_flows_kernelxsums
 *   - the per-frame DPDK calls it makes, rte_ipv4_cksum + rte_ipv4_udptcp_cksum
 *     (DPDK 19.11 rte_ip.h, not vendored; called at fast_flows.c:1066-1067)
 *     -> batched on the GPU by tasx_tcp4_cksum_batch_dev / _host
 *   - rte_raw_cksum over packet payloads
 *     -> tasx_raw_cksum_batch_dev / _host
 *   - the batch boundary tx_flush(ctx), tas/fast/fastemu.c:544-566 -> tasx_flush
 *
 * Conventions:
 *   - Plain C types only.  `stream` is a hipStream_t passed as void* (NULL =
 *     the null stream).  Device-resident (_dev) entry points are asynchronous
 *     on that stream; everything else returns after the work is complete.
 *   - Return 0 on success or a negative errno (-EINVAL bad argument, -ENOMEM,
 *     -ENODEV no usable GPU, -EIO a HIP runtime error; tasx_last_error()
 *     describes the last one).  There is NO CPU fallback inside libtasx: a
 *     frame whose checksum could not be computed on the GPU is reported, never
 *     silently computed elsewhere.  The reference's per-frame calls cannot
 *     fail (void), so the deferred forms hand such frames
 *     back (tasx_take_unfinished, ABI 8) and TAS's integration finishes them
 *     with its own rte_ipv4_cksum / rte_ipv4_udptcp_cksum and keeps running
 *     (INTEGRATION.md section 3).
 *   - Checksum results are native (little-endian) uint16 values, exactly what
 *     tcp_checksums() stores into ip.chksum / tcp.chksum
 *     (include/packet_defs.h:96,165): their bytes are the network-order
 *     RFC 1071 checksum.
 *   - Arithmetic is bit-exact with DPDK 19.11: rte_raw_cksum (folded, not
 *     inverted, 0 only for all-zero input), rte_ipv4_cksum (20 B, IHL ignored,
 *     0xffff kept), rte_ipv4_udptcp_cksum (L4 length from ip.total_length,
 *     0 when total_length < 20, result 0 -> 0xffff).
 */
#ifndef TASX_XSUM_H_
#define TASX_XSUM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TASX_XSUM_ABI 10
#define TASX_ABI_VERSION TASX_XSUM_ABI /* tasx_abi_version() */

/* flags for the TCP4 batch entry points */
#define TASX_F_INPLACE 0x1u /* also store ip.chksum / tcp.chksum into the frames */
/* host batches over offsets (ABI 5): read the packets where they lie, in
 * pinned or registered memory, over PCIe instead of gathering them */
#define TASX_F_ZEROCOPY 0x2u

/* largest RAW packet: DPDK's 32-bit accumulator cannot wrap below this
 * (65536 words * 0xffff + 0xff < 2^32), so results stay bit-exact. */
#define TASX_RAW_MAX_LEN 131073u

/* TAS frame layout (struct pkt_tcp, include/packet_defs.h:215-219) */
#define TASX_TAS_IP_OFF 14u
#define TASX_TAS_L4_OFF 34u

/* Maximum fast-path contexts (fp_cores_max <= FLEXNIC_PL_APPST_CTX_MCS = 16,
 * tas/fast/fastemu.c:87-91). */
#define TASX_MAX_CTX 16u

int tasx_abi_version(void);
const char *tasx_last_error(void);
/* number of visible GPUs (-EIO on runtime failure) */
int tasx_device_count(void);

/* ---------------------------------------------------------------------- */
/* Device-resident batches.  All pointers are device pointers (or host memory
 * the device can address).  Packet i starts at base + off[i], or at
 * base + i * stride when off == NULL.  Asynchronous on `stream`.  Kernels
 * read whole 16-byte aligned chunks: only chunks holding at least one byte of
 * the packet (or of the hinted / room range below), so a read never leaves
 * the pages the packet lies in, and bytes outside it never enter a result. */

/* RAW: out[i] = rte_raw_cksum(base + off_i, len_i); len_i = len[i], or len0
 * when len == NULL; len_i <= TASX_RAW_MAX_LEN (device-side lengths are the
 * caller's responsibility). */
int tasx_raw_cksum_batch_dev(const void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *len, uint32_t len0, uint32_t n,
    uint16_t *out, void *stream);

/* TCP4: for each frame, the flag-off branch of tcp_checksums(): with
 * ip = frame + ip_off and tcp = frame + l4_off (ip.chksum and tcp.chksum
 * taken as zero), out[2i] = rte_ipv4_cksum(ip), out[2i+1] =
 * rte_ipv4_udptcp_cksum(ip, tcp).  `out` (4-byte aligned) may be NULL when
 * TASX_F_INPLACE is set.  Frames must not overlap. */
int tasx_tcp4_cksum_batch_dev(void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint16_t *out, uint32_t flags, void *stream);

/* The offload branch of tcp_checksums() (config.fp_xsumoffload set,
 * tas/fast/fast_flows.c:1060-1064): per frame, ip.chksum = 0 and tcp.chksum =
 * tx_xsum_enable() = network_ip_phdr_xsum(ip.src, ip.dest, IP_PROTO_TCP,
 * l3_paylen) (tas/fast/fastemu.h:97-102, tas/fast/network.h:157-173): the
 * pseudo-header sum folded twice and not inverted, for the NIC to finish, with
 * l3_paylen = ip.total_length - 20 (what every caller passes).  out[i] (may be
 * NULL with TASX_F_INPLACE, which stores both fields in the frame).  The mbuf's
 * offload flags (network_buf_tcpxsums, network.h:175-187) stay with TAS. */
int tasx_tcp4_offload_batch_dev(void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint16_t *out, uint32_t flags, void *stream);

/* Same, with frame-length hints: flen[i] (or flen0 when flen == NULL) is the
 * frame's length from its start -- the mbuf data_len that tx_send() sets
 * (tas/fast/fastemu.h:81-95) before tx_flush().  Hints only let the kernel
 * issue a frame's data loads together with its header loads; results always
 * follow ip.total_length, whatever the hint (0 = no hint).  The kernel may read
 * the 16-byte aligned chunks covering [frame, frame + hint), so a hint must
 * not exceed the frame's buffer.  One uniform hint for a uniform-MTU batch of
 * TAS frames (IPv4 at 14 mod 16) selects the fastest kernel. */
int tasx_tcp4_cksum_batch_dev_hint(void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t n,
    uint32_t ip_off, uint32_t l4_off, uint16_t *out, uint32_t flags,
    void *stream);

/* Same, with a room: `room` bytes from every frame's start are mapped and may
 * be read (TAS: the mbuf data room, BUFFER_SIZE = 2048,
 * tas/fast/internal.h:34; 0 = unknown).  room >= l4_off + 18, and in stride
 * mode room <= stride.  A room lets a row issue its loads before it knows its
 * ip.total_length: a batch without per-frame hints whose frames have room for
 * a full MTU (IPv4 at 14 mod 16: room >= 1536 from the 16-byte aligned start)
 * is read at the uniform-hint speed (rows load the whole MTU at once and mask
 * by their own total_length).  Per-frame hints mark a data/ACK mix, whose rows
 * read exactly their hinted bytes instead (whole-room reads would cost every
 * ACK 1.5 KB); a hint beyond the room is not trusted for reads.  Results still
 * follow ip.total_length only. */
int tasx_tcp4_cksum_batch_dev_room(void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t room,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out,
    uint32_t flags, void *stream);

/* Receive-side verification (new behaviour: TAS never verifies RX checksums,
 * tas/fast/fast_flows.c:242-251, and requests no RX offloads,
 * tas/fast/network.c:174).  flags[i] bit 0: the 20-byte IPv4 header folds to
 * 0xffff; bit 1: DPDK (>= 21.11) rte_ipv4_udptcp_cksum_verify() passes, i.e.
 * fold(rte_raw_cksum(L4) + rte_ipv4_phdr_cksum()) == 0xffff (total_length < 20
 * fails); bit 2: IHL != 5 (TAS drops such frames, fast_flows.c:247).
 * Received frames are untrusted: the kernel reads a frame's 20-byte IPv4
 * header and, beyond it, nothing past the frame's bound -- its received length
 * (the hint, below), else the room, else its stride slot (stride mode); a
 * datagram whose ip_off + total_length exceeds the bound fails bit 1 without
 * being read.  Only offsets batches with neither hints nor a room trust
 * total_length (their buffers must hold ip_off + total_length bytes).
 * Asynchronous on `stream`. */
#define TASX_RX_IP_OK 0x1u
#define TASX_RX_L4_OK 0x2u
#define TASX_RX_IHL_NOT5 0x4u
int tasx_tcp4_verify_batch_dev(const void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint8_t *flags, void *stream);
/* Same, with the received frame lengths (the mbuf data_len, flen[i], or flen0
 * for the whole batch when flen == NULL; 0 = none): the read bound above, and
 * a prefetch hint; the flags always follow ip.total_length. */
int tasx_tcp4_verify_batch_dev_hint(const void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t n,
    uint32_t ip_off, uint32_t l4_off, uint8_t *flags, void *stream);
/* Same, with a room (as tasx_tcp4_cksum_batch_dev_room): the read bound of
 * frames without a received length. */
int tasx_tcp4_verify_batch_dev_room(const void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t room,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint8_t *flags, void *stream);

/* Fused TX segment build: the payload copy of
 * flow_tx_segment() -- flow_tx_read() from the flow's circular transmit buffer
 * in the shared-memory region, wrap-around split included
 * (tas/fast/fast_flows.c:833-846, dma_read tas/fast/dma.h:39-53, placement
 * :930-933) -- fused with the tcp_checksums() that follows it (:936 ->
 * :1058-1069), in one pass over the payload.  The host has already filled the
 * headers (:891-928).  Per segment, one 32-byte descriptor: */
typedef struct tasx_tx_seg {
  uint64_t frame_off; /* frame start, offset from `frames` */
  uint64_t tx_base;   /* fs->tx_base: the flow's TX buffer, offset in shm */
  uint32_t tx_len;    /* fs->tx_len */
  uint32_t pos;       /* payload_pos, the read position in the TX buffer */
  uint16_t payload;   /* payload bytes */
  uint16_t hdrs_len;  /* payload offset in the frame (66 in TAS data segments) */
  uint32_t room;      /* bytes from the frame start the build may rewrite (with
                       * their own values past the frame): the mbuf data room,
                       * BUFFER_SIZE in TAS (tas/fast/internal.h:34); 0 = only
                       * [0, hdrs_len + payload).  | TASX_TXSEG_SCRATCH: the
                       * room's bytes past the frame are scratch (an mbuf holds
                       * nothing past data_len) */
} tasx_tx_seg;
/* In tasx_tx_seg.room: the bytes from the frame's end to the end of its
 * 128-byte block (counted from `frames`, within the room) may be overwritten;
 * their contents afterwards are unspecified.  Lets the build write whole
 * blocks: no read of the frame's tail and no partial-line write. */
#define TASX_TXSEG_SCRATCH 0x80000000u
/* For each segment: copy `payload` bytes from shm + tx_base at circular
 * position pos into frame + hdrs_len, then store ip.chksum / tcp.chksum into
 * the frame exactly as tcp_checksums() would over the finished frame (lengths
 * from ip.total_length).  out[i] (optional, 4-byte aligned) = ip.chksum |
 * tcp.chksum << 16.  A descriptor that dma_read()'s assertions would reject
 * (pos >= tx_len with payload > 0, payload > tx_len, tx_base + tx_len >
 * shm_len) or with hdrs_len < l4_off + 20 leaves its frame untouched and gets
 * out[i] = 0, which no valid segment produces (ip.chksum is never 0).
 * shm, frames, segs and out are device (or device-mapped host) pointers;
 * shm_len < 4 GiB (TAS's shared region is far smaller); l4_off >= ip_off + 20.
 * Frames must not overlap.  Besides the payload and the two checksum fields,
 * the header bytes [0, hdrs_len) are rewritten with their own values (whole
 * cache lines avoid HBM read-modify-write), and so are the bytes between the
 * frame's end and the end of its last 16-byte chunk when `room` covers them.
 * TX frames are trusted (TAS's own header code writes ip.total_length =
 * hdrs_len - ip_off + payload, :897): a frame whose total_length claims more
 * than that is summed over what it claims, so its buffer must hold
 * ip_off + total_length bytes.  Asynchronous on `stream`. */
int tasx_tx_segment_batch_dev(const void *shm, uint64_t shm_len, void *frames,
    const tasx_tx_seg *segs, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint32_t *out, void *stream);

/* RX flow lookup: the batch hash-table lookup
 * of fast_flows_packet_fss() (tas/fast/fast_flows.c:1084-1163).  For frame i
 * (ip = frame + ip_off, tcp = frame + l4_off) the key is (local = ip.dest /
 * tcp.dest, remote = ip.src / tcp.src) and its hash flow_hash()
 * (:1078-1082): CRC32C (Castagnoli, SSE4.2 crc32 semantics: no pre/post
 * inversion) with initial value 0 over the 12 bytes ip.dest, ip.src,
 * tcp.dest, tcp.src in packet order.  Up to TASX_FLOWHT_NBSZ entries
 * flowht[(h + j) % ht_entries] are probed in order; an entry matches when it
 * is valid, its flow_hash equals h, and the 4-tuple stored in the flow state
 * of its flow id (low 29 bits) equals the key.  fid_out[i] = that flow id, or
 * TASX_FLOW_NONE (fss[i] = NULL in the reference).  hash_out (optional) gets
 * h.  Layouts are TAS's: flowht = struct flextcp_pl_flowhte {u32 flow_id, u32
 * flow_hash}[ht_entries] (include/tas_memif.h:320-327); flow state i at flowst
 * + i * fs_stride holds local_ip, remote_ip (network order), local_port,
 * remote_port at fs_key_off (struct flextcp_pl_flowst: stride 128, offset 32,
 * tas_memif.h:231-252).  A flow id >= fs_num never matches (the reference
 * would read past the array).  fs_stride and fs_key_off are multiples of 4;
 * flowht is 8-byte and flowst 4-byte aligned.  Asynchronous on `stream`. */
#define TASX_FLOWHT_NBSZ 4u          /* FLEXNIC_PL_FLOWHT_NBSZ */
#define TASX_FLOWHTE_VALID 0x80000000u /* FLEXNIC_PL_FLOWHTE_VALID */
#define TASX_FLOWHTE_POSSHIFT 29     /* FLEXNIC_PL_FLOWHTE_POSSHIFT */
#define TASX_FLOW_NONE 0xffffffffu
int tasx_flow_lookup_batch_dev(const void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    const void *flowht, uint32_t ht_entries, const void *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *hash_out, uint32_t *fid_out, void *stream);

/* One RX pass (ABI 4): tasx_tcp4_verify_batch_dev_room() and
 * tasx_flow_lookup_batch_dev() of the same frames, with the same arguments,
 * read bounds, errors and outputs (flags[i]; fid_out[i], hash_out[i]) as the
 * two calls in turn.  Where the verify call would take a TAS row kernel (IPv4
 * at 14 mod 16, TCP at +20, stride mode or offsets), both run in ONE launch:
 * the grid's first blocks look up 256 frames each (512 with a uniform flen0),
 * each block the frames of the verify blocks on its own XCD, the rest verify,
 * so the lookup's dependent bucket / flow-state loads overlap the checksum
 * loads and the verify rows find each frame's first line in L2 (64K received
 * frames: 1.33x the two calls at half ACKs).
 * Other batches run the two kernels in turn.  The lookup reads the 12 key
 * bytes at ip_off + 12 of every frame, as tasx_flow_lookup_batch_dev does.
 * Asynchronous on `stream`. */
int tasx_rx_batch_dev(const void *base, const uint64_t *off, uint64_t stride,
    const uint32_t *flen, uint32_t flen0, uint32_t room, uint32_t n,
    uint32_t ip_off, uint32_t l4_off, uint8_t *flags,
    const void *flowht, uint32_t ht_entries, const void *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *hash_out, uint32_t *fid_out, void *stream);

/* ---------------------------------------------------------------------- */
/* Per-fast-path-core contexts (one per dataplane_context, no shared state,
 * no locks: tas/fast/fastemu.c:87-91).  A context owns a GPU, streams, pinned
 * host staging and device buffers sized for `max_batch_bytes` per pipeline
 * slot (0 = 64 MiB). */
int tasx_ctx_init(unsigned ctx_id, int device, size_t max_batch_bytes);
int tasx_ctx_destroy(unsigned ctx_id);

/* Host-memory batches, end to end: pinned hipMemcpyAsync H2D of the frames,
 * GPU checksum, D2H of the results, pipelined over the context's slots.
 * Frames are read from [base + off_i, base + off_i + extent) where extent is
 * `stride` (stride mode) -- i.e. whole mbuf data rooms are copied.
 * Register `base` with tasx_host_register (or allocate it with
 * tasx_host_alloc) for full PCIe speed. */
int tasx_tcp4_cksum_batch_host(unsigned ctx_id, void *base, uint64_t stride,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out,
    uint32_t flags);
int tasx_raw_cksum_batch_host(unsigned ctx_id, const void *base,
    uint64_t stride, uint32_t len0, uint32_t n, uint16_t *out);

/* Host-memory batches over scattered packets (ABI 5; SURVEY.md section 8b:
 * "(base, offsets[], lengths[], n) -> u16[n] ... host-pointer variants").
 * TAS's frames are mbufs scattered over a per-core mempool
 * (tas/fast/network.c:320-330) and leave through tx_flush
 * (tas/fast/fastemu.c:544-566); these are the end-to-end forms of the _dev
 * batches for such frames.  Packet i starts at base + off[i], or at the
 * address off[i] when base == NULL (staged form only).  off, len, flen and out
 * are host arrays; results are as the _dev forms'.
 *   staged (flags without TASX_F_ZEROCOPY): the calling thread gathers only
 *     the bytes that are summed (RAW: len_i bytes; TCP4: the 20-byte IPv4
 *     header and max(total_length - 20, 18) L4 bytes) into the context's
 *     pinned staging, one hipMemcpyAsync H2D per chunk, the kernel from HBM,
 *     one D2H of the results; the gather of chunk k + 1 overlaps the GPU's
 *     work on chunk k.
 *   zero-copy (TASX_F_ZEROCOPY): base is pinned (tasx_host_alloc) or
 *     registered (tasx_host_register / tasx_ctx_register_frames) memory and
 *     the kernel reads the packets in place over PCIe, only the 16-byte
 *     aligned chunks that hold summed bytes (so up to 15 bytes past a packet
 *     must be readable); TCP4 with TASX_F_INPLACE stores both fields into the
 *     frames from the GPU.
 * RAW: len[i] (or len0 for all when len == NULL) <= TASX_RAW_MAX_LEN.
 * TCP4: flen (optional) holds frame lengths from the frame start (the mbuf
 * data_len); the zero-copy kernel takes them as per-frame read geometry, as
 * tasx_tcp4_cksum_batch_dev_hint does; results follow ip.total_length.  out
 * (4-byte aligned) may be NULL with TASX_F_INPLACE. */
int tasx_tcp4_cksum_batch_host_offs(unsigned ctx_id, void *base,
    const uint64_t *off, const uint32_t *flen, uint32_t n, uint32_t ip_off,
    uint32_t l4_off, uint16_t *out, uint32_t flags);
int tasx_raw_cksum_batch_host_offs(unsigned ctx_id, const void *base,
    const uint64_t *off, const uint32_t *len, uint32_t len0, uint32_t n,
    uint16_t *out, uint32_t flags);

/* The calling thread's context: TAS runs one dataplane_context per fast-path
 * thread (dataplane_loop, tas/fast/fastemu.c:142), so the thread that will call
 * tcp_checksums() binds its context once, and the per-frame calls pass
 * TASX_CTX_SELF instead of a context id (tcp_checksums() and
 * fast_flows_kernelxsums() have no ctx parameter, fast_flows.c:1058,1071).
 * Every call that takes a ctx_id accepts TASX_CTX_SELF. */
#define TASX_CTX_SELF 0xffffffffu
int tasx_set_thread_ctx(unsigned ctx_id);
/* the calling thread's context id, or -EINVAL if none is bound */
int tasx_thread_ctx(void);

/* Deferred per-frame surface.  tasx_tcp_checksums() has the reference's
 * argument list plus the context id; it only records the frame (no device
 * work, safe under the per-flow spinlock).  tasx_flush() -- called where TAS
 * calls tx_flush(), outside any flow lock -- checksums every recorded frame
 * on the GPU and stores ip.chksum / tcp.chksum into the frames before it
 * returns.  Frames must stay valid and unmodified until then.
 * Recorded frames are read up to ip_off + ip.total_length.  tasx_flush
 * gathers the frames into pinned staging, which the kernel reads directly;
 * results land in pinned memory.  It then waits by spinning on a completion
 * word that a one-lane kernel posts after the checksum launch, not in
 * hipStreamSynchronize.  The spin polls the stream now and then, so a failed
 * stream returns -EIO. */
int tasx_tcp_checksums(unsigned ctx_id, void *nbh, void *p, uint32_t ip_s,
    uint32_t ip_d, uint16_t l3_paylen);
int tasx_fast_flows_kernelxsums(unsigned ctx_id, void *nbh, void *p);
int tasx_defer_tcp4(unsigned ctx_id, void *frame, uint16_t ip_off,
    uint16_t l4_off);
/* frames recorded and not yet flushed */
int tasx_pending(unsigned ctx_id);
int tasx_flush(unsigned ctx_id);

/* Asynchronous flushes: tasx_flush() is tasx_flush_submit() + tasx_flush_wait().
 * A GPU round trip (launch + completion) costs ~13 us whatever the batch size,
 * far more than a core's CPU checksums of one tx_flush batch (DESIGN.md
 * section 5.1); split, a fast-path core submits a batch, keeps polling its
 * queues, and hands the batch's frames to the NIC once its ticket completes,
 * with up to 4 batches in flight per context.
 *   tasx_flush_submit: launches every recorded frame (one or more flushes) and
 *     returns in *ticket the ticket of the last one (the last submitted ticket
 *     when nothing was recorded; 0 before the first flush).  Blocks only when
 *     4 flushes are already in flight (it completes the oldest).
 *   tasx_flush_poll: 1 when flush `ticket` and every earlier one are complete
 *     (both checksum fields stored in their frames), 0 if not yet; never
 *     blocks.  Completes flushes in ticket order.
 *   tasx_flush_wait: spins until flush `ticket` is complete.
 * Frames must stay valid and unmodified until their ticket completes.
 * Tickets count up from 1 and wrap at 2^32 (comparisons are wrap-safe; after
 * the wrap 0 is an ordinary ticket, and flush t always uses slot t % 4). */
int tasx_flush_submit(unsigned ctx_id, uint32_t *ticket);
int tasx_flush_poll(unsigned ctx_id, uint32_t ticket);
int tasx_flush_wait(unsigned ctx_id, uint32_t ticket);

/* Zero-copy frames: declare the host region the context's frames live in
 * (TAS: the per-core mbuf mempool, tas/fast/network.c:320-330).  It is pinned
 * with hipHostRegister unless it already is (tasx_host_alloc).  A flush whose
 * frames all lie in the region (TAS layout, tcp = ip + 20) is done without any
 * copy: the kernel reads the frames over PCIe and stores both checksum fields
 * in place.  Other flushes take the staged path. */
int tasx_ctx_register_frames(unsigned ctx_id, void *base, size_t bytes);
/* counts of zero-copy and staged flushes since tasx_ctx_init */
int tasx_ctx_stats(unsigned ctx_id, uint32_t *zerocopy_flushes,
    uint32_t *staged_flushes);

/* Shared feeder: one thread per GPU serves the zero-copy flushes of every
 * attached context with one launch per sweep, so the launch and completion
 * round trip is paid once per sweep by the feeder's core, not once per flush
 * by each fast-path core.  An attached context's tasx_flush_submit() hands its
 * batch over by copying the frame pointers into its own lock-free queue (8
 * batches deep; it spins only when all 8 are waiting) -- no HIP call on the
 * fast-path core; tasx_flush_poll/_wait see the feeder's completions, in
 * ticket order as before.  A batch with a frame outside the context's
 * registered region (or without 14 bytes before its IPv4 header there) is
 * flushed by the context itself after its feeder tickets complete.
 *   tasx_feeder_start(device): the feeder thread for `device` (one per GPU)
 *   tasx_ctx_use_feeder(ctx, 1 / 0): attach (needs a running feeder and a
 *     registered frame region) / detach (waits for the context's tickets)
 *   tasx_feeder_stop(device): -EBUSY while contexts are attached
 *   tasx_feeder_stats: sweeps launched and frames done since start
 *   tasx_ctx_feeder_flushes: batches the context handed to the feeder */
int tasx_feeder_start(int device);
int tasx_feeder_stop(int device);
int tasx_feeder_stats(int device, uint64_t *sweeps, uint64_t *frames);
int tasx_ctx_use_feeder(unsigned ctx_id, int on);
int tasx_ctx_feeder_flushes(unsigned ctx_id, uint32_t *feeder_flushes);

/* Flush server (ABI 6): a persistent kernel per GPU takes the flushes of
 * every attached context from pinned host memory, so a fast-path core's
 * tasx_flush_submit(), _poll() and _wait() make NO HIP call (the server's
 * epoch thread watches the kernel) and the GPU pays no launch per batch.
 * Each context has a ring of TASX_SRV_RING (8) descriptor slots, up to 64
 * frames each: submit writes the frames' offsets in the context's registered
 * region and their ip.total_length into the next slot, the header last, and
 * returns; two workgroups of the server kernel poll that ring over PCIe
 * (each every other position: one takes the next batch while the other sums
 * the current one, and they read frames in turn, which bounds what a busy
 * server costs other device work on the GPU), sum the frames in place and
 * store both checksum fields into them, then post each slot's done word,
 * which tasx_flush_poll/_wait
 * reap in position order (ticket order as before; submit spins only when 8
 * batches are in flight).  A ring idle for 2 ms is polled by its header alone.  Frames
 * the server does not take -- outside the registered region, not TAS layout,
 * a frame start (ip - 14) not 16-byte aligned, or total_length outside
 * [38, 1522] -- are flushed by the context itself after its server tickets.
 * Frames must stay unmodified until their ticket completes; a frame whose
 * total_length changed meanwhile is left alone, and from then on the
 * context's poll/wait return -EIO, until tasx_ctx_use_server(ctx, 0), which
 * still detaches and returns -EIO once.  The TAS path this replaces: tx_flush
 * (tas/fast/fastemu.c:544-566) after tcp_checksums (fast_flows.c:1058-1069).
 *   tasx_server_start(device): launch the server kernel (2 * TASX_MAX_CTX
 *     workgroups of 1024 threads) and its epoch thread.  (ABI 10) The kernel
 *     runs in epochs of 5 ms: each launch leaves at its rings' positions after
 *     its period and the epoch thread keeps the next launch queued behind it
 *     on the server's stream, so a HIP call elsewhere in the process that
 *     waits for all of the device's work -- hipDeviceSynchronize
 *     (torch.cuda.synchronize), the frees (hipFree, hipHostFree,
 *     hipHostUnregister, torch.cuda.empty_cache), synchronous copies, waits on
 *     the null stream -- waits for the epochs queued when it was made (about
 *     10 ms), not for the server's stop; and a process that is gone queues no
 *     further epoch (INTEGRATION.md 4f lists the calls, measured)
 *   tasx_server_stop(device): -EBUSY while contexts are attached; waits up
 *     to 5 s for the kernel to leave, else -EIO
 *   tasx_ctx_use_server(ctx, 1 / 0): attach (needs a running server and a
 *     registered frame region below 4 GiB; not together with the feeder) /
 *     detach (waits for the context's tickets; the ring's position is kept
 *     for the next context attached under that id)
 *   While a server runs, HIP's frees wait for its queued epochs:
 *     tasx_ctx_destroy hands the context's memory to the server (released at
 *     its stop), and tasx_host_free, tasx_host_unregister, tasx_dev_free and
 *     tasx_feeder_stop return -EBUSY (a fast-path core must never wait on
 *     the GPU); a pause lets every free through at once:
 *   tasx_server_pause(device): the kernel leaves at its rings' current
 *     positions (a batch being summed is finished first; at most 5 s, else
 *     -EIO: the stop word stays, so a kernel that leaves later is seen gone
 *     by the contexts, tasx_take_unfinished); contexts stay attached, submit as before
 *     (the slots wait in the rings; a full ring waits inside the call) and
 *     poll "not done"; frees do not wait, and the four calls above work.
 *     -EALREADY when paused already, -EIO after an abort or a kernel exit.
 *     Detaching (tasx_ctx_use_server(ctx, 0)) waits for the resume.
 *   tasx_server_resume(device): launch the kernel again at those positions
 *     (-EINVAL when not paused); the paused batches are served from there.
 *     A server may also be stopped (once detached) or aborted while paused.
 *   tasx_server_stats: batches and frames submitted since start
 *   tasx_server_epochs (ABI 10): epochs completed, and the epoch thread's
 *     waits longer than 50 ms (a HIP call of its, or an epoch overdue: another
 *     thread in a device-wide wait) with the longest in ms; the first is also
 *     reported once on stderr (TASX_SERVER_QUIET=1 silences it)
 *   tasx_ctx_server_flushes: batches the context handed to the server */
/* (ABI 7) The fused TX segment build through the flush server (the copy of
 * flow_tx_segment's payload from the app's TX buffer plus tcp_checksums,
 * tas/fast/fast_flows.c:930-936, at tx_flush time with no HIP call): the
 * fast-path core fills the headers as now and, instead of dma_read +
 * tcp_checksums, hands each segment's descriptor (tasx_tx_seg; frame_off
 * from the registered frame region's start, tx_base from the registered
 * shared-memory region's start) to tasx_server_tx_segments, which returns a
 * ticket (tasx_flush_poll / _wait, in order with the context's other
 * tickets).  The server gathers the payload and writes it into the frame,
 * both checksums included, over PCIe.  TAS layout (ip at +14, tcp at +34),
 * frame starts 16-byte aligned, hdrs_len in [54, 240], room below 32 KiB,
 * frames (and their rooms) inside the frame region: else -EINVAL and nothing
 * is submitted.  Descriptors dma_read() would reject leave their frame as it
 * is (tasx_tx_segment_batch_dev).  Up to 41 segments go in one of the ring's
 * 8 slots (a run of equal hdrs_len and room: TAS's 32-segment flush takes one
 * slot); with every slot out, the call waits inside for the oldest one to
 * finish.
 *   tasx_ctx_register_shm(ctx, shm, bytes): the app's shared-memory region
 *     (pinned and mapped here unless it already is; below 4 GiB) */
int tasx_ctx_register_shm(unsigned ctx_id, void *shm, size_t bytes);
int tasx_server_tx_segments(unsigned ctx_id, const tasx_tx_seg *segs, uint32_t n, uint32_t *ticket);
int tasx_server_start(int device);
int tasx_server_stop(int device);
int tasx_server_pause(int device);
int tasx_server_resume(int device);
int tasx_server_stats(int device, uint64_t *batches, uint64_t *frames);
int tasx_server_epochs(int device, uint64_t *epochs, uint32_t *slow_waits, uint32_t *max_wait_ms);
int tasx_ctx_use_server(unsigned ctx_id, int on);
int tasx_ctx_server_flushes(unsigned ctx_id, uint32_t *server_flushes);

/* ---------------------------------------------------------------------- */
/* Error recovery (ABI 8).  SURVEY.md section 8b: TAS's per-frame calls cannot
 * fail, so a batch whose GPU work fails must not drop frames.  libtasx still
 * computes nothing on the CPU; instead it hands the unfinished frames back and
 * the caller finishes them with TAS's own CPU path -- the #else branch of
 * tcp_checksums (rte_ipv4_cksum / rte_ipv4_udptcp_cksum,
 * tas/fast/fast_flows.c:1065-1067) for frames, flow_tx_read + tcp_checksums
 * (fast_flows.c:930-936) for TX segments -- and keeps running
 * (INTEGRATION.md section 3).
 *   tasx_take_unfinished(ctx, frames, max): valid at any time, meant after any
 *     call on the context returned non-zero.  The first call settles the
 *     context: it waits for in-flight work whose path is still healthy, then
 *     collects every recorded frame whose checksum fields the GPU did not
 *     store -- batches of a server whose kernel has gone (stopped by
 *     tasx_server_abort, an epoch that failed, a fault), of a failed feeder, of a
 *     failed or stalled stream, and frames recorded but not submitted -- marks
 *     every ticket complete, and detaches the context from a dead server or
 *     feeder.  Each call then writes up to max of them ({ip, l4} as recorded)
 *     and returns how many, 0 once none are left; the context is usable again
 *     (pending 0, every ticket polled complete).  -ENOMEM (once, after the
 *     rest) if the library could not allocate room to keep some of them.  A GPU that wrote a field
 *     after all is harmless: the caller recomputes both fields from zero.
 *   tasx_take_unfinished_segs(ctx, segs, max): the same for TX segments given
 *     to tasx_server_tx_segments (descriptors as submitted; after an -EIO
 *     from that call, its segments not yet handed to the server too).  Call
 *     tasx_take_unfinished first (it settles the context).
 *   tasx_server_abort(device): stops the server kernel even with contexts
 *     attached (a watchdog, or TAS leaving the GPU path); their outstanding
 *     batches become unfinished, their next poll/wait/submit returns -EIO, and
 *     tasx_take_unfinished (or tasx_ctx_use_server(ctx, 0), which detaches
 *     from a gone kernel with -EIO) hands them back; tasx_server_stop then
 *     releases it once every context has detached.
 * A frame the server left alone because its total_length changed after
 * submission (the sticky -EIO above) is not returned: the caller broke the
 * deferred contract, and the frame's bytes are no longer what was submitted. */
typedef struct tasx_frame_ref {
  void *ip; /* the IPv4 header, as recorded */
  void *l4; /* the TCP header */
} tasx_frame_ref;
int tasx_take_unfinished(unsigned ctx_id, tasx_frame_ref *frames, uint32_t max);
int tasx_take_unfinished_segs(unsigned ctx_id, tasx_tx_seg *segs, uint32_t max);
int tasx_server_abort(int device);

/* ---------------------------------------------------------------------- */
/* Kernel selection, for tests.  Per calling thread (TAS runs one
 * fast-path core, i.e. one context, per thread); set it before launching.
 *   0 automatic: RAW -> 7 with per-packet lengths, else raw_sad_kernel; TCP4 ->
 *     6 when it applies, else 3 for the TAS layout in stride mode with a hint,
 *     else 2
 *   2 raw_sad_kernel (general form) / tcp4_frame_kernel (any layout)
 *   3 tcp4_tas_kernel (TAS layout, stride mode; falls back to 2)
 *   6 tcp4_tas14_kernel: TAS layout with the IPv4 header at 14 mod 16 from a
 *     16-byte aligned frame start.  Stride mode with one uniform hint flen0
 *     (ip_off + 64 <= flen0, the datagram within 96 chunks: uniform-MTU
 *     batches up to ip.len 1522) fixes every row's geometry; otherwise (stride
 *     mode or an offsets array, no uniform hint) each row takes its extent from
 *     its own ip.total_length, loading ahead as far as the room allows (see
 *     tasx_tcp4_cksum_batch_dev_room); rows it cannot take go to 2's bodies.
 *     Otherwise as 0.  RAW: as 0 without lengths.
 *   7 RAW: raw_wave_kernel (a wave's 4 packets summed as one chunk sequence:
 *     mixed lengths keep every lane loading); TCP4 as 0
 * Any other number is rejected with -EINVAL (the comparison variants of
 * rounds 1-5 were retired in round 6). */
int tasx_set_kernel_variant(int variant);
/* Name of the kernel the calling thread's last batch call launched (its entry
 * kernel; rows it cannot take are redone inside it by a general body), "" if
 * none.  For tests that assert which kernel a call ran. */
const char *tasx_last_kernel(void);

/* ---------------------------------------------------------------------- */
/* Memory helpers (plumbing for callers without their own HIP code). */
void *tasx_host_alloc(size_t bytes);          /* pinned host memory */
int tasx_host_free(void *p);
int tasx_host_register(void *p, size_t bytes);  /* pin existing memory */
/* the device's address of pinned host memory (zero-copy kernel access) */
void *tasx_host_device_pointer(void *p);
int tasx_host_unregister(void *p);
void *tasx_dev_alloc(int device, size_t bytes);
int tasx_dev_free(void *p);
int tasx_memcpy_h2d(void *dst, const void *src, size_t bytes);
int tasx_memcpy_d2h(void *dst, const void *src, size_t bytes);
int tasx_stream_sync(void *stream);

#ifdef __cplusplus
}
#endif
#endif
