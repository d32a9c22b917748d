/* tasx_kernels.h -- internal interface between the C host layer (tasx_host.c)
 * and the HIP kernels (xsum_kernels.hip).  Plain C structs, passed by value
 * to the kernels. */
#ifndef TASX_KERNELS_H_
#define TASX_KERNELS_H_

#include <stdint.h>

#include "../../include/tasx_xsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* library-internal: not exported from libtasx.so */
#define TASX_INTERNAL __attribute__((visibility("hidden")))

typedef struct tasx_raw_params {
  const uint8_t *base;   /* device pointer */
  const uint64_t *off;   /* device, n entries, or NULL -> i * stride */
  const uint32_t *len;   /* device, n entries, or NULL -> len0 */
  uint16_t *out;         /* device, n entries */
  uint64_t stride;
  uint32_t len0;
  uint32_t n;
  uint32_t xrun;         /* XCD-ordered grid (xcd_run), set by the launcher */
} tasx_raw_params;

typedef struct tasx_tcp4_params {
  uint8_t *base;         /* device pointer to frames */
  const uint64_t *off;   /* device, n entries, or NULL -> i * stride */
  uint16_t *out;         /* device, 2n entries (4-byte aligned) or NULL */
  uint64_t stride;
  uint32_t n;
  uint32_t ip_off;       /* IPv4 header offset in the frame (TAS: 14) */
  uint32_t l4_off;       /* TCP header offset in the frame (TAS: 34) */
  uint32_t flags;        /* TASX_F_* */
  const uint32_t *flen;  /* device, n frame-length hints (bytes from the frame
                          * start, the mbuf data_len), or NULL -> flen0 */
  uint32_t flen0;        /* uniform hint; 0 = none */
  uint32_t room;         /* bytes from each frame's start that may be read (the
                          * mbuf data room); 0 = unknown */
  /* the RX flow lookup fused into verification (tasx_rx_batch_dev) */
  const uint32_t *flowht; /* {flow_id, flow_hash} pairs */
  const uint8_t *flowst;
  uint32_t *fid_out;
  uint32_t *hash_out;     /* or NULL */
  uint32_t ht_entries;
  uint32_t fs_num;
  uint32_t fs_stride;
  uint32_t fs_key_off;
  uint32_t xrun;          /* XCD-ordered grid (xcd_run), set by the launcher */
} tasx_tcp4_params;

typedef struct tasx_txseg_params {
  const uint8_t *shm;      /* device view of the shared-memory region */
  uint64_t shm_len;
  uint8_t *frames;         /* device pointer; segment frames at frame_off */
  const tasx_tx_seg *segs; /* device, n descriptors (16-byte aligned) */
  uint32_t *out;           /* device, n entries, or NULL */
  uint32_t n;
  uint32_t ip_off;
  uint32_t l4_off;
} tasx_txseg_params;

typedef struct tasx_flow_params {
  const uint8_t *base;     /* device pointer to RX frames */
  const uint64_t *off;     /* device, n entries, or NULL -> i * stride */
  uint64_t stride;
  const uint32_t *flowht;  /* {flow_id, flow_hash} pairs */
  const uint8_t *flowst;
  uint32_t *hash_out;      /* or NULL */
  uint32_t *fid_out;
  uint32_t n;
  uint32_t ip_off;
  uint32_t l4_off;
  uint32_t ht_entries;
  uint32_t fs_num;
  uint32_t fs_stride;
  uint32_t fs_key_off;
} tasx_flow_params;

/* The persistent flush server (server_kernels.hip): one block of coherent
 * pinned host memory per GPU, host-written lines apart from GPU-written ones.
 *   [TASX_SRV_CTL]     u64: stop (low word, host); the high word is unused
 *   [TASX_SRV_DONE(r)] ring r's GPU-written line: u32 done[TASX_SRV_RING]
 *                      (done[p mod RING] = p + 1 once position p is finished),
 *                      u32 error at word TASX_SRV_ERRW (sticky)
 *   [TASX_SRV_WGL(b)]  workgroup b's line: u32 at TASX_SRV_POSW(b) = the
 *                      ring position it polled when it left, u64 at
 *                      TASX_SRV_TACT(b) = the wall-clock time of its last
 *                      batch (the next epoch's launch, and a paused
 *                      server's, resumes there: tasx_server_resume,
 *                      server_epochs)
 *   [TASX_SRV_SLOTP(r, p)] ring r, position p: a 1 KiB descriptor slot,
 *     u64 h0 = n | min(region bytes, 2^32 - 1) << 16 | tag << 48,
 *     u64 h1 = region device address (48 bits) | tag << 48,
 *     then n <= TASX_SRV_FB entries u64 = frame offset in the region (32
 *     bits) | ip.total_length << 32 | tag << 48,
 *   tag = (p + 1) mod 2^16; the host writes the entries (all TASX_SRV_FB of
 *   them: the unused ones carry the tag alone), then h1, then h0.
 * Workgroup k of ring r's P.k takes its positions p = k mod P.k. */
#define TASX_SRV_RING 8u   /* slots per ring */
/* TX segment slots (tasx_server_tx_segments): h0's n field | TASX_SRV_SEG, at
 * most TASX_SRV_SEGS segments sharing one hdrs_len and room; entry 0 = shm
 * device address (48 bits), entry 1 = shm_len (32) | ip_off << 32 | l4_off <<
 * 40, entry 2 = hdrs_len | room16 << 16 (room & 0x7fff, bit 15 =
 * TASX_TXSEG_SCRATCH), then per segment 3 entries: frame_off (32) | payload
 * << 32, pos (32) | (tx_len & 0xffff) << 32, tx_base (32) | (tx_len >> 16) <<
 * 32; every entry | tag << 48.  Round 5: a TX slot uses the whole 1 KiB
 * (TASX_SRV_WORDS entries, 41 segments: TAS's 32-segment flush in one slot);
 * the server reads the entries past TASX_SRV_FB in a second round trip, once
 * the first has shown a taken header (the host wrote them before it). */
#define TASX_SRV_SEG 0x8000u
#define TASX_SRV_WORDS 126u /* entry words in a 1 KiB slot */
#define TASX_SRV_SEGS 41u   /* (TASX_SRV_WORDS - TASX_SRV_SEGW0) / 3 */
#define TASX_SRV_SEGW0 3u /* entry of segment 0's first word */
#define TASX_SRV_FB 64u    /* frames per slot */
#define TASX_SRV_KMAX 8u   /* workgroups per ring, a divisor of TASX_SRV_RING */
#define TASX_SRV_SLOT 1024u
#define TASX_SRV_HDR 16u
#define TASX_SRV_CTL 0u
#define TASX_SRV_DONE(r) (128u * (1u + (r)))
#define TASX_SRV_ERRW TASX_SRV_RING
#define TASX_SRV_WGL(b) (4096u + 64u * (b))
#define TASX_SRV_POSW(b) (TASX_SRV_WGL(b))
#define TASX_SRV_TACT(b) (TASX_SRV_WGL(b) + 8u)
#define TASX_SRV_RINGS (4096u + 64u * TASX_MAX_CTX * TASX_SRV_KMAX)
#define TASX_SRV_SLOTP(r, p) (TASX_SRV_RINGS + ((r) * TASX_SRV_RING + (p) % TASX_SRV_RING) * TASX_SRV_SLOT)
#define TASX_SRV_BYTES (TASX_SRV_RINGS + TASX_MAX_CTX * TASX_SRV_RING * TASX_SRV_SLOT)

typedef struct tasx_srv_params {
  uint8_t *mem;          /* device view of the server's pinned block (the GPU-written lines) */
  uint8_t *ring;         /* device view of the host-written lines (control word, slots): mem */
  uint64_t period_ticks; /* an epoch: wall-clock ticks from its launch after which each workgroup
                            leaves at its next poll (the host has the next epoch queued behind it) */
  uint64_t hot_ticks;    /* ticks after a batch during which a ring is polled without backoff */
  uint64_t cold_ticks;   /* ticks after a batch from which only the header is polled */
  uint32_t k;            /* workgroups per ring (a divisor of TASX_SRV_RING, <= TASX_SRV_KMAX) */
  uint32_t resume;       /* 0: every ring at position 0 (a zeroed block); 1: each workgroup at the
                            position it left at (TASX_SRV_POSW): every epoch after the first */
  uint32_t *tok;         /* device memory, one 128-byte line per ring (TASX_SRV_TOKW words apart):
                            the ring position whose frames may be read next (k > 1) */
} tasx_srv_params;
#define TASX_SRV_TOKW 32u

/* variant: see tasx_set_kernel_variant (0 = automatic).  0 on success. */
TASX_INTERNAL int tasx_launch_raw(const tasx_raw_params *p, int variant, void *stream);
TASX_INTERNAL int tasx_launch_tcp4(const tasx_tcp4_params *p, int variant, void *stream);
/* receive-side verification; p->out points to n flag bytes */
TASX_INTERNAL int tasx_launch_tcp4_verify(const tasx_tcp4_params *p, int variant, void *stream);
/* RX verification (flags to p->out) and the flow lookup (p->fid_out,
 * p->hash_out) of the same frames: one pass where the row kernel takes the
 * batch, else the two kernels in turn */
TASX_INTERNAL int tasx_launch_tcp4_rx(const tasx_tcp4_params *p, int variant, void *stream);
/* RX flow lookup (flow_kernels.hip) */
TASX_INTERNAL int tasx_launch_flow_lookup(const tasx_flow_params *p, int variant, void *stream);
/* one-lane kernel storing seq into *word (pinned host memory, device view)
 * with system-scope release, after everything before it on the stream */
TASX_INTERNAL int tasx_launch_post_done(uint32_t *word, uint32_t seq, void *stream);
/* offload branch of tcp_checksums: pseudo-header sums into tcp.chksum */
TASX_INTERNAL int tasx_launch_tcp4_offload(const tasx_tcp4_params *p, void *stream);
/* fused TX segment build (txseg_kernels.hip) */
TASX_INTERNAL int tasx_launch_txseg(const tasx_txseg_params *p, void *stream);
/* the flush server: TASX_MAX_CTX * p->k workgroups, p->k per ring; -1 for a bad p->k */
TASX_INTERNAL int tasx_launch_server(const tasx_srv_params *p, void *stream);
/* record the name of the kernel the calling thread launches (tasx_last_kernel) */
TASX_INTERNAL void tasx_note_kernel(const char *name);

/* test support for the comparison build's export tasx_ab_ctx_set_tickets:
 * library-internal, never exported */
TASX_INTERNAL int tasx_ctx_set_tickets_internal(unsigned ctx_id, uint32_t start);

#ifdef __cplusplus
}
#endif
#endif
