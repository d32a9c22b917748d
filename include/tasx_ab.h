/*
 * tasx_ab.h -- extra entry points of libtasx's comparison build
 * (tas_amd/_lib/libtasx_ab.so: the product's own objects plus
 * tas_amd/csrc/ab/).  It holds the kernels bench.py prices the product
 * against -- access patterns with the arithmetic removed, pure streaming reads
 * and copies -- the round-2 TX segment kernel the tests run beside the
 * product, and one test hook.  It changes nothing in the product's paths:
 * everything in tasx_xsum.h is exported as well and behaves as in libtasx.so.
 * The kernel variants of rounds 1-5 (the numbers in profiles/r01_* and
 * profiles/r02-r05/INDEX.md) were retired in round 6.
 */
#ifndef TASX_AB_H_
#define TASX_AB_H_

#include "tasx_xsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The RX flow lookup's bare access pattern (tasx_flow_lookup_batch_dev's
 * frame-header -> bucket -> flow-key chain with no hashing or key compare):
 * the ceiling that chain allows, timed by bench.py beside the lookup. */
int tasx_ab_flow_pattern(const void *base, uint64_t stride, uint32_t n, uint32_t ip_off,
    const void *flowht, uint32_t ht_entries, const void *flowst, uint32_t fs_num, uint32_t fs_stride,
    uint32_t fs_key_off, uint32_t *out, void *stream);

/* The headline kernel's access pattern (tcp4_tas14_kernel<hint>: same rows,
 * loads, result store and residency) with no checksum logic -- the ceiling
 * that pattern allows, timed by bench.py beside the headline.  Uniform-hint
 * stride-mode TAS batches only (-EINVAL otherwise); out[i] is not a checksum. */
int tasx_ab_tcp4_pattern(const void *base, uint64_t stride, uint32_t n, uint32_t flen0, uint32_t ip_off,
    uint32_t *out, void *stream);

/* The data/ACK mix's access pattern (tcp4_tas14_kernel<hints>, per-frame hints
 * as the row geometry) with no checksum logic: chain = 0 reads what the
 * product reads, chain = 1 only each row's hint and the chunk holding its
 * frame's end (the row's dependent chain, almost no bytes).  bench.py prices
 * the flush_mix and rx_verify_mix legs against them (their latency roofline).
 * Stride-mode TAS batches (ip_off 14 mod 16, 16-byte aligned rooms >= 1536 B,
 * n * stride < 4 GiB; -EINVAL otherwise); out[i] is not a checksum. */
int tasx_ab_tcp4_mix_pattern(const void *base, uint64_t stride, uint32_t n, const uint32_t *flen,
    uint32_t ip_off, int chain, uint32_t *out, void *stream);

/* The device's read+write streaming rate: a grid-stride copy of `bytes` (16-byte
 * multiple, 16-byte aligned), one non-temporal 16-byte load and store per
 * lane -- the TX segment build's ceiling, timed by bench.py. */
int tasx_ab_stream_copy(const void *src, void *dst, size_t bytes, void *stream);

/* A pure streaming read of `bytes` (1 KiB multiple, 16-byte aligned): path 0
 * register loads (8 KiB per block, two non-temporal 16-byte loads per lane);
 * path 2 + k (k = 0..11): the same with the blocks XCD-ordered in runs of 2^k
 * (xcd_run).  Path 1 (LDS-DMA staging) was deleted in round 6: -22.  bench.py
 * times them beside each leg and reports the fastest as its read ceiling.
 * sink: a device word (never written for real data). */
int tasx_ab_stream_read(const void *src, size_t bytes, int path, uint32_t *sink, void *stream);

/* The TX segment build's kept forms over a batch (the arguments of
 * tasx_tx_segment_batch_dev; TAS's layout, ip_off 14 and l4_off 34, only):
 * form 30 = tx_segment_tas_kernel, the round-2 product (one unaligned
 * non-temporal window load per frame chunk); form 40 = the product's access
 * pattern alone (its aligned loads and whole-block stores with no realignment
 * or sums: timing only, frames and results wrong) -- bench.py's tx_segment
 * pattern ceiling.  -22 for anything else. */
int tasx_ab_tx_segment_form(int form, const void *shm, uint64_t shm_len, void *frames, const tasx_tx_seg *segs,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint32_t *out, void *stream);

/* Test hook: restart a context's flush tickets at `start` (nothing pending or
 * in flight, no feeder), so a test can run flushes across the 2^32 wrap. */
int tasx_ab_ctx_set_tickets(unsigned ctx_id, uint32_t start);

#ifdef __cplusplus
}
#endif
#endif
