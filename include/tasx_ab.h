/*
 * tasx_ab.h -- extra entry points of the A/B build of libtasx
 * (tas_amd/_lib/libtasx_ab.so: the product's own objects plus
 * tas_amd/csrc/ab/, which hooks its variants and knobs into the product
 * launchers through tasx_ext; used by tools/, bench.py's live ceilings and the
 * variant tests, never by the product path).  Everything in tasx_xsum.h is
 * exported as well, and tasx_set_kernel_variant() also accepts:
 *   1  the first-generation group-per-packet kernels (raw_cksum_kernel,
 *      tcp4_cksum_kernel)
 *   2  RAW: raw_group_kernel (64-bit dword accumulators)
 *   4  tcp4_tas_kernel with wave-timeline stamps into the diag buffer
 *   5  tcp4_tas_kernel with 32-lane groups (TCP4 only)
 *   8  tcp4_wave_kernel: a wave's 4 frames flattened over their hinted
 *      datagrams (TCP4; needs l4_off == ip_off + 20)
 *   9, 10, 11  tcp4_tas14_kernel without a uniform hint forced into its
 *      total_length-first / head-5 / whole-room row mode where the room allows
 *   12, 13, 14  tcp4_tas14_rows_kernel: persistent total_length-first rows
 *      (resident grid / 2 / 4 frames per row; stride mode, no uniform hint)
 *   15..18  tcp4_tas14_kernel<tl_first> in blocks of 64 / 128 / 512 / 1024
 *   19  tcp4_mix_kernel (16 frames per wave, short frames one per lane, data
 *      frames compacted onto rows; TASX_MIX_F8=1: 8 frames per wave) where a
 *      room of 80 B allows; measured slower than the default for data/ACK
 *      mixes
 *   20  tcp4_tas14_kernel<hints> forced (the per-frame-hint default)
 *   21  tcp4_tas14_kernel<hints_pred>: the same with lanes past a row's last
 *      chunk loading nothing (needs per-frame hints)
 *   22..25  tcp4_tas14_kernel<hints> in blocks of 64 / 128 / 512 / 1024
 *   26  tasx_rx_batch_dev with the flow lookup inside the verify rows
 *      (tcp4_tas14_kernel<...,flow_row>) instead of in lookup blocks ahead of
 *      the verify blocks; slower wherever ACKs are present
 *   28  tcp4_tas14_kernel<hints_sorted>: per-frame hints, a block's rows take
 *      its frames long ones first, so waves of short frames load one chunk
 *   27, 29..43  RX-pass and row forms (tasx_rx_batch_dev split grids, lookup
 *      placements, timing ablations; profiles/r03, profiles/r04)
 *   45..48  RAW rows of 32 / 64 lanes and without the residency cap
 * The environment knobs, read once at load: TASX_TAS14_*_LDS and
 * TASX_WAVE_TCP4_LDS (KiB of reserved LDS for the A/B variants' launches),
 * TASX_XRUN (XCD order of every grid), TASX_FEEDER_SWEEPS, and for the flush
 * server TASX_SRV_K (workgroups per ring), TASX_SRV_HOT_US / TASX_SRV_COLD_US
 * (poll backoff), TASX_SRV_SEGMAX (TX segments per slot), TASX_SRV_DIAG (its
 * timing form: tasx_ab_server_diag); read at each use: TASX_TXSEG_DEBUG (TX
 * segment diagnostics kernels, at each TX launch; 29 = tx_segment_wave_kernel,
 * one segment per wave from aligned loads) and TASX_SRV_ACQ (at each server
 * start: 1 / 2 = the per-batch acquire at agent scope / left out, for pricing
 * the server only -- not correct forms).
 */
#ifndef TASX_AB_H_
#define TASX_AB_H_

#include "tasx_xsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device buffer for variant 4: 4 x u64 s_memrealtime (100 MHz) stamps per
 * wave.  NULL disables. */
int tasx_set_diag_buffer(void *dev_buf);

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

/* A pure streaming read of `bytes` (1 KiB multiple, 16-byte aligned) by one of
 * the two load paths (round 4): path 0 register loads (8 KiB per block, two
 * non-temporal 16-byte loads per lane), path 1 LDS-DMA (global_load_lds_dwordx4
 * nt into a 4-slot ring per wave); path 2 + k (round 5): the register path
 * with the blocks XCD-ordered in runs of 2^k (xcd_run).  bench.py times them
 * beside each leg and reports the fastest as its read ceiling.  sink: a device
 * word (never written for real data). */
int tasx_ab_stream_read(const void *src, size_t bytes, int path, uint32_t *sink, void *stream);

/* XCD order of every grid launch_groups makes (round 5): xrun 0 = grid order,
 * k > 0 = runs of 2^(k-1) blocks per XCD (xcd_run), -1 = the product's rule
 * (runs of 256 from 16,384 blocks).  Default: TASX_XRUN, else -1. */
int tasx_ab_set_xrun(int xrun);

/* The flush server's timing sums for ring r (TASX_SRV_DIAG=1 in the
 * environment at tasx_server_start), in us: out[0] detection -> frames
 * loaded, out[1] frames loaded -> stores acknowledged, out[2] completion ->
 * next detection, over out[3] batches; out[4] empty polls. */
int tasx_ab_server_diag(int device, unsigned r, double *out);

/* Test hook: restart a context's flush tickets at `start` (nothing pending or
 * in flight, no feeder), so a test can run flushes across the 2^32 wrap. */
int tasx_ab_ctx_set_tickets(unsigned ctx_id, uint32_t start);

#ifdef __cplusplus
}
#endif
#endif
