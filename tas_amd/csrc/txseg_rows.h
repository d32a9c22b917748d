// txseg_rows.h -- the fused TX segment build's kernels (SURVEY.md section 8f
// row 1; flow_tx_read + tcp_checksums of flow_tx_segment,
// /root/reference/tas/fast/fast_flows.c:833-846, :930-936), shared by the
// product launcher (txseg_kernels.hip, which describes them) and the A/B
// build's diagnostics forms (ab/ab_txseg.hip).
#ifndef TASX_TXSEG_ROWS_H_
#define TASX_TXSEG_ROWS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"
#include "xsum_device.h"
#include "txseg_device.h"

namespace {


// row_ror:15 -- lane k of each 16-lane row gets lane (k + 1) % 16's value
__device__ __forceinline__ uint32_t ror15(uint32_t x)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x12f, 0xf, 0xf, false);
}

// bytes [0, k) from a, [k, 16) from b
__device__ __forceinline__ u32x4 merge_at(u32x4 a, u32x4 b, int k)
{
  const u32x4 lo = mask_chunk(a, 0, k), hi = mask_chunk(b, k, 16);
  return u32x4{lo.x | hi.x, lo.y | hi.y, lo.z | hi.z, lo.w | hi.w};
}

__device__ __forceinline__ u32x4 clear_byte(u32x4 v, int b)
{
  const uint32_t m = ~(0xffu << (8 * (b & 3)));
  const int j = b >> 2;
  return u32x4{j == 0 ? v.x & m : v.x, j == 1 ? v.y & m : v.y, j == 2 ? v.z & m : v.z,
               j == 3 ? v.w & m : v.w};
}

// The aligned chunk pair whose funnel gives the 16-byte window starting at
// byte address S, of which bytes [lo, hi) (0 <= lo < hi <= 16) are wanted:
// each chunk holds at least one wanted byte, so neither load can fault.
__device__ __forceinline__ void window_pair(uintptr_t S, int lo, int hi, const u32x4 *&pa, const u32x4 *&pb)
{
  const uintptr_t a = (S + (uintptr_t) lo) & ~(uintptr_t) 15;
  const uintptr_t b1 = (S & ~(uintptr_t) 15) + 16, b2 = (S + (uintptr_t) hi - 1) & ~(uintptr_t) 15;
  pa = (const u32x4 *) a;
  pb = (const u32x4 *) (b1 < b2 ? b1 : b2);
}

// One 16-lane group per segment.  l4-relative coordinates (l4 = frame +
// l4_off): payload D = [dlo, dhi), summed bytes [0, send); chunk c covers
// [16c - head, +16).  The header chunks (the frame's bytes [0, hdrs_len)) are
// read by lane k and written back whole at the end with both checksums
// inserted -- the frame's first cache lines are then written in full, which
// avoids the HBM read-modify-write of a partly written line.  Payload chunks
// [cp0, nend) go to lane (c - cp0) % 16, slot (c - cp0) / 16.  A chunk holding
// both (the first payload chunk) is summed and stored in two parts.  All
// loads of a round are issued before any is consumed, so a segment costs one
// memory latency after its descriptor (plus one per extra 96-chunk round).
// MODE (diagnostics, TASX_TXSEG_DEBUG): bit 0 = no full-chunk payload stores,
// bit 1 = temporal instead of non-temporal stores, bit 3 = no header
// write-back, bit 4 = no partial-chunk stores.
template <int U, int MODE = 0>
__global__ __launch_bounds__(kBlock) void tx_segment_kernel(tasx_txseg_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group leaves together
  // descriptor: two dwordx4 loads, same address on all 16 lanes
  const u32x4 d0 = ld16((const u32x4 *) p.segs, 2 * i), d1 = ld16((const u32x4 *) p.segs, 2 * i + 1);
  const uint64_t frame_off = d0.x | ((uint64_t) d0.y << 32);
  const uint64_t tx_base = d0.z | ((uint64_t) d0.w << 32);
  const uint32_t tx_len = d1.x, pos = d1.y, pay = d1.z & 0xffffu, hl = d1.z >> 16;
  const bool ok = (pay == 0 || pos < tx_len) && pay <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl >= p.l4_off + 20;
  if (!ok) {
    if (gl == 15 && p.out)
      stg(p.out, i, 0u);
    return;
  }
  uint8_t *const f = p.frames + frame_off;
  uint8_t *const ip = f + p.ip_off;
  uint8_t *const l4 = f + p.l4_off;
  const int dlo = (int) (hl - p.l4_off), dhi = dlo + (int) pay;
  const int head = (int) ((uintptr_t) l4 & 15);
  const u32x4 *const c0p = (const u32x4 *) ((uintptr_t) l4 & ~(uintptr_t) 15);
  const uint32_t cp0 = (uint32_t) ((head + dlo) >> 4);                 // first payload chunk
  const uint32_t nend = pay ? (uint32_t) ((head + dhi + 15) >> 4) : cp0; // payload chunks [cp0, nend)
  const int wrap = (int) (tx_len - pos);           // payload index where the buffer wraps
  // Source offsets are 32-bit, relative to shm (shm_len < 4 GiB, checked by
  // the host): payload piece 1 = indices [0, min(wrap, pay)) at s1 + j, piece 2
  // = [wrap, pay) at s2 + j (modular u32 arithmetic; only valid j are used).
  // Chunk c's window starts at payload index j0 = 16c - head - dlo, in the
  // piece of its first payload byte; the lane owning c loads L_c, the aligned
  // chunk holding that window start with j clamped into the piece (so it cannot
  // fault), and takes the window's second chunk from the lane owning c + 1 (DPP
  // row rotate): one source load per chunk.  Exceptions: the chunk ce at the
  // piece switch (the straddle chunk cs, or the last piece-1 chunk when the
  // wrap falls on a chunk boundary) loads its own second chunk (xb1); the
  // straddle chunk's bytes past the wrap come from a piece-2 pair (xa2, xb2).
  const uint8_t *const shm = p.shm;
  const uint32_t s1 = (uint32_t) (tx_base + pos), s2 = s1 - tx_len;
  const bool wraps = wrap < (int) pay;
  const int end1 = min(wrap, (int) pay) - 1; // last piece-1 index
  const int pw = dlo + wrap;
  const uint32_t kw = (uint32_t) ((head + pw) >> 4);
  const bool straddle = wraps && ((head + pw) & 15);
  const uint32_t cs = straddle ? kw : 0xffffffffu;
  const uint32_t ce = wraps ? (straddle ? kw : kw - 1) : 0xffffffffu;
  // chunk c: shm offset of L_c, and the window start's byte position (sh)
  auto window = [&](uint32_t c, int &sh) -> uint32_t {
    const int j0 = 16 * (int) c - head - dlo, blo = max(-j0, 0);
    const bool p2 = wraps && j0 + blo >= wrap;
    const uint32_t sb = p2 ? s2 : s1;
    const int jc = min(max(j0, p2 ? wrap : 0), p2 ? (int) pay - 1 : end1);
    sh = (int) ((sb + (uint32_t) j0) & 15u);
    return (sb + (uint32_t) jc) & ~15u;
  };
  auto shm_chunk = [&](uint32_t off) -> u32x4 { return ld16nt((const u32x4 *) (shm + off), 0); };

  // ---- loads, all unconditional (clamped to valid addresses) so that none is
  // sunk into a branch: header bytes, header chunks, the exception chunks
  const uint32_t tl = (ld8(ip + 2) << 8) | ld8(ip + 3);
  const int wl = min(gl, 9);
  const uint32_t w_ = ld8(ip + 2 * wl) | (ld8(ip + 2 * wl + 1) << 8);
  const uint32_t w = gl < 10 ? w_ : 0u;
  // header chunks: the frame's bytes [0, hl), written back whole at the end
  // with the checksums inserted (the frame's first cache lines are then
  // written in full)
  const int fh = (int) ((uintptr_t) f & 15);
  const u32x4 *const f0p = (const u32x4 *) ((uintptr_t) f & ~(uintptr_t) 15);
  const uint32_t nhc = (uint32_t) ((fh + (int) hl + 15) >> 4);
  u32x4 hv = ld16nt(f0p, min((uint32_t) gl, nhc - 1));
  // lanes map to chunks by ADDRESS (lane = absolute chunk index % 16), so each
  // slot's 16 stores cover whole 256-byte blocks: the frame's payload lines are
  // written whole by one instruction, not merged across instructions in L2
  // (chunk indices below cp0 are idle lanes; signed, as base0 may be < 0)
  const int aoff = (int) (((uintptr_t) c0p >> 4) & 15u);
  const int base0 = (int) cp0 - (((int) cp0 + aoff) & 15);
  auto lane_of = [&](uint32_t c) -> uint32_t { return (uint32_t) ((int) c - base0) & 15u; };
  const bool own_ce = ce != 0xffffffffu && lane_of(ce) == (uint32_t) gl;
  uint32_t o1 = 0, oa = 0, ob = 0; // exception chunks (offset 0 on other lanes)
  {
    const int j0 = 16 * (int) ce - head - dlo;
    o1 = own_ce ? ((s1 + (uint32_t) min(j0 + 16, end1)) & ~15u) : 0u;
    // straddle: piece-2 bytes [wrap - j0, bhi) of the window at s2 + j0,
    // i.e. buffer indices [0, j0 + bhi - wrap): chunks of tx_base and of the
    // window's second slot, clamped to the last wanted byte
    const int bhi = min(dhi - (16 * (int) cs - head), 16);
    const int64_t S = (int64_t) tx_base + (j0 - wrap);
    const int64_t b1 = (S & ~(int64_t) 15) + 16, b2 = ((int64_t) tx_base + (j0 + bhi - wrap) - 1) & ~(int64_t) 15;
    oa = (own_ce && straddle) ? (uint32_t) (tx_base & ~(uint64_t) 15) : 0u;
    ob = (own_ce && straddle) ? (uint32_t) (b1 < b2 ? b1 : b2) : 0u;
  }
  const u32x4 xb1 = shm_chunk(o1), xa2 = shm_chunk(oa), xb2 = shm_chunk(ob);
  const uint32_t len = tl >= 20 ? tl - 20 : 0;
  const int send = min((int) len, dhi);

  // ---- payload chunks: gather, store, sum
  uint64_t acc = 0;
  u32x4 vfirst = u32x4{0, 0, 0, 0}, vlast = vfirst;
  for (int base = base0; base < (int) nend; base += 16 * U) {
    u32x4 a[U];
    int sh;
#pragma unroll
    for (int u = 0; u < U; ++u)
      a[u] = shm_chunk(window((uint32_t) max(base + gl + 16 * u, (int) cp0), sh));
    const u32x4 ext = shm_chunk(window((uint32_t) max(base + 16 * U, (int) cp0), sh)); // lane 15's last neighbour
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ci = base + gl + 16 * u;
      const bool valid = ci >= (int) cp0 && ci < (int) nend;
      const uint32_t c = valid ? (uint32_t) ci : cp0 - 1; // idle lanes: a chunk holding no payload
      const int o = 16 * (int) c - head, j0 = o - dlo;
      const int blo = min(max(-j0, 0), 16), bhi = min(dhi - o, 16);
      // second chunk: a[u] of lane (gl + 1) % 16 (lane 15: slot u + 1 of lane 0)
      const u32x4 nx = (u + 1 < U) ? a[u + 1 < U ? u + 1 : u] : ext;
      const u32x4 t0 = u32x4{ror15(a[u].x), ror15(a[u].y), ror15(a[u].z), ror15(a[u].w)};
      const u32x4 t1 = u32x4{ror15(nx.x), ror15(nx.y), ror15(nx.z), ror15(nx.w)};
      u32x4 bn = gl == 15 ? ((u + 1 < U) ? t1 : ext) : t0;
      if (c == ce)
        bn = xb1;
      window(c, sh);
      u32x4 v = funnel16(a[u], bn, sh);
      if (c == cs) // bytes from the wrap on come from the buffer start
        v = merge_at(v, funnel16(xa2, xb2, (int) ((s2 + (uint32_t) j0) & 15u)), wrap - j0);
      uint8_t *const cp = (uint8_t *) (c0p + c);
      if (valid && blo == 0 && bhi == 16) {
        if (MODE & 2)
          *(__attribute__((address_space(1))) u32x4 *) cp = v;
        else if (!(MODE & 1))
          __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
      }
      // the (at most two) partial payload chunks are stored after the loop
      if (valid && c == cp0)
        vfirst = v;
      if (valid && c == nend - 1)
        vlast = v;
      const int sh = valid ? min(bhi, send - o) : blo; // summed: [blo, sh)
      if (blo > 0 || sh < 16)
        v = mask_chunk(v, blo, max(sh, blo));
      acc += (uint64_t) v.x + v.y + v.z + v.w;
    }
  }
  if (!(MODE & 16) && nend > cp0) {
    // partial first / last payload chunks, on the lanes that own them
    if (lane_of(cp0) == (uint32_t) gl) {
      const int o = 16 * (int) cp0 - head;
      store_range((uint8_t *) (c0p + cp0), vfirst, max(dlo - o, 0), min(dhi - o, 16));
    }
    if (lane_of(nend - 1) == (uint32_t) gl && nend - 1 > cp0) {
      const int o = 16 * (int) (nend - 1) - head;
      store_range((uint8_t *) (c0p + (nend - 1)), vlast, 0, min(dhi - o, 16));
    }
  }
  // ---- header chunks: L4 bytes [0, min(dlo, send)) summed, tcp.chksum as zero
  const int hend = min(dlo, send);
  const int hbase = fh + (int) p.l4_off; // chunk k's byte b is l4 byte 16k + b - hbase
  for (uint32_t k = (uint32_t) gl; k < nhc; k += 16u) {
    u32x4 v = k < 16u ? hv : ld16nt(f0p, k); // > 16 header chunks: rare, loaded here
    const int o = 16 * (int) k - hbase;
    v = mask_chunk(v, min(max(-o, 0), 16), min(max(hend - o, 0), 16));
    if (16 - o >= 0 && 16 - o < 16)
      v = clear_byte(v, 16 - o);
    if (17 - o >= 0 && 17 - o < 16)
      v = clear_byte(v, 17 - o);
    acc += (uint64_t) v.x + v.y + v.z + v.w;
  }
  uint32_t part = fold64_to_18(acc);
  if ((int) len > dhi) { // total_length reaches past the payload: frame bytes
    const Chunks<U> t = chunk_range<U>(l4 + dhi, len - (uint32_t) dhi);
    part += group_lane_sum<U>(t, gl);
  }
  const uint32_t c_ip = (gl < 10 && gl != 5) ? w : 0u;
  const uint32_t c_ph = (gl >= 6 && gl < 10) ? w : (gl == 4 ? (w & 0xff00u) : 0u);
  part = row_sum16(part);
  const uint32_t s_ip = row_sum16(c_ip), s_ph = row_sum16(c_ph);
  // results, valid in lane 15 of the group, then broadcast to the group
  const uint32_t ipc = inv_result(residue(fold32_to_16(s_ip)));
  uint32_t tcpc = 0;
  if (tl >= 20) {
    uint32_t r4 = fold32_to_16(part);
    if (head & 1)
      r4 = bswap16(r4);
    tcpc = inv_result(residue(fold32_to_16(r4 + s_ph + bswap16(len))));
  }
  const uint32_t res = (uint32_t) __shfl((int) (ipc | (tcpc << 16)), (int) ((threadIdx.x & 63u) | 15u), 64);
  if (gl == 15 && p.out)
    stg(p.out, i, res);
  // header write-back: bytes [0, hl) of the frame, checksum fields inserted
  const int fi = (int) p.ip_off + 10 + fh, ft = (int) p.l4_off + 16 + fh; // chunk-grid positions
  for (uint32_t k = (uint32_t) gl; k < nhc; k += 16u) {
    u32x4 v = k < 16u ? hv : ld16nt(f0p, k);
    const int b0 = 16 * (int) k;
    v = put_byte(v, fi - b0, res);
    v = put_byte(v, fi + 1 - b0, res >> 8);
    v = put_byte(v, ft - b0, res >> 16);
    v = put_byte(v, ft + 1 - b0, res >> 24);
    if (!(MODE & 8))
      store_range((uint8_t *) (f0p + k), v, max(fh - b0, 0), min(fh + (int) hl - b0, 16), false);
  }
}

// ---------------------------------------------------------------------------
// tx_segment_u_kernel: the same segment build with ONE UNALIGNED 16-byte load
// per destination chunk (gfx950 global loads take any byte address; measured
// as fast as aligned loads for this copy, tools/copy_unaligned.hip), so there
// is no funnel shift, no neighbour exchange and no exception chunk: the lane
// that owns frame chunk k loads the payload window that lands in it straight
// from the TX buffer, stores it and sums it from the registers.
//   frame chunk k = frame bytes [16k - fh, +16) (fh = frame start mod 16);
//   payload index j at s1 + j before the buffer wraps (j < wrap), s2 + j after;
//   the window of chunk k starts at payload index j0 = 16k - fh - hdrs_len.
// Window loads are clamped to [0, shm_len - 16]; a window that had to be
// clamped (a flow buffer within 16 bytes of the region's ends) is gathered
// byte by byte instead.  The chunk holding the wrap takes its bytes from
// index `wrap` on from a piece-2 window loaded up front.  Header chunks (frame
// bytes [0, hdrs_len), at most 16 of them: the host checks that the checksum
// fields lie in the first 256 bytes) are loaded up front, get their payload
// bytes spliced in, and are written back at the end with both checksums
// inserted; payload chunks are stored as they are built (byte-exact stores at
// the frame's last partial chunk, nothing outside [0, hdrs_len + payload)).
// Lanes own chunks by ADDRESS (lane = absolute chunk index mod 16), so each
// store instruction covers whole 256-byte blocks.  Sums are exact 32-bit word
// sums (v_sad_u16) over frame bytes [l4_off, l4_off + len), tcp.chksum as 0.

template <int U, bool NTS>
__global__ __launch_bounds__(kBlock) void tx_segment_u_kernel(tasx_txseg_params p)
{
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group leaves together
  txseg_row<U, NTS>(p, i, threadIdx.x & 15);
}

// DPP row rotate: lane k of each 16-lane row gets lane (k - N) % 16's value
template <int N>
__device__ __forceinline__ uint32_t row_ror(uint32_t x)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x120 + N, 0xf, 0xf, false);
}

// ---------------------------------------------------------------------------
// tx_segment_tas_kernel: TAS data segments as flow_tx_segment() builds them
// (fast_flows.c:877-955): IPv4 at frame + 14, TCP at + 34 (host-checked for
// the batch), hdrs_len 66 (TCP header + 12-byte timestamp option, :887-888),
// frames 16-byte aligned (the mbuf data room).  The header geometry is then
// fixed and the per-chunk work is the copy itself: frame chunk k >= 5 holds
// payload [16k - 66, 16k - 50), one unaligned window load, one store, four
// v_sad_u16.  Chunks 0..4 (ethernet + IPv4 + TCP + option, and chunk 4's
// first 14 payload bytes) are read from the frame and written back whole at
// the end with both checksums inserted; the IPv4 / pseudo-header channels
// come from chunks 0..2 as in tcp4_tas14_kernel (xsum_kernels.hip).  A
// segment with another hdrs_len or frame alignment, or whose ip.total_length
// is not 52 + payload (:897), is done by the general body (txseg_row), which
// rewrites the same payload bytes and then the checksums.  When the
// descriptor's room (the mbuf data room) covers the frame's last 16-byte
// chunk, that chunk is written whole, its bytes past the frame with their own
// values, instead of by dword and byte stores.
// OPT: how the frame's first block is written, and A/B ablations.
//   kTxHeaderFirst (the product): chunks 0..4 (headers with stale checksum
//     fields, chunk 4's payload) are stored right after the first round's loads
//     are issued, every payload chunk as soon as it lands, and at the end only
//     the two 16-bit checksum fields -- into lines the kernel has just written,
//     merged in L2 (44.9-45.0 against 46.0 us, traffic 1.126 against 1.143 x
//     algorithmic; profiles/r02/r02ar).
//   kTxDppTail (the product, with kTxHeaderFirst): the row total reaches every
//     lane by row rotations and the lane holding chunk 1 finishes and writes
//     both fields, instead of four ds_bpermute round trips to and from lane 15
//     (0.1-0.3 us better in 4 of 4 same-box pairs; profiles/r02/r02ax, r02ay).
//     Occupancy: the kernel holds 105 VGPRs (4 waves per SIMD); 5 waves
//     (WPE 5: 96 VGPRs, a small spill) costs 48 us and residency capped at 3
//     or 2 blocks per CU 46 / 50 us.
//   0: the round-1 form -- the first 256-byte block (headers with both
//     checksums + the payload chunks kept in vfb) written by one instruction
//     at the end; kTxLineKeep: keep only chunk 4's 128-byte line; kTxFieldsOnly:
//     keep nothing, write back chunks 1, 3, 4; kTxSimple: branch-free loop for
//     the common case (profiles/r02/r02v, r02x).
//   Ablations (timing only, results wrong; profiles/r02/r02u): kTxNoScratch,
//     kTxNoWriteBack, kTxNoWindows (chunk-4 / piece-2 window loads),
//     kTxNoFallback (general body not compiled in), kTxNoPayloadStores.
enum : int {
  kTxNoScratch = 1, kTxNoWriteBack = 2, kTxNoWindows = 4, kTxNoFallback = 8, kTxNoPayloadStores = 16,
  kTxLineKeep = 32, kTxFieldsOnly = 64, kTxSimple = 128, kTxHeaderFirst = 256, kTxDppTail = 512,
  kTxNoHeaderStore = 1024, kTxNoFields = 2048, kTxNoSums = 4096 // timing-only ablations (profiles/r02/r02az)
};
template <int U, bool NTS, int WPE = 1, int OPT = kTxHeaderFirst | kTxDppTail>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void tx_segment_tas_kernel(tasx_txseg_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group leaves together
  const u32x4 d0 = ld16((const u32x4 *) p.segs, 2 * i), d1 = ld16((const u32x4 *) p.segs, 2 * i + 1);
  const uint64_t frame_off = d0.x | ((uint64_t) d0.y << 32);
  const uint64_t tx_base = d0.z | ((uint64_t) d0.w << 32);
  const uint32_t tx_len = d1.x, pos = d1.y, pay_ = d1.z & 0xffffu, hl_ = d1.z >> 16;
  const bool ok = (pay_ == 0 || pos < tx_len) && pay_ <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl_ >= p.l4_off + 20;
  uint8_t *const f = p.frames + frame_off;
  bool fast = ok && hl_ == 66u && ((uintptr_t) f & 15u) == 0;
  if (fast) {
    const int pay = (int) pay_, fend = 66 + pay;
    const int K = (fend + 15) >> 4;
    // the descriptor's room covers the last chunk: write it whole, the bytes
    // past the frame with their own values (sub-dword stores cost ~10% here).
    // A scratch room (TASX_TXSEG_SCRATCH) also lets the build write the frame's
    // last 128-byte block whole, with zeros past the frame: no read of the last
    // chunk and no partial-line write for the memory side to merge.
    const uint32_t room = d1.w & ~TASX_TXSEG_SCRATCH;
    const bool scratch = (d1.w & TASX_TXSEG_SCRATCH) != 0u && room >= 16u * (uint32_t) K;
    const bool whole = room >= 16u * (uint32_t) K;
    int kend = K; // chunks [K, kend): scratch zeros up to the block's end
    if (scratch) {
      const uint64_t be = (frame_off + (uint64_t) fend + 127u) & ~127ull;
      kend = max(K, min((int) ((be - frame_off + 15u) >> 4), (int) (room >> 4)));
    }
    const int aoff = (int) (((uintptr_t) f >> 4) & 15u);
    const int kh = (gl - aoff) & 15; // this lane's chunk in the frame's first 256-byte block
    const uint8_t *const shm = p.shm;
    const uint32_t s1 = (uint32_t) (tx_base + pos);
    const int wrap = (int) tx_len - (int) pos;
    const int wrapc = (pay > 0 && wrap < pay) ? wrap : 0x7fffffff; // payload index where piece 2 starts
    const uint32_t smax = (uint32_t) (p.shm_len - 16u);
    auto woff = [&](int j0) -> uint32_t { return s1 + (uint32_t) j0 - (j0 >= wrapc ? tx_len : 0u); };
    const bool straddle = wrapc < pay && ((66 + wrap) & 15);
    const int ks = straddle ? (66 + wrap) >> 4 : -1;
    const uint32_t xoff = straddle ? s1 - tx_len + (uint32_t) (16 * ks - 66) : s1;
    // up front: the header chunk, chunk 4's window (payload [-2, 14)), the piece-2 window
    const u32x4 hv = ld16((const u32x4 *) f, (uint32_t) min(kh, 4));
    const uint32_t o4 = s1 - 2u;
    const u32x4 w4 = (OPT & kTxNoWindows) ? hv : ld16u(shm, min(o4, smax));
    const u32x4 xw = (OPT & kTxNoWindows) ? hv : ld16u(shm, min(xoff, smax));
    u32x4 tv = {0u, 0u, 0u, 0u};
    if (!scratch)
      tv = ld16((const u32x4 *) f, (uint32_t) (K - 1)); // the frame's last chunk as it is

    // whole payload chunks 5..K-1; each store instruction covers whole 256-byte
    // blocks.  The payload chunks of the frame's first block (k < fbe) are kept
    // in vfb and stored at the end together with the header chunks, so the
    // block's lines are written whole by one instruction (a line written in two
    // parts at different times costs an HBM read-modify-write).
    int fbe = aoff <= 10 ? 16 - aoff : 0;
    if (OPT & kTxLineKeep) { // A/B: keep only the payload chunks of chunk 4's 128-byte line
      const int lo8 = aoff & 7;
      fbe = min(fbe, 8 * ((lo8 + 4) / 8 + 1) - lo8);
    }
    if (OPT & (kTxFieldsOnly | kTxHeaderFirst)) // A/B: keep nothing (64: the write-back stores chunks 1, 3, 4 only;
      fbe = 0;          // 256: chunks 0..4 stored early, the two checksum fields at the end)
    // chunks 0..4 (tcp4_tas14_kernel's map for 0..3; chunk 4 = option pad + payload [0, 14))
    auto header_chunk = [&]() -> u32x4 {
      u32x4 h = hv;
      if (kh == 4) {
        u32x4 win = o4 <= smax ? w4 : gather16(shm, o4, p.shm_len);
        if (ks == 4)
          win = splice(win, xoff <= smax ? xw : gather16(shm, xoff, p.shm_len), wrap + 2, 16);
        h = splice(hv, win, 2, fend - 64);
      }
      return h;
    };
    auto store_header = [&](const u32x4 &h) {
      uint8_t *const cp = f + 16 * kh;
      const int hi = fend - 16 * kh;
      if (kh < 5 && hi >= 16)
        *(__attribute__((address_space(1))) u32x4 *) cp = h;
      else if (kh < 5 && whole && kh < K) // h holds the frame's own bytes past its end
        *(__attribute__((address_space(1))) u32x4 *) cp = h;
      else if (kh < 5)
        store_range(cp, h, 0, hi, false);
    };
    u32x4 vfb = hv;
    uint32_t acc = 0;
    const int base0 = 5 - ((5 + aoff) & 15);
    // the common case, wave-wide: every row a fast one with no wrap inside its
    // payload, every window inside the region, one round of chunks.  Its loop
    // has no per-chunk branches but the store's predicate (sums by select)
    const bool simple_row = fast && wrapc == 0x7fffffff && o4 <= smax && base0 + 16 * U >= K &&
                            s1 + (uint32_t) (16 * (K - 1) - 66) <= smax;
    const bool simple = (OPT & kTxSimple) && __builtin_amdgcn_ballot_w64(!simple_row) == 0ull;
    if (simple) {
      u32x4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(max(base0 + gl + 16 * u, 5), K - 1);
        a[u] = ld16u(shm, s1 + (uint32_t) (16 * k - 66));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = base0 + gl + 16 * u, hi = fend - 16 * k;
        const u32x4 v = a[u];
        const bool in = k >= 5 && k < K, full = in && hi >= 16;
        const bool keep = u == 0 && k < fbe;
        if (full && !keep)
          __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
        if (u == 0)
          vfb = full && keep ? v : vfb;
        const uint32_t sv = sad4(v, 0u);
        acc += full ? sv : 0u;
        if (in && hi < 16) { // the frame's last chunk (one lane per row)
          acc += sad_below(v, (uint32_t) hi);
          uint8_t *const cp = f + 16 * k;
          if (whole)
            *(__attribute__((address_space(1))) u32x4 *) cp = splice(tv, v, 0, hi);
          else
            store_range(cp, v, 0, hi, false);
        }
      }
    }
    for (int base = base0; !simple && base < K; base += 16 * U) {
      u32x4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(max(base + gl + 16 * u, 5), K - 1);
        a[u] = ld16u(shm, min(woff(16 * k - 66), smax));
      }
      if ((OPT & kTxHeaderFirst) && !(OPT & kTxNoHeaderStore) && base == base0) // the header chunks (stale checksum fields) go out first
        store_header(header_chunk());
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = base + gl + 16 * u, j0 = 16 * k - 66;
        if (k < 5 || k >= K)
          continue;
        u32x4 v = a[u];
        const uint32_t off = woff(j0);
        if (off > smax) // a window reaching past the region's end: byte by byte
          v = gather16(shm, off, p.shm_len);
        if (k == ks)
          v = splice(v, xoff <= smax ? xw : gather16(shm, xoff, p.shm_len), wrap - j0, 16);
        uint8_t *const cp = f + 16 * k;
        const int hi = fend - 16 * k;
        if (u == 0 && k < fbe && hi >= 16) {
          vfb = v;
          acc = sad4(v, acc);
        } else if (hi >= 16) {
          if (OPT & kTxNoPayloadStores)
            ;
          else if (NTS)
            __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
          else
            *(__attribute__((address_space(1))) u32x4 *) cp = v;
          if (!(OPT & kTxNoSums))
            acc = sad4(v, acc);
        } else {
          acc += sad_below(v, (uint32_t) hi);
          if (whole)
            *(__attribute__((address_space(1))) u32x4 *) cp = splice(tv, v, 0, hi);
          else
            store_range(cp, v, 0, hi, false);
        }
      }
    }

    if (scratch && !(OPT & kTxNoScratch)) { // the scratch chunks past the frame outside its first block
      const int k = K + gl;
      if (k < kend && k >= fbe)
        __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
    }

    u32x4 h = header_chunk();
    const uint32_t m0 = kh == 2 ? 0xffff0000u : (kh == 3 ? 0x0000ffffu : 0xffffffffu);
    uint32_t l4 = sad4(u32x4{h.x & m0, h.y, h.z, h.w}, 0u);
    if (kh == 4 && fend < 80)
      l4 = sad_below(h, (uint32_t) (fend - 64));
    acc += (kh >= 2 && kh <= 4) ? l4 : 0u;
    const uint32_t c0d3 = row_ror<1>(h.w), c2d0 = row_ror<15>(h.x);
    const uint32_t addrs = sadw(h.z & 0xffff0000u, sadw(h.w, sadw(c2d0 & 0xffffu, 0u)));
    const uint32_t ph = sadw(h.y & 0xff000000u, addrs);
    const uint32_t ipsum = sadw(c0d3 & 0xffff0000u, sadw(h.x, sadw(h.y, addrs)));
    const int l1 = (int) ((threadIdx.x & 63u) & ~15u) + ((1 + aoff) & 15); // lane holding chunk 1
    if ((OPT & kTxDppTail) && (OPT & kTxHeaderFirst)) {
      // no LDS round trips: every lane gets the row total by row rotations,
      // and the lane holding chunk 1 (ip.len, the IP header and pseudo-header
      // sums) finishes both checksums and writes both fields itself
      acc += row_ror<8>(acc);
      acc += row_ror<4>(acc);
      acc += row_ror<2>(acc);
      acc += row_ror<1>(acc);
      const bool ok1 = kh == 1 && bswap16(h.x & 0xffffu) == 52u + (uint32_t) pay;
      fast = (__builtin_amdgcn_ballot_w64(ok1) >> l1) & 1ull; // otherwise the general body redoes the segment
      if (ok1) {
        const uint32_t ipc = inv_result(residue(fold32_to_16(ipsum)));
        const uint32_t tcpc = inv_result(
            residue(fold32_to_16(fold32_to_16(acc) + fold32_to_16(ph) + bswap16(32u + (uint32_t) pay))));
        if (p.out)
          stg(p.out, i, ipc | (tcpc << 16));
        if (!(OPT & kTxNoFields)) {
          *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) ipc;
          *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) tcpc;
        }
      }
    } else {
    acc = row_sum16(acc);
    const uint32_t ip1 = (uint32_t) __shfl((int) ipsum, l1, 64), ph1 = (uint32_t) __shfl((int) ph, l1, 64);
    const uint32_t tl = bswap16((uint32_t) __shfl((int) (h.x & 0xffffu), l1, 64));
    fast = tl == 52u + (uint32_t) pay; // otherwise the general body redoes the segment
    const uint32_t ipc = inv_result(residue(fold32_to_16(ip1)));
    const uint32_t len = 32u + (uint32_t) pay;
    const uint32_t tcpc = inv_result(residue(fold32_to_16(fold32_to_16(acc) + fold32_to_16(ph1) + bswap16(len))));
    const uint32_t res = (uint32_t) __shfl((int) (ipc | (tcpc << 16)), (int) ((threadIdx.x & 63u) | 15u), 64);
    if ((OPT & kTxHeaderFirst) && fast) { // only the two fields are left to write
      if (gl == 15 && p.out)
        stg(p.out, i, res);
      if (kh == 1)
        *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) res;
      if (kh == 3)
        *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) (res >> 16);
    } else if (fast && !(OPT & kTxNoWriteBack)) {
      if (gl == 15 && p.out)
        stg(p.out, i, res);
      // the first block: header chunks with the checksums inserted (ip.chksum:
      // chunk 1 bytes 8-9, tcp.chksum: chunk 3 bytes 2-3) and the kept payload chunks
      if (kh == 1)
        h.z = (h.z & 0xffff0000u) | (res & 0xffffu);
      if (kh == 3)
        h.x = (h.x & 0x0000ffffu) | (res & 0xffff0000u);
      uint8_t *const cp = f + 16 * kh;
      const int hi = fend - 16 * kh;
      if ((OPT & kTxFieldsOnly) && (kh == 0 || kh == 2))
        ; // unchanged header chunks
      else if ((kh < 5 || kh < fbe) && hi >= 16)
        *(__attribute__((address_space(1))) u32x4 *) cp = kh < 5 ? h : vfb;
      else if (kh < 5 && whole && kh < K) // h holds the frame's own bytes past its end
        *(__attribute__((address_space(1))) u32x4 *) cp = h;
      else if (kh < 5)
        store_range(cp, h, 0, hi, false);
      else if (!(OPT & kTxNoScratch) && kh >= K && kh < kend && kh < fbe) // scratch chunks inside the first block
        *(__attribute__((address_space(1))) u32x4 *) cp = u32x4{0u, 0u, 0u, 0u};
    }
    }
  }
  if (!(OPT & kTxNoFallback) && !fast) // (3 chunks per lane and round: keeps the fallback's registers below the fast path's)
    txseg_row<3, NTS>(p, i, gl);
}

// ---------------------------------------------------------------------------
// tx_segment_lds_kernel (round 3, the product for TAS's layout): the same
// segment build, one 16-lane row per segment, with the payload read by
// ALIGNED, L2-allocating 16-byte loads and realigned through a per-row LDS
// slice instead of one unaligned non-temporal window load per frame chunk.
//   For the frame's (at most 96) chunks the row loads the aligned source chunks that
//   cover the payload windows: piece A (before the circular buffer
//   wraps) from its 128-byte line on, so that lanes own whole lines, then piece
//   B (after the wrap).  Lane gl, slot u loads virtual chunk gl + 16u (7 slots:
//   112 chunks, enough for 96 frame chunks at any shift) and writes it to slot
//   1 + gl + 16u of the slice.  Each lane then reads its frame chunk's 16-byte
//   window back at its byte offset as five dwords and funnel-shifts them
//   (v_alignbyte_b32); the chunk that straddles the wrap splices a piece-B
//   window in.  Header chunks 0..3 (read from the frame) and chunk 4 (header
//   bytes 64-65 + payload [0, 14)) go out in round 0's store instructions with
//   stale checksum fields, every store non-temporal and covering whole 256-byte
//   blocks (lanes own frame chunks by address); the two 16-bit fields are
//   stored at the end by the lane holding chunk 1, after the row total has
//   reached it by DPP row rotations.
//   Why: an unaligned window shares its first and last 128-byte lines with the
//   neighbouring windows, and with non-temporal loads those lines were fetched
//   again; aligned temporal loads let L2 merge them.  On the bench's pattern
//   (tools/txseg_lds_probe.hip, profiles/r03/r03c-r03d): 43.3 us for the
//   unaligned non-temporal windows, 39.4 us for the same windows temporal,
//   34.2-34.9 us for this scheme.
//   Aligned loads never leave the pages of the bytes they hold, and each load
//   address is clamped to the aligned chunks that touch the shm region, so no
//   load faults; bytes outside what a window needs are masked away.
//   Rows that are not TAS data segments (hdrs_len != 66, a frame off 16-byte
//   alignment, total_length != 52 + payload, a rejected descriptor) go to the
//   general body (txseg_row), as before.
// SLOTS load slots per lane: 6 (96 aligned chunks: piece A from its 16-byte
// chunk on, 25.3 KiB of LDS per block, 6 blocks per CU) or 7 (112: piece A from
// its 128-byte line on, so lanes own whole lines; 29.4 KiB, 5 blocks per CU).
// A window's bytes [o, o + 16) lie in the loaded chunks; its fifth dword, read
// past them, lies in the same aligned chunk as byte o + 15.
constexpr int kLdsLead = 64; // lead bytes: chunk 0's window (payload index -66) stays in the slice
template <int SLOTS>
constexpr int lds_slice() { return kLdsLead + 16 * 16 * SLOTS + 32; } // lead, the slots, tail slack

// 16 bytes at a dword-aligned LDS address shifted by r bytes: five dwords and a funnel shift
__device__ __forceinline__ u32x4 lds_window_at(const uint8_t *wp, uint32_t r)
{
  const uint32_t *w = (const uint32_t *) wp;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
               __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r)};
}

// 16 bytes at LDS byte offset o of the slice: five dwords and a funnel shift
__device__ __forceinline__ u32x4 lds_window(const uint8_t *sl, uint32_t o)
{
  return lds_window_at(sl + (o & ~3u), o & 3u);
}

// OPT (comparison forms of libtasx_ab.so): 1 = no general-body fallback
// compiled in, 2 = wraps ignored (piece A only) -- both timing only, results
// wrong -- 4 = the first block stored non-temporal too (correct), 8 = the
// access pattern alone (timing only: the aligned source chunks stored as
// loaded, no LDS realignment or splice; bench.py's tx_segment pattern_ceiling).
// Round 6 deleted two forms: windows read back by ds_read_b128 at 4-byte
// aligned LDS addresses, and the source chunks landed by LDS-DMA through
// inline asm that moved M0 (profiles/r06/INDEX.md, r06a).
template <bool NTS, int SLOTS = 6, int WPE = 1, int OPT = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void tx_segment_lds_kernel(tasx_txseg_params p)
{
  constexpr int kLdsSlots = SLOTS, kLdsSlice = lds_slice<SLOTS>();
  constexpr uintptr_t kAlignA = SLOTS >= 7 ? 127u : 15u;
  __shared__ __attribute__((aligned(16))) uint8_t lds[(kBlock / 16) * kLdsSlice];
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group leaves together
  uint8_t *const sl = lds + (threadIdx.x / 16) * kLdsSlice;
  const u32x4 d0 = ld16((const u32x4 *) p.segs, 2 * i), d1 = ld16((const u32x4 *) p.segs, 2 * i + 1);
  const uint64_t frame_off = d0.x | ((uint64_t) d0.y << 32);
  const uint64_t tx_base = d0.z | ((uint64_t) d0.w << 32);
  const uint32_t tx_len = d1.x, pos = d1.y, pay_ = d1.z & 0xffffu, hl_ = d1.z >> 16;
  const bool ok = (pay_ == 0 || pos < tx_len) && pay_ <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl_ >= p.l4_off + 20;
  uint8_t *const f = p.frames + frame_off;
  // one round of 96 frame chunks: frames up to 1536 bytes (TAS's data
  // segments are at most 66 + TCP_MSS = 1514, fast_flows.c:37, :887-888);
  // larger ones go to the general body
  bool fast = ok && hl_ == 66u && ((uintptr_t) f & 15u) == 0 && pay_ <= 1536u - 66u;
  if (fast) {
    const int pay = (int) pay_, fend = 66 + pay;
    const int K = (fend + 15) >> 4;
    // the room: the last chunk written whole (its bytes past the frame with
    // their own values), or -- scratch -- the frame's last 128-byte block
    // written whole with zeros past the frame (no read, no partial line; within
    // the round's 96 chunks)
    const uint32_t room = d1.w & ~TASX_TXSEG_SCRATCH;
    const bool scratch = (d1.w & TASX_TXSEG_SCRATCH) != 0u && room >= 16u * (uint32_t) K;
    const bool whole = room >= 16u * (uint32_t) K;
    int kend = K; // chunks [K, kend): scratch zeros up to the block's end
    if (scratch) {
      const uint32_t fo7 = (uint32_t) frame_off & 127u;
      kend = max(K, min(min((int) ((((fo7 + (uint32_t) fend + 127u) & ~127u) - fo7 + 15u) >> 4), (int) (room >> 4)), 96));
    }
    const int aoff = (int) (((uintptr_t) f >> 4) & 15u);
    const int kh = (gl - aoff) & 15; // this lane's chunk in every 16-chunk group of the frame
    // Shm positions as 32-bit offsets from the region's first aligned chunk
    // sbase (an SGPR base; shm_len < 4 GiB, checked by the host), modulo 2^32:
    // loads are clamped to the aligned chunks that touch the region, so an
    // offset that wrapped below the region (payload index -2 of a buffer at its
    // start: chunk 4's don't-care bytes) reads some chunk of the region.
    const uintptr_t sb = (uintptr_t) p.shm;
    const uint8_t *const sbase = (const uint8_t *) (sb & ~(uintptr_t) 15);
    const uint32_t sh0 = (uint32_t) (sb & 15u);
    const uint32_t hi_ok = (uint32_t) ((sb + p.shm_len - 1u) & ~(uintptr_t) 15) - (uint32_t) (sb & ~(uintptr_t) 15);
    const uint32_t t0 = sh0 + (uint32_t) tx_base, s1 = t0 + pos; // ring start, payload index 0
    const int wrap = (int) tx_len - (int) pos;
    const int wrapc = (pay > 0 && wrap < pay && !(OPT & 2)) ? wrap : 0x7fffffff; // payload index where piece B starts
    const u32x4 hv = ld16((const u32x4 *) f, (uint32_t) min(kh, 4)); // header chunks 0..4
    uint32_t acc = 0;
    u32x4 vlast = hv; // the frame's last chunk when it is partial (its lane: kh == (K - 1) & 15)
    const int hlast = fend - 16 * (K - 1); // bytes of the frame in its last chunk, 1..16
    {
      // payload windows of chunks [4, K): payload [jlo, jhi)
      const int jlo = -2, jhi = 16 * K - 66;
      const int aend = min(jhi, wrapc);
      // piece A: payload [jlo, aend) at s1 + j, from its 16-byte chunk (7 slots:
      // its 128-byte line) on
      const uint32_t bA = s1 + (uint32_t) jlo, cA = bA & ~(uint32_t) kAlignA;
      const int nA = aend > jlo ? (int) ((((bA + (uint32_t) (aend - jlo) + 15u) & ~15u) - cA) >> 4) : 0;
      // piece B: payload [max(jlo, wrapc), jhi) at the ring start + j - wrapc
      const int jb = max(jlo, wrapc);
      const uint32_t bB = t0 + (uint32_t) (jb > wrapc ? jb - wrapc : 0), cB = bB & ~15u;
      const int nB = jhi > wrapc ? (int) ((((bB + (uint32_t) (jhi - jb) + 15u) & ~15u) - cB) >> 4) : 0;
      // virtual chunk v is piece A's chunk v, else piece B's chunk v - nA; past
      // the end the last one again (an L2 hit)
      const int nAB = max(nA + nB, 1);
      const uint32_t dB = nB > 0 ? cB - cA - 16u * (uint32_t) nA : 0u;
      u32x4 a[kLdsSlots];
#pragma unroll
      for (int u = 0; u < kLdsSlots; ++u) {
        const int v = min(gl + 16 * u, nAB - 1);
        const uint32_t ro = cA + 16u * (uint32_t) v + (v >= nA ? dB : 0u);
        a[u] = ld16_off(sbase, min(ro, hi_ok));
      }
      if constexpr (!(OPT & 8)) {
#pragma unroll
        for (int u = 0; u < kLdsSlots; ++u)
          *(u32x4 *) (sl + kLdsLead + 16 * (gl + 16 * u)) = a[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      // LDS byte offsets: payload index 0 in piece A, piece B's first byte;
      // window u at o0 + 256u (+ dW for a window in piece B)
      const int oA = kLdsLead + (int) (s1 - cA);
      const int oB = kLdsLead + 16 * nA + (int) (t0 - cB);
      const int o0 = oA + 16 * kh - 66; // >= 0: the lead covers chunk 0's window
      const int dW = wrapc < pay ? oB - oA - wrapc : 0;
      u32x4 w[6]; // the windows of frame chunks 16u + kh
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        const int j0 = 16 * (16 * u + kh) - 66;
        const int o = min(o0 + 256 * u + (j0 >= wrapc ? dW : 0), kLdsSlice - 20);
        w[u] = (OPT & 8) ? a[u] : lds_window(sl, (uint32_t) o);
      }
      // the chunk holding the wrap (a row whose payload wraps off a chunk
      // boundary): its bytes from wrapc - j0 on are piece B's
      const int ks = wrapc < pay ? (66 + wrapc) >> 4 : -1;
      const bool strad = !(OPT & 8) && ks >= 0 && ((66 + wrapc) & 15) != 0 && kh == (ks & 15);
      if (__builtin_amdgcn_ballot_w64(strad) != 0ull) {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int j0 = 16 * (16 * u + kh) - 66;
          if (strad && u == (ks >> 4))
            w[u] = splice(w[u], lds_window(sl, (uint32_t) min(max(oB + j0 - wrapc, 0), kLdsSlice - 20)),
                          wrapc - j0, 16);
        }
      }
      // slot 0: header chunks 0..3 as read, chunk 4 = header bytes 64-65 +
      // payload [0, 14); L4 sums from chunk 2's byte 2 on (TCP starts at 34),
      // chunk 3 without tcp.chksum (bytes 2-3).  Slot 0 (the frame's first two
      // lines, both checksum fields) is stored L2-allocating so that the fields
      // stored at the end merge there; the rest non-temporal.
      if (kh < 4)
        w[0] = hv;
      else if (kh == 4)
        w[0] = splice(hv, w[0], 2, 16);
      const uint32_t mx = kh == 2 ? 0xffff0000u : (kh == 3 ? 0x0000ffffu : kh < 2 ? 0u : 0xffffffffu);
      const uint32_t mr = kh < 2 ? 0u : 0xffffffffu;
      if (__builtin_amdgcn_ballot_w64(K < 81) == 0ull) {
        // every row of the wave holds at least 81 chunks: slots 0..4 are whole
        // frame chunks, only slot 5 holds the frame's end
        acc = sad4(u32x4{w[0].x & mx, w[0].y & mr, w[0].z & mr, w[0].w & mr}, acc);
        if (OPT & 4)
          __builtin_nontemporal_store(w[0], (__attribute__((address_space(1))) u32x4 *) (f + 16 * kh));
        else
          *(__attribute__((address_space(1))) u32x4 *) (f + 16 * kh) = w[0];
#pragma unroll
        for (int u = 1; u < 5; ++u) {
          acc = sad4(w[u], acc);
          __builtin_nontemporal_store(w[u], (__attribute__((address_space(1))) u32x4 *) (f + 16 * (16 * u + kh)));
        }
        const int k = 80 + kh;
        const bool full = k < K - 1 || (k == K - 1 && hlast == 16);
        const uint32_t t = sad4(w[5], acc);
        acc = full ? t : acc;
        vlast = k == K - 1 ? w[5] : vlast;
        if (full || (k >= K && k < kend))
          __builtin_nontemporal_store(k < K ? w[5] : u32x4{0u, 0u, 0u, 0u}, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
      } else {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int k = 16 * u + kh;
          const u32x4 v = w[u];
          // whole chunks here, the partial last one after the loop
          const bool full = k < K - 1 || (k == K - 1 && hlast == 16);
          const uint32_t t = u == 0 ? sad4(u32x4{v.x & mx, v.y & mr, v.z & mr, v.w & mr}, acc) : sad4(v, acc);
          acc = full ? t : acc;
          vlast = k == K - 1 ? v : vlast;
          // whole chunks, and scratch zeros past the frame to its block's end
          if (full || (k >= K && k < kend)) {
            const u32x4 sv = k < K ? v : u32x4{0u, 0u, 0u, 0u};
            if (u == 0 && !(OPT & 4))
              *(__attribute__((address_space(1))) u32x4 *) (f + 16 * k) = sv;
            else
              __builtin_nontemporal_store(sv, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
          }
        }
      }
    }
    if (hlast < 16 && kh == ((K - 1) & 15)) { // the frame's partial last chunk (one lane)
      acc += sad_below(vlast, (uint32_t) hlast);
      uint8_t *const cp = f + 16 * (K - 1);
      if (whole) // its bytes past the frame with their own values (scratch: zeros)
        __builtin_nontemporal_store(splice(scratch ? u32x4{0u, 0u, 0u, 0u} : ld16((const u32x4 *) cp, 0u), vlast, 0, hlast),
                                    (__attribute__((address_space(1))) u32x4 *) cp);
      else
        store_range(cp, vlast, 0, hlast, false);
    }
    // IPv4 and pseudo-header channels from header chunks 0..2 (tcp4_tas14_kernel's map)
    const uint32_t c0d3 = row_ror<1>(hv.w), c2d0 = row_ror<15>(hv.x);
    const uint32_t addrs = sadw(hv.z & 0xffff0000u, sadw(hv.w, sadw(c2d0 & 0xffffu, 0u)));
    const uint32_t ph = sadw(hv.y & 0xff000000u, addrs);
    const uint32_t ipsum = sadw(c0d3 & 0xffff0000u, sadw(hv.x, sadw(hv.y, addrs)));
    const int l1 = (int) ((threadIdx.x & 63u) & ~15u) + ((1 + aoff) & 15); // lane holding chunk 1
    acc += row_ror<8>(acc);
    acc += row_ror<4>(acc);
    acc += row_ror<2>(acc);
    acc += row_ror<1>(acc);
    const bool ok1 = kh == 1 && bswap16(hv.x & 0xffffu) == 52u + (uint32_t) pay;
    fast = (__builtin_amdgcn_ballot_w64(ok1) >> l1) & 1ull; // otherwise the general body redoes the segment
    if (ok1) {
      const uint32_t ipc = inv_result(residue(fold32_to_16(ipsum)));
      const uint32_t tcpc = inv_result(
          residue(fold32_to_16(fold32_to_16(acc) + fold32_to_16(ph) + bswap16(32u + (uint32_t) pay))));
      if (p.out)
        stg(p.out, i, ipc | (tcpc << 16));
      *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) ipc;
      *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) tcpc;
    }
  }
  if (!(OPT & 1) && !fast)
    txseg_row<3, NTS>(p, i, gl);
}

// ---------------------------------------------------------------------------
// tx_segment_wave_kernel: the TAS-layout build with ONE segment per wave.  The
// segment's geometry is wave-uniform, so the descriptor comes in by scalar
// loads and every branch on it is uniform.  The payload is read by ALIGNED
// 16-byte loads: lane L holds the aligned source chunks under frame chunks L
// and L + 64 and gets the next aligned chunk from lane L + 1 by DPP wave_rol:1
// (lane 63: lane 0's second chunk by readlane), then funnel-shifts the pair
// by the segment's source shift (a uniform dword select + v_alignbyte).  The
// bare copy pattern measured 36.6 us this way against 38.6 us for unaligned
// window loads on 16-lane rows (tools/copy_unaligned.hip, profiles/r02/r02bp).
// A segment whose payload wraps in its circular buffer, or whose aligned
// span leaves the shm region, takes unaligned window loads (the row kernel's
// woff / splice / gather scheme) on the same lanes; one that is not TAS's
// data-segment geometry goes to the general row body (txseg_row, lanes 0-15).
// Frame chunk k of lane L, round r: k = L + 64 r.  Chunks 0..3 are headers
// read from the frame, chunk 4 = header bytes 64-65 + payload [0, 14), chunks
// 5.. K-1 payload [16k - 66, +16).  Header-first stores as the row kernel's
// product form: every chunk stored as soon as it is built (stale checksum
// fields), the two 16-bit fields at the end.
__device__ __forceinline__ uint32_t wave_rol1(uint32_t x)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x134, 0xf, 0xf, false); // lane L <- lane L + 1
}
__device__ __forceinline__ u32x4 wave_rol1_4(u32x4 v)
{
  return u32x4{wave_rol1(v.x), wave_rol1(v.y), wave_rol1(v.z), wave_rol1(v.w)};
}
__device__ __forceinline__ u32x4 readlane0_4(u32x4 v)
{
  return u32x4{(uint32_t) __builtin_amdgcn_readlane((int) v.x, 0), (uint32_t) __builtin_amdgcn_readlane((int) v.y, 0),
               (uint32_t) __builtin_amdgcn_readlane((int) v.z, 0), (uint32_t) __builtin_amdgcn_readlane((int) v.w, 0)};
}
// bytes [sh, sh + 16) of a:b, sh wave-uniform
__device__ __forceinline__ u32x4 funnel_uniform(u32x4 a, u32x4 b, uint32_t sh)
{
  const uint32_t r8 = sh & 3u;
  uint32_t w0, w1, w2, w3, w4;
  switch (sh >> 2) {
  case 0: w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; break;
  case 1: w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; break;
  case 2: w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; break;
  default: w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; break;
  }
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, r8), __builtin_amdgcn_alignbyte(w2, w1, r8),
               __builtin_amdgcn_alignbyte(w3, w2, r8), __builtin_amdgcn_alignbyte(w4, w3, r8)};
}
__device__ __forceinline__ uint32_t rl(uint32_t v, int lane)
{
  return (uint32_t) __builtin_amdgcn_readlane((int) v, lane);
}

template <bool NTS>
__global__ __launch_bounds__(kBlock) void tx_segment_wave_kernel(tasx_txseg_params p)
{
  const uint32_t L = threadIdx.x & 63u;
  const uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * (kBlock / 64u) + threadIdx.x / 64u);
  if (i >= p.n)
    return; // the whole wave
  const uint32_t *sd = (const uint32_t *) p.segs + 8u * i; // scalar loads: i is uniform
  const uint64_t frame_off = sd[0] | ((uint64_t) sd[1] << 32);
  const uint64_t tx_base = sd[2] | ((uint64_t) sd[3] << 32);
  const uint32_t tx_len = sd[4], pos = sd[5], pay = sd[6] & 0xffffu, hl = sd[6] >> 16, roomw = sd[7];
  const bool ok = (pay == 0 || pos < tx_len) && pay <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl >= p.l4_off + 20;
  uint8_t *const f = p.frames + frame_off;
  bool fast = ok && hl == 66u && ((uintptr_t) f & 15u) == 0 && p.shm_len >= 16u;
  if (fast) {
    const uint32_t fend = 66u + pay, K = (fend + 15u) >> 4;
    const uint32_t room = roomw & ~TASX_TXSEG_SCRATCH;
    const bool whole = room >= 16u * K, scratch = (roomw & TASX_TXSEG_SCRATCH) != 0u && whole;
    uint32_t kend = K; // scratch zeros in chunks [K, kend): up to the frame's last 128-byte block end
    if (scratch) {
      const uint64_t be = (frame_off + fend + 127u) & ~127ull;
      kend = max(K, min((uint32_t) ((be - frame_off + 15u) >> 4), room >> 4));
    }
    const uint8_t *const shm = p.shm;
    const uint64_t s1 = tx_base + pos;
    const uint32_t wrap = tx_len - pos;                     // payload index where piece 2 starts
    const bool wraps = pay > 0 && wrap < pay;
    // aligned span: frame chunk k >= 4 reads source [s1 - 2 + 16 (k - 4), +16)
    const uint64_t a0 = s1 - 2u, abase = a0 & ~15ull;
    const uint32_t sh = (uint32_t) (a0 & 15u);
    const uint32_t na = K - 3u;                              // aligned chunks abase .. abase + 16 (na - 1)
    const bool aligned = !wraps && s1 >= 2u && abase + 16ull * na <= p.shm_len;
    // the frame's header chunks (lanes 0..4) and, if kept, its last chunk
    const u32x4 hv = ld16((const u32x4 *) f, min(L, 4u));
    const u32x4 tv = (!scratch && whole) ? ld16((const u32x4 *) f, K - 1u) : u32x4{0u, 0u, 0u, 0u};
    // unaligned windows: payload index j at s1 + j before the wrap, at
    // s1 + j - tx_len (= tx_base + j - wrap) from it on; a window outside
    // the region is gathered byte by byte (bytes outside it as 0)
    const int64_t smax = (int64_t) p.shm_len - 16;
    auto load_at = [&](int64_t off) -> u32x4 {
      if (off >= 0 && off <= smax)
        return __builtin_nontemporal_load((gcu4u *) (shm + off));
      return gather16(shm, (uint32_t) off, p.shm_len);
    };
    auto window = [&](uint32_t k) -> u32x4 {
      const int j0 = 16 * (int) k - 66;
      const bool in2 = wraps && j0 >= (int) wrap;
      u32x4 v = load_at((int64_t) s1 + j0 - (in2 ? (int64_t) tx_len : 0));
      if (wraps && j0 < (int) wrap && j0 + 16 > (int) wrap) // the straddle chunk: piece 2 from byte wrap - j0 on
        v = splice(v, load_at((int64_t) s1 + j0 - (int64_t) tx_len), (int) wrap - j0, 16);
      return v;
    };
    auto aload = [&](uint32_t c) -> u32x4 { // aligned source chunk c (clamped to the span)
      return __builtin_nontemporal_load(
          (const __attribute__((address_space(1))) u32x4 *) (shm + abase + 16ull * min(c, na - 1u)));
    };
    // build, store and sum frame chunk k from its payload window v
    uint32_t acc = 0u;
    auto emit = [&](uint32_t k, u32x4 v) {
      if (k >= kend)
        return;
      uint8_t *const cp = f + 16u * k;
      if (k >= K) { // scratch past the frame
        __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, (__attribute__((address_space(1))) u32x4 *) cp);
        return;
      }
      const int hi = (int) fend - 16 * (int) k; // frame bytes in this chunk (>= 1)
      if (k < 4u) {
        // L4 bytes of the header chunks: chunk 2 from byte 34, chunk 3 without tcp.chksum
        const uint32_t m0 = k == 2u ? 0xffff0000u : (k == 3u ? 0x0000ffffu : 0u);
        if (k >= 2u)
          acc = sad4(u32x4{hv.x & m0, hv.y, hv.z, hv.w}, acc);
        *(__attribute__((address_space(1))) u32x4 *) cp = hv;
        return;
      }
      if (k == 4u)
        v = splice(hv, v, 2, hi); // header bytes 64-65, payload [0, 14); past the frame: its own bytes
      if (hi >= 16) {
        acc = sad4(v, acc);
        if (k == 4u || !NTS)
          *(__attribute__((address_space(1))) u32x4 *) cp = v;
        else
          __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
      } else { // the frame's last chunk
        acc += sad_below(v, (uint32_t) hi);
        if (k == 4u && whole)
          *(__attribute__((address_space(1))) u32x4 *) cp = v;
        else if (whole)
          *(__attribute__((address_space(1))) u32x4 *) cp = splice(tv, v, 0, hi);
        else
          store_range(cp, v, 0, hi, false);
      }
    };
    // 128 frame chunks per round: lane L builds chunks base + L and base + 64 + L
    for (uint32_t base = 0; base < kend; base += 128u) {
      const uint32_t k0 = base + L, k1 = base + 64u + L;
      u32x4 w0, w1;
      if (aligned) { // frame chunk k >= 4 = aligned chunks k - 4 and k - 3 funnelled by sh
        const u32x4 v0 = aload(k0 >= 4u ? k0 - 4u : 0u), v1 = aload(k1 - 4u);
        const u32x4 vx = aload(base + 124u); // under chunk base + 128: lane 63's second neighbour
        u32x4 n0 = wave_rol1_4(v0), n1 = wave_rol1_4(v1);
        const u32x4 l0 = readlane0_4(v1);
        if (L == 63u) {
          n0 = l0;
          n1 = vx;
        }
        w0 = funnel_uniform(v0, n0, sh);
        w1 = funnel_uniform(v1, n1, sh);
      } else {
        w0 = window(max(k0, 4u));
        w1 = window(min(k1, K - 1u));
      }
      emit(k0, w0);
      emit(k1, w1);
    }
    // wave totals: 16-lane rows by DPP, the four rows by readlane
    acc += row_ror<8>(acc);
    acc += row_ror<4>(acc);
    acc += row_ror<2>(acc);
    acc += row_ror<1>(acc);
    const uint32_t l4 = rl(acc, 0) + rl(acc, 16) + rl(acc, 32) + rl(acc, 48);
    // the IPv4 header (bytes 14..33, ip.chksum as 0) and pseudo-header from chunks 0..2
    const uint32_t h0w = rl(hv.w, 0), h1x = rl(hv.x, 1), h1y = rl(hv.y, 1), h1z = rl(hv.z, 1), h1w = rl(hv.w, 1),
                   h2x = rl(hv.x, 2);
    const uint32_t addrs = sadw(h1z & 0xffff0000u, sadw(h1w, sadw(h2x & 0xffffu, 0u)));
    const uint32_t ph = sadw(h1y & 0xff000000u, addrs);
    const uint32_t ipsum = sadw(h0w & 0xffff0000u, sadw(h1x, sadw(h1y, addrs)));
    fast = bswap16(h1x & 0xffffu) == 52u + pay; // otherwise the general body redoes the segment
    if (fast && L == 0u) {
      const uint32_t ipc = inv_result(residue(fold32_to_16(ipsum)));
      const uint32_t tcpc = inv_result(residue(fold32_to_16(fold32_to_16(l4) + fold32_to_16(ph) + bswap16(32u + pay))));
      if (p.out)
        stg(p.out, i, ipc | (tcpc << 16));
      *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) ipc;
      *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) tcpc;
    }
  }
  if (!fast && L < 16u)
    txseg_row<3, NTS>(p, i, (int) L);
}

} // namespace
#endif
