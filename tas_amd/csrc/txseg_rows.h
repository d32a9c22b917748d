// txseg_rows.h -- the fused TX segment build's kernels (SURVEY.md section 8f
// row 1; flow_tx_read + tcp_checksums of flow_tx_segment,
// /root/reference/tas/fast/fast_flows.c:833-846, :930-936), launched by
// txseg_kernels.hip (which describes them): tx_segment_lds_kernel (TAS's
// layout), tx_segment_u_kernel (any layout with both checksum fields in the
// frame's first 256 bytes) and tx_segment_kernel (any other layout); the
// general row body is txseg_device.h's.
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
template <int U>
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
      if (valid && blo == 0 && bhi == 16)
        __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
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
  if (nend > cp0) {
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
// 6 load slots per lane: 96 aligned chunks, piece A from its 16-byte chunk on;
// 25.3 KiB of LDS per block, 6 blocks per CU.  A window's bytes [o, o + 16) lie in the loaded chunks; its fifth dword, read
// past them, lies in the same aligned chunk as byte o + 15.
constexpr int kLdsLead = 64; // lead bytes: chunk 0's window (payload index -66) stays in the slice
constexpr int kLdsSlots = 6;
template <int SLOTS = kLdsSlots>
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

// (The comparison build keeps this kernel's round-3 options, among them the
// access pattern alone that bench.py prices it against: ab/ab_txseg_rows.h.)
template <bool NTS>
__global__ __launch_bounds__(kBlock) void tx_segment_lds_kernel(tasx_txseg_params p)
{
  constexpr int kLdsSlice = lds_slice();
  constexpr uintptr_t kAlignA = 15u;
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
    const int wrapc = (pay > 0 && wrap < pay) ? wrap : 0x7fffffff; // payload index where piece B starts
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
#pragma unroll
      for (int u = 0; u < kLdsSlots; ++u)
        *(u32x4 *) (sl + kLdsLead + 16 * (gl + 16 * u)) = a[u];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
        w[u] = lds_window(sl, (uint32_t) o);
      }
      // the chunk holding the wrap (a row whose payload wraps off a chunk
      // boundary): its bytes from wrapc - j0 on are piece B's
      const int ks = wrapc < pay ? (66 + wrapc) >> 4 : -1;
      const bool strad = ks >= 0 && ((66 + wrapc) & 15) != 0 && kh == (ks & 15);
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
            if (u == 0)
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
  if (!fast)
    txseg_row<3, NTS>(p, i, gl);
}

} // namespace
#endif
