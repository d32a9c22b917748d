// xsum_rows.h -- the checksum kernels' device code (SURVEY.md section 8a:
// rte_raw_cksum, rte_ipv4_cksum, rte_ipv4_udptcp_cksum as tcp_checksums()
// calls them, /root/reference/tas/fast/fast_flows.c:1058-1069) and the
// launch helpers, used by the product launchers (xsum_kernels.hip, whose
// header comment gives the layout and arithmetic) and by the comparison
// build's access-pattern kernels (ab/ab_xsum.hip).
#ifndef TASX_XSUM_ROWS_H_
#define TASX_XSUM_ROWS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <errno.h>
#include <string.h>

#include "tasx_kernels.h"

#include "xsum_device.h"

namespace {


// RAW, any layout, word sums by v_sad_u16 into exact 32-bit accumulators
// (variant 6).  Rounds of U chunk loads per lane, clamped to the packet's last
// chunk and issued back to back; chunk-index selects keep the clamped
// re-reads out.  Bytes before the packet in chunk 0 come off on lane 0; bytes
// past it in the last chunk on lane 15, whose last load of the final round is
// always that chunk (its partial may wrap: the group total, < 2^32 for
// TASX_RAW_MAX_LEN, is exact mod 2^32).
// S32: stride mode from a 16-byte aligned base (host-checked): 32-bit byte
// offsets from the block's first packet (a uniform 64-bit base: 16 strides
// from a 16-byte aligned base stay 16-byte aligned), so each load is
// global_load_dwordx4 v, v_off, s[base] (one VGPR per address) at any batch size.
// (32- and 64-lane packet groups measured no faster at config 4's sizes,
// profiles/r04/INDEX.md r04b.)
template <int U, bool S32 = false>
__global__ __launch_bounds__(kBlock) void raw_sad_kernel(tasx_raw_params p)
{
  constexpr int G = 16;
  const int gl = threadIdx.x & (G - 1);
  const uint32_t blk = xcd_run(blockIdx.x, gridDim.x, p.xrun);
  const uint32_t i = blk * (kBlock / G) + threadIdx.x / G;
  if (i >= p.n)
    return;
  const uint32_t len = p.len ? ldg(p.len, i) : p.len0;
  const uint8_t *s = nullptr;
  const uint8_t *const bb = p.base + (uint64_t) (blk * (kBlock / G)) * p.stride;
  uint32_t o0 = 0, head, last;
  if constexpr (S32) {
    const uint32_t so = (threadIdx.x / G) * (uint32_t) p.stride;
    o0 = so & ~15u;
    head = so & 15u;
    last = (head + len - 1u) >> 4; // valid when len > 0
  } else {
    s = p.base + pkt_offset(p.off, p.stride, i);
    head = (uint32_t) ((uintptr_t) s & 15u);
    last = (head + len - 1u) >> 4;
  }
  const u32x4 *c0p = (const u32x4 *) ((uintptr_t) s & ~(uintptr_t) 15);
  uint32_t acc = 0;
  if (len) {
    u32x4 t;
    for (uint32_t cb = 0; cb <= last; cb += (uint32_t) G * U) {
      u32x4 v[U];
      if constexpr (S32) {
        const uint32_t lb = o0 + 16u * (cb + (uint32_t) gl), lastoff = o0 + 16u * last;
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = ld16nt_off(bb, min(lb + 16u * G * u, lastoff));
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = ld16nt(c0p, min(cb + (uint32_t) gl + (uint32_t) G * u, last));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t a = sad4(v[u], acc);
        acc = cb + (uint32_t) gl + (uint32_t) G * u <= last ? a : acc;
      }
      if (cb == 0)
        acc -= gl == 0 ? sad_below(v[0], head) : 0u;
      t = v[U - 1];
    }
    acc -= gl == G - 1 ? sad_from(t, head + len - 16u * last) : 0u;
  }
  acc = group_total<G>(acc);
  if (gl == G - 1) {
    uint32_t f = fold32_to_16(acc);
    if (head & 1)
      f = bswap16(f);
    stg(p.out, i, (uint16_t) f);
  }
}

// RAW with per-packet lengths (variant 7; the automatic choice when lengths
// are given).  The 16-lane-group kernels keep a wave for as many rounds as its
// longest packet needs while the other groups' lanes idle: on the
// {64,576,1500,9000} B mix two waves in three hold a 9000 B packet and keep
// ~30% of their lanes loading.  Here a wave's 4 packets form ONE chunk
// sequence (packet k owns flattened chunks [P_k, P_k+1)) and all 64 lanes load
// consecutive flattened chunks, U per lane per round: ceil(total / 64U) rounds.
// Whole chunks go into cumulative accumulators A_j = sum over the chunks of
// packets >= j, so packet k's sum is A_k - A_{k+1}, exact mod 2^32 (every
// packet sum is < 2^32 for len <= TASX_RAW_MAX_LEN).  The bytes outside
// packet k in its first / last chunk come off on lane k / 4 + k, whose loads
// of those two chunks are issued before round 0 (their addresses come from
// the descriptors: no dependent load phase).
template <int U, bool S32>
__device__ __forceinline__ void wave_chunk_sums(uint64_t lo, const uint64_t (&B)[4], const uint32_t (&P)[4],
                                                uint32_t T, uint32_t lane, uint32_t (&A)[4])
{
  // B[k] = chunk-aligned start of packet k - 16 P_k (mod 2^64): flattened
  // chunk f of packet k is at B[k] + 16 f.  S32: every chunk lies within
  // 4 GiB above lo, so the address is lo + 32-bit offset (one VGPR).
  uint32_t d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    d[k] = (uint32_t) (B[k] - lo);
  const uint8_t *sb = (const uint8_t *) (uintptr_t) lo;
  for (uint32_t f0 = 0; f0 < T; f0 += 64u * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t fc = min(f0 + 64u * u + lane, T - 1u);
      if constexpr (S32) {
        const uint32_t dk = fc >= P[3] ? d[3] : fc >= P[2] ? d[2] : fc >= P[1] ? d[1] : d[0];
        v[u] = ld16nt_off(sb, dk + 16u * fc);
      } else {
        const uint64_t bk = fc >= P[3] ? B[3] : fc >= P[2] ? B[2] : fc >= P[1] ? B[1] : B[0];
        v[u] = __builtin_nontemporal_load((gcu4 *) (uintptr_t) (bk + 16ull * fc));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t f = f0 + 64u * u + lane;
      const uint32_t s = f < T ? sad4(v[u], 0u) : 0u;
      A[0] += s;
      A[1] += f >= P[1] ? s : 0u;
      A[2] += f >= P[2] ? s : 0u;
      A[3] += f >= P[3] ? s : 0u;
    }
  }
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l)
{
  const uint32_t lo = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) x, l);
  const uint32_t hi = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) (x >> 32), l);
  return ((uint64_t) hi << 32) | lo;
}

// The flattened sum of a wave's 4 packets (raw_wave_kernel, tcp4_wave_kernel):
// lanes k and 4 + k hold packet k's start address a and length len (len 0 =
// nothing to sum); returns on lane k < 4 the exact 32-bit sum of packet k's
// little-endian 16-bit words counted in the address frame (from even addresses).
template <int U>
__device__ __forceinline__ uint32_t wave4_sums(uint32_t lane, uint64_t a, uint32_t len)
{
  const uint32_t k = lane & 3u;
  const uint32_t head = (uint32_t) a & 15u;
  const uint32_t nch = len ? (head + len + 15u) >> 4 : 0u;
  const uint64_t c0 = a & ~15ull;
  // packet k's first (lane k) and last (lane 4 + k) chunk, in flight with round 0
  u32x4 bv = {0u, 0u, 0u, 0u};
  if (lane < 8u && nch)
    bv = ld16nt((const u32x4 *) (uintptr_t) c0, lane < 4u ? 0u : nch - 1u);

  uint64_t B[4];
  uint32_t P[4];
  uint32_t T = 0;
  uint64_t lo = ~0ull, hi = 0;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const uint32_t nk = (uint32_t) __builtin_amdgcn_readlane((int) nch, kk);
    const uint64_t ck = readlane64(c0, kk);
    P[kk] = T;
    B[kk] = ck - 16ull * T;
    if (nk) {
      lo = min(lo, ck);
      hi = max(hi, ck + 16ull * nk);
    }
    T += nk;
  }
  uint32_t A[4] = {0u, 0u, 0u, 0u};
  if (T) {
    if (hi - lo <= 0xffffffffull)
      wave_chunk_sums<U, true>(lo, B, P, T, lane, A);
    else
      wave_chunk_sums<U, false>(lo, B, P, T, lane, A);
  }
  // boundary bytes of packet k off A_0..A_k (packet k's sum is A_k - A_{k+1})
  uint32_t corr = 0;
  if (lane < 8u && nch)
    corr = lane < 4u ? sad_below(bv, head) : sad_from(bv, head + len - 16u * (nch - 1u));
  A[0] -= corr;
  A[1] -= k >= 1u ? corr : 0u;
  A[2] -= k >= 2u ? corr : 0u;
  A[3] -= k == 3u ? corr : 0u;
  uint32_t t[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    t[j] = (uint32_t) __builtin_amdgcn_readlane((int) group_total<64>(A[j]), 63);
  return k == 0u ? t[0] - t[1] : k == 1u ? t[1] - t[2] : k == 2u ? t[2] - t[3] : t[3];
}

template <int U>
__global__ __launch_bounds__(kBlock) void raw_wave_kernel(tasx_raw_params p)
{
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t i0 = xcd_run(blockIdx.x, gridDim.x, p.xrun) * (kBlock / 16) + (threadIdx.x >> 6) * 4u;
  if (i0 >= p.n) // wave-uniform
    return;
  const uint32_t i = i0 + (lane & 3u);
  // lanes k and 4 + k hold packet k's descriptor
  uint64_t a = 0;
  uint32_t len = 0;
  if (lane < 8u && i < p.n) {
    a = (uint64_t) (uintptr_t) p.base + pkt_offset(p.off, p.stride, i);
    len = p.len ? ldg(p.len, i) : p.len0;
  }
  const uint32_t s = wave4_sums<U>(lane, a, len);
  if (lane < 4u && i < p.n) {
    uint32_t f = fold32_to_16(s);
    if (a & 1u)
      f = bswap16(f);
    stg(p.out, i, (uint16_t) f);
  }
}

// The bytes a frame owns from its start: the batch's room, else its stride
// slot (stride mode); ~0 when nothing bounds it.
__device__ __forceinline__ uint32_t slot_bound(const tasx_tcp4_params &p)
{
  if (p.room)
    return p.room;
  if (!p.off && p.stride)
    return p.stride < 0xffffffffull ? (uint32_t) p.stride : 0xffffffffu;
  return 0xffffffffu;
}

// Receive-side read bound of a frame, in bytes from its start: the received
// frame length (the hint: the mbuf data_len) capped at the frame's room or
// stride slot (a hint beyond them is not trusted for reads), else the room /
// slot; ~0 when nothing bounds it (offsets without hints or room: the buffer
// must then hold ip_off + total_length bytes, as DPDK assumes).
__device__ __forceinline__ uint32_t rx_bound(const tasx_tcp4_params &p, uint32_t hint)
{
  const uint32_t b = slot_bound(p);
  return hint ? min(hint, b) : b;
}

// TCP4, any frame layout: header words and the checksum-field bytes by byte
// loads, then the segment chunks.  With a frame-length hint (the mbuf
// data_len tx_send() sets before tx_flush) the chunk loads are issued together
// with the header loads; the hint drives only the prefetch: results always
// follow ip.total_length (chunks past it are dropped, chunks the hint missed
// are loaded after the header arrives).
//
// VERIFY = true is the receive-side check (TAS itself
// never verifies, fast_flows.c:242-251): the checksum fields are summed as they
// are, and out[i] gets a flag byte: bit 0 = the header folds to 0xffff, bit 1
// = rte_ipv4_udptcp_cksum_verify passes (DPDK >= 21.11: fold1(raw(L4) +
// phdr) == 0xffff; total_length < 20 fails), bit 2 = IHL != 5 (TAS drops
// such frames, fast_flows.c:247; bits 0/1 then describe a 20-byte header).
// Received frames are untrusted: reads stay below the frame's rx_bound() (the
// received length, else the room, else the stride slot), and a datagram whose
// total_length reaches past it fails the L4 check (bit 1 clear) without being
// read; the 20-byte IPv4 header is always read.
// One frame (i) per 16-lane DPP row, lane gl (the body of tcp4_frame_kernel).
template <int U, bool VERIFY = false>
__device__ __forceinline__ void tcp4_frame_row(const tasx_tcp4_params &p, uint32_t i, int gl)
{
  uint8_t *f = p.base + pkt_offset(p.off, p.stride, i);
  uint8_t *ip = f + p.ip_off;
  uint8_t *l4 = f + p.l4_off;
  const uint32_t hint = p.flen ? ldg(p.flen, i) : p.flen0;
  // speculative chunk loads first, then the header bytes
  const uint32_t slen = hint > p.l4_off ? min(hint - p.l4_off, 65535u) : 0u;
  const Chunks<U> sr = chunk_range<U>(l4, slen);
  u32x4 v[U];
  if (sr.nch) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt(sr.c0p, min((uint32_t) gl + 16u * u, sr.nch - 1));
  }
  const uint32_t tl = (ld8(ip + 2) << 8) | ld8(ip + 3);
  uint32_t w = 0;
  if (gl < 10)
    w = ld8(ip + 2 * gl) | (ld8(ip + 2 * gl + 1) << 8);
  const uint32_t len = tl >= 20 ? tl - 20 : 0;
  bool trunc = false; // RX: the datagram reaches past the frame's bound
  uint32_t rlen = len;
  if constexpr (VERIFY) {
    const uint32_t b = rx_bound(p, hint);
    const uint32_t have = b > p.l4_off ? b - p.l4_off : 0u;
    trunc = len > have;
    rlen = trunc ? have : len;
  }
  const Chunks<U> r = chunk_range<U>(l4, rlen);
  // first 16*U chunks: reuse the speculative loads when they cover them
  uint64_t acc = 0;
  if (r.nch) {
    const uint32_t need = min(r.nch, 16u * U);
    if (sr.nch < need) { // hint too short (or absent): load now
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = ld16nt(r.c0p, min((uint32_t) gl + 16u * u, r.nch - 1));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool keep = (uint32_t) gl + 16u * u < r.nch;
      acc += keep ? (uint64_t) v[u].x + v[u].y + v[u].z + v[u].w : 0ull;
    }
    if (gl == 0 && r.head)
      acc -= chunk_prefix_sum(v[0], r.head);
    const uint32_t last = r.nch - 1;
    if (last < 16u * U && (last & 15u) == (uint32_t) gl && r.tail < 16) {
      const uint32_t ut = last >> 4;
      u32x4 t = v[0];
#pragma unroll
      for (int u = 1; u < U; ++u)
        if (ut == (uint32_t) u)
          t = v[u];
      acc -= (uint64_t) t.x + t.y + t.z + t.w - chunk_prefix_sum(t, r.tail);
    }
  }
  if (!VERIFY && len > 16) {
    // tcp.chksum (segment bytes 16, 17) is taken as zero: subtract its bytes
    // exactly on the lane that holds their chunk (chunk index <= 2, so u = 0)
    const int p16 = r.head + 16, p17 = p16 + 1;
    if (gl == (p16 >> 4))
      acc -= (uint64_t) chunk_byte(v[0], p16 & 15) << (8 * (p16 & 3));
    if (len > 17 && gl == (p17 >> 4))
      acc -= (uint64_t) chunk_byte(v[0], p17 & 15) << (8 * (p17 & 3));
  }
  uint32_t part = fold64_to_18(acc);
  if (r.nch > 16u * U) { // long segments: the rest in the plain loop
    Chunks<U> rest = r;
    rest.c0p = r.c0p + 16u * U;
    rest.nch = r.nch - 16u * U;
    rest.head = 0;
    part += group_lane_sum<U>(rest, gl);
  }
  uint32_t c_ip = (gl < 10 && (VERIFY || gl != 5)) ? w : 0u;
  uint32_t c_ph = (gl >= 6 && gl < 10) ? w : (gl == 4 ? (w & 0xff00u) : 0u);
  const uint32_t w0 = (uint32_t) __shfl((int) w, (threadIdx.x & 63) & ~15, 64); // version/IHL byte
  part = row_sum16(part);
  c_ip = row_sum16(c_ip);
  c_ph = row_sum16(c_ph);
  if (VERIFY && gl == 15) {
    // exact rte_raw_cksum values: every sum above is exact and non-negative
    const uint32_t ri = fold32_to_16(c_ip);
    uint32_t flags = (ri == 0xffffu) ? 1u : 0u;
    if (tl >= 20 && !trunc) {
      uint32_t r4 = fold32_to_16(part);
      if (r.head & 1)
        r4 = bswap16(r4);
      const uint32_t ph = fold32_to_16(c_ph + bswap16(len)); // rte_ipv4_phdr_cksum
      uint32_t c = r4 + ph;
      c = (c >> 16) + (c & 0xffffu);
      flags |= (c == 0xffffu) ? 2u : 0u;
    }
    if ((w0 & 0x0fu) != 5u)
      flags |= 4u;
    stg((uint8_t *) p.out, i, (uint8_t) flags);
  }
  if (!VERIFY && gl == 15) {
    const uint32_t ipc = inv_result(residue(fold32_to_16(c_ip)));
    uint32_t tcpc = 0;
    if (tl >= 20) {
      uint32_t r4 = fold32_to_16(part);
      if (r.head & 1)
        r4 = bswap16(r4);
      tcpc = inv_result(residue(fold32_to_16(r4 + c_ph + bswap16(len))));
    }
    if (p.out)
      stg((uint32_t *) p.out, i, ipc | (tcpc << 16));
    if (p.flags & TASX_F_INPLACE) {
      st8(ip + 10, ipc);
      st8(ip + 11, ipc >> 8);
      st8(l4 + 16, tcpc);
      st8(l4 + 17, tcpc >> 8);
    }
  }
}

template <int U, bool VERIFY = false>
__global__ __launch_bounds__(kBlock) void tcp4_frame_kernel(tasx_tcp4_params p)
{
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group (one DPP row) leaves together
  tcp4_frame_row<U, VERIFY>(p, i, threadIdx.x & 15);
}


// mask of the bytes of a dword (first byte at ip-relative offset `base`) that
// fall in [lo, hi)
__device__ __forceinline__ uint32_t in_range(int base, int lo, int hi)
{
  const int bl = min(max(lo - base, 0), 4);
  const int bh = min(max(hi - base, 0), 4);
  if (bh <= bl)
    return 0u;
  return (uint32_t) (((1ull << (8 * bh)) - 1ull) & ~((1ull << (8 * bl)) - 1ull));
}

// TCP4, TAS frame layout (tcp = ip + 20), stride mode: one chunk range
// [ip, ip + 20 + L4 length) carries the IPv4 header, the pseudo-header fields
// and the segment, so no byte loads are issued at all.  The (up to 4) lanes
// holding chunks with header bytes split them into three channels:
//   IP = header bytes [0,10) + [12,20)            (ip.chksum taken as 0)
//   PH = proto (offset 9) + src/dst [12,20)       (pseudo-header fields)
//   L4 = [20, 20+len) minus the tcp.chksum bytes [36,38)
// with byte masks from three 64-bit constants (bit x+16 = ip-relative byte x
// is in the channel) expanded by one multiply.  total_length comes from the
// chunk holding offsets 2..3 by a lane shuffle.  32-bit byte offsets from the
// 16-byte aligned batch base make every load global_load_dwordx4 v, v_off,
// s[base] (one VGPR per address).  With a frame-length hint all chunk loads
// are issued at once; without one, after total_length is known.
constexpr uint64_t kPatIP = (((1ull << 10) - 1) << 16) | (((1ull << 8) - 1) << 28);  // [0,10)+[12,20)
constexpr uint64_t kPatPH = (1ull << 25) | (((1ull << 8) - 1) << 28);                // {9}+[12,20)
constexpr uint64_t kPatNL4 = ((1ull << 36) - 1) | (3ull << 52);                     // [-16,20)+{36,37}
// receive-side check: the checksum fields are summed as received
constexpr uint64_t kPatIPV = ((1ull << 20) - 1) << 16;                               // [0,20)
constexpr uint64_t kPatNL4V = (1ull << 36) - 1;                                      // [-16,20)

__device__ __forceinline__ uint32_t expand4(uint32_t bits)
{
  return ((bits * 0x204081u) & 0x01010101u) * 0xffu; // 4 bits -> 4 byte masks
}

__device__ __forceinline__ uint32_t pat_bits(uint64_t pat, int s)
{
  return s < 64 ? (uint32_t) (pat >> s) & 0xfu : 0u;
}


// one frame (i) per 16-lane group (a DPP row); lane gl, the row's first lane
// gbase in the wave.  VERIFY: the receive-side flags of tcp4_frame_kernel<U,
// true> instead.
template <int U, bool VERIFY = false>
__device__ __forceinline__ void tcp4_tas_frame(tasx_tcp4_params p, uint32_t i, int gl, int gbase)
{
  constexpr int G = 16;
  constexpr uint64_t pat_ip = VERIFY ? kPatIPV : kPatIP, pat_nl4 = VERIFY ? kPatNL4V : kPatNL4;
  const uint8_t *base = p.base; // 16-byte aligned, batch span < 4 GiB (host-checked)
  const uint32_t fo = (uint32_t) pkt_offset(p.off, p.stride, i);
  const uint32_t ipo = fo + p.ip_off;
  const uint32_t a0 = ipo & ~15u;
  const int hb = (int) (ipo & 15u);
  const uint32_t hint = p.flen ? ldg(p.flen, i) : p.flen0;
  const uint32_t hend = hint > p.ip_off + 20u ? min(hint - p.ip_off, 65535u) : 20u;
  const uint32_t nld = (uint32_t) (hb + hend + 15) >> 4;
  // round 1: U loads back to back, no branches (lanes past the hinted range
  // re-read its last chunk: same line, no extra HBM traffic)
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = ld16nt_off(base, a0 + 16u * min((uint32_t) gl + (uint32_t) G * u, nld - 1));
  const int ca = (hb + 2) >> 4, cb = (hb + 3) >> 4;
  const uint32_t ba = (uint32_t) __shfl((int) chunk_byte(v[0], (hb + 2) & 15), gbase + ca, 64);
  const uint32_t bb = (uint32_t) __shfl((int) chunk_byte(v[0], (hb + 3) & 15), gbase + cb, 64);
  const uint32_t tl = (ba << 8) | bb;
  const uint32_t len = tl >= 20 ? tl - 20 : 0;
  int E = 20 + (int) len;
  bool trunc = false; // RX: the datagram reaches past the frame's bound (rx_bound)
  if constexpr (VERIFY) {
    const uint32_t b = rx_bound(p, hint);
    const uint32_t have = b > p.ip_off + 20u ? min(b - p.ip_off, 65535u) : 20u;
    trunc = (uint32_t) E > have;
    E = trunc ? (int) have : E;
  }
  const uint32_t nch = (uint32_t) (hb + E + 15) >> 4;
  const uint32_t need = min(nch, (uint32_t) G * U);
  if (__builtin_amdgcn_ballot_w64(nld < need) != 0ull) {
    const uint32_t top = max(need, nld);
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt_off(base, a0 + 16u * min((uint32_t) gl + (uint32_t) G * u, top - 1));
  }
  const uint32_t last = nch - 1;
  const int tail = (int) ((ipo + (uint32_t) E) - ((ipo + (uint32_t) E - 1) & ~15u));
  uint64_t acc = 0, acc_ip = 0, acc_ph = 0;
  if (gl < 4) {
    const uint32_t w[4] = {v[0].x, v[0].y, v[0].z, v[0].w};
    const bool l4ok = (uint32_t) gl <= last;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sft = 16 * gl + 4 * j - hb + 16;
      acc_ip += w[j] & expand4(pat_bits(pat_ip, sft));
      acc_ph += w[j] & expand4(pat_bits(kPatPH, sft));
      uint32_t ml4 = ~expand4(pat_bits(pat_nl4, sft));
      if ((uint32_t) gl == last) // a short segment ends in this chunk: bytes < tail only
        ml4 &= in_range(4 * j, 0, tail);
      acc += l4ok ? (w[j] & ml4) : 0u;
    }
  } else if ((uint32_t) gl < nch) {
    acc += (uint64_t) v[0].x + v[0].y + v[0].z + v[0].w;
  }
#pragma unroll
  for (int u = 1; u < U; ++u) {
    const uint32_t c = (uint32_t) gl + (uint32_t) G * u;
    acc += c < nch ? (uint64_t) v[u].x + v[u].y + v[u].z + v[u].w : 0ull;
  }
  if (last >= 4u && last < (uint32_t) G * U && (last % G) == (uint32_t) gl && tail < 16) {
    const uint32_t ut = last / G;
    u32x4 t = v[0];
#pragma unroll
    for (int u = 1; u < U; ++u)
      if (ut == (uint32_t) u)
        t = v[u];
    acc -= (uint64_t) t.x + t.y + t.z + t.w - chunk_prefix_sum(t, tail);
  }
  uint32_t part = fold64_to_18(acc);
  if (nch > (uint32_t) G * U) {
    Chunks<U> rest;
    rest.c0p = (const u32x4 *) (base + a0) + (uint32_t) G * U;
    rest.nch = nch - (uint32_t) G * U;
    rest.head = 0;
    rest.tail = tail;
    part += group_lane_sum<U, G>(rest, gl);
  }
  uint32_t c_ip = fold64_to_18(acc_ip);
  uint32_t c_ph = fold64_to_18(acc_ph);
  part = group_total<G>(part);
  c_ip = group_total<G>(c_ip);
  c_ph = group_total<G>(c_ph);
  if constexpr (VERIFY) {
    const uint32_t vihl = (uint32_t) __shfl((int) chunk_byte(v[0], hb & 15), gbase + (hb >> 4), 64);
    if (gl == G - 1) {
      // every sum above is exact, so the folds are rte_raw_cksum's values
      uint32_t ri = fold32_to_16(c_ip);
      if (hb & 1)
        ri = bswap16(ri);
      uint32_t flags = ri == 0xffffu ? TASX_RX_IP_OK : 0u;
      if (tl >= 20 && !trunc) {
        uint32_t r4 = fold32_to_16(part), rp = fold32_to_16(c_ph);
        if (hb & 1) {
          r4 = bswap16(r4);
          rp = bswap16(rp);
        }
        uint32_t c = r4 + fold32_to_16(rp + bswap16(len)); // + rte_ipv4_phdr_cksum
        c = (c >> 16) + (c & 0xffffu);
        flags |= c == 0xffffu ? TASX_RX_L4_OK : 0u;
      }
      flags |= (vihl & 0xfu) != 5u ? TASX_RX_IHL_NOT5 : 0u;
      stg((uint8_t *) p.out, i, (uint8_t) flags);
    }
  } else if (gl == G - 1) {
    uint32_t ri = fold32_to_16(c_ip), rp = fold32_to_16(c_ph), r4 = fold32_to_16(part);
    if (hb & 1) {
      ri = bswap16(ri);
      rp = bswap16(rp);
      r4 = bswap16(r4);
    }
    const uint32_t ipc = inv_result(residue(ri));
    uint32_t tcpc = 0;
    if (tl >= 20)
      tcpc = inv_result(residue(fold32_to_16(r4 + rp + bswap16(len))));
    if (p.out)
      stg((uint32_t *) p.out, i, ipc | (tcpc << 16));
    if (p.flags & TASX_F_INPLACE) {
      uint8_t *ip = p.base + ipo;
      st8(ip + 10, ipc);
      st8(ip + 11, ipc >> 8);
      st8(ip + 36, tcpc);
      st8(ip + 37, tcpc >> 8);
    }
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void tcp4_tas_kernel(tasx_tcp4_params p)
{
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return;
  tcp4_tas_frame<U>(p, i, threadIdx.x & 15, (threadIdx.x & 63) & ~15);
}

// TCP4 headline kernel: TAS frames in 16-byte aligned mbuf rooms (IPv4 header
// at 14 mod 16, TCP at +20), one frame per 16-lane DPP row, U = 6 chunks per
// lane (96 chunks: datagrams up to 1522 B in one round).  The per-lane work is
// the fold itself: one v_sad_u16 per dword (both LE 16-bit words of the dword
// added into a 32-bit accumulator: the address-aligned word sum, exact), U
// loads, U selects, and a fixed header split.  Chunk map (chunk c = frame
// bytes [16c, 16c+16), dN = its dword N):
//   chunk 0 = eth[0,14) + ip[0,2)   IP: d3.hi
//   chunk 1 = ip[2,18)              IP: d0, d1, d2.hi, d3 (ip.chksum = d2.lo left out)
//                                   PH: d1 byte 3 (proto), d2.hi, d3 (src, dst)
//   chunk 2 = ip[18,20) + tcp[0,14) IP, PH: d0.lo;  L4: d0.hi, d1..d3
//   chunk 3 = tcp[14,30)            L4: d0.lo, d1..d3 (tcp.chksum = d0.hi left out)
//   chunks 4.. = the segment        L4 (bytes past ip + total_length subtracted
//                                   on the lane holding the last chunk)
// Lane 1 (chunk 1) forms IP and PH with chunk 0's d3 and chunk 2's d0 moved in
// by DPP.  How a row learns its datagram's extent (MODE):
//   kHint    one uniform frame-length hint (flen0, the mbuf data_len of a
//            uniform-MTU batch) fixes the geometry for every row; a row whose
//            ip.total_length differs is redone by the general body.  One
//            dependent memory latency per frame.
//   kTlFirst the row reads chunk 1 (ip.total_length; all 16 lanes, one line)
//            first, then exactly its datagram: two dependent latencies, no
//            byte read past ip.total_length (DPDK's own trust in the header).
//   kHintArr per-frame hints (the mbuf data_len of each frame): the row's own
//            hint fixes its geometry and lane 15 checks it against
//            ip.total_length after the loads (a mismatch, or a hint outside
//            [ip_off + 38, ip_off + 1522] or beyond the room, is redone by
//            the general body).  One dependent latency after the hint load,
//            which 4 rows share a line of.
//   kRoom    all 96 chunks of the frame's room at once, masked per row by its
//            total_length after the loads: one latency for every frame, at the
//            price of reading whole rooms.  Needs a room of 1536 B.
// Rows with total_length outside [38, 1522], or beyond the RX
// read bound, take the general body (tcp4_tas_frame; tcp4_frame_row with OFFS).
// OFFS (not kHint): frames at base + off[i] instead of i * stride; a row whose
// frame start (base + off[i] + (ip_off & ~15)) is not 16-byte aligned loads
// only the aligned chunk holding the IPv4 header start and is redone by the
// general row body.
// (Round 6: the head-5 mode, tcp4_mix_kernel's, the per-frame-hint rows that
// leave lanes past the last chunk idle and the sorted-rows form -- all measured
// slower, profiles/r02 -- are gone from the source.)
enum Tas14Mode : int { kHint = 0, kTlFirst = 1, kRoom = 3, kHintArr = 5 /* per-frame hints as the geometry */ };

// The row body after the loads: v[] holds the row's chunks (lane gl: chunks
// gl + 16u), hend the datagram extent it assumed; sums, results, stores, and
// the general body for a row the fast path cannot take.
template <int U, int MODE, bool VERIFY, bool OFFS>
__device__ __forceinline__ void tas14_finish(const tasx_tcp4_params &p, uint32_t i, int gl, const uint8_t *fb,
                                             uint32_t a0, uint32_t hend, bool in_range, const u32x4 (&v)[U])
{
  const uint32_t last = (14u + hend - 1u) >> 4;
  const uint32_t tail = 14u + hend - 16u * last; // bytes of the last chunk inside, 1..16

  // chunks 0..3: the L4 part of chunk gl (none for 0, 1), whole chunks elsewhere
  const u32x4 h = v[0];
  const uint32_t m0 = gl == 2 ? 0xffff0000u : (gl == 3 && !VERIFY ? 0x0000ffffu : 0xffffffffu);
  uint32_t acc = sad4(u32x4{h.x & m0, h.y, h.z, h.w}, 0u);
  acc = (gl < 2 || (uint32_t) gl > last) ? 0u : acc;
  // IP and PH channels on lane 1
  const uint32_t c0d3 = row_shr<1>(h.w), c2d0 = row_shl<1>(h.x);
  const uint32_t addrs = sadw(h.z & 0xffff0000u, sadw(h.w, sadw(c2d0 & 0xffffu, 0u))); // src, dst
  const uint32_t ph = sadw(h.y & 0xff000000u, addrs);
  uint32_t ipsum = sadw(c0d3 & 0xffff0000u, sadw(h.x, sadw(h.y, addrs)));
  if constexpr (VERIFY) // the received ip.chksum is part of the check
    ipsum = sadw(h.z & 0xffffu, ipsum);
  const uint32_t tlw = h.x & 0xffffu; // ip[2,4): total_length, network order
#pragma unroll
  for (int u = 1; u < U; ++u) {
    const uint32_t s = sad4(v[u], acc);
    acc = ((uint32_t) gl + 16u * u <= last) ? s : acc;
  }
  // bytes [tail, 16) of the last chunk lie past the datagram: the lane holding
  // that chunk takes them off (its own partial may wrap; the group total is
  // exact mod 2^32).  Clamped loads leave it in lane 15's last slot; kRoom
  // picks slot last / 16 on lane last % 16.
  {
    uint32_t gm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = tail > 4u * j ? min(tail - 4u * j, 4u) : 0u;
      gm[j] = (uint32_t) (~0ull << (8u * k));
    }
    u32x4 t = v[U - 1];
    uint32_t tlane = 15u;
    if constexpr (MODE == kRoom) {
      const uint32_t ut = last >> 4;
      t = v[0];
#pragma unroll
      for (int u = 1; u < U; ++u)
        t = ut == (uint32_t) u ? v[u] : t;
      tlane = last & 15u;
    }
    const uint32_t g = sad4(u32x4{t.x & gm[0], t.y & gm[1], t.z & gm[2], t.w & gm[3]}, 0u);
    acc -= (uint32_t) gl == tlane ? g : 0u;
  }
  acc = row_sum16(acc);
  const uint32_t ip15 = row_shr<14>(ipsum), ph15 = row_shr<14>(ph), tl15 = bswap16(row_shr<14>(tlw));
  constexpr bool kArr = MODE == kHintArr;
  const bool bad = MODE == kHint ? tl15 != hend : kArr ? (tl15 != hend || !in_range) : !in_range; // kHint*: meaningful on lane 15
  if constexpr (VERIFY) {
    const uint32_t vihl = row_shr<14>(c0d3 >> 16); // ip[0]: version / IHL
    if (gl == 15 && !bad) {
      // exact rte_raw_cksum values (every sum above is exact)
      uint32_t flags = fold32_to_16(ip15) == 0xffffu ? TASX_RX_IP_OK : 0u;
      uint32_t c = fold32_to_16(acc) + fold32_to_16(ph15 + bswap16(hend - 20u)); // + rte_ipv4_phdr_cksum
      c = (c >> 16) + (c & 0xffffu);
      flags |= c == 0xffffu ? TASX_RX_L4_OK : 0u;
      flags |= (vihl & 0xfu) != 5u ? TASX_RX_IHL_NOT5 : 0u;
      stg((uint8_t *) p.out, i, (uint8_t) flags);
    }
  } else if (gl == 15 && !bad) {
    const uint32_t ipc = inv_result(residue(fold32_to_16(ip15)));
    const uint32_t r = fold32_to_16(acc) + fold32_to_16(ph15) + bswap16(hend - 20u);
    const uint32_t tcpc = inv_result(residue(fold32_to_16(r)));
    if (p.out)
      stg((uint32_t *) p.out, i, ipc | (tcpc << 16));
    if (p.flags & TASX_F_INPLACE) {
      uint8_t *ip = (uint8_t *) fb + a0 + 14u;
      st8(ip + 10, ipc);
      st8(ip + 11, ipc >> 8);
      st8(ip + 36, tcpc);
      st8(ip + 37, tcpc >> 8);
    }
  }
  if (__builtin_amdgcn_ballot_w64(gl == 15 && bad) != 0ull) {
    const int gbase = (threadIdx.x & 63) & ~15;
    const bool rbad = (MODE == kHint || kArr) ? (bool) __shfl((int) bad, gbase + 15, 64) : bad;
    if (rbad) {
      if constexpr (OFFS)
        tcp4_frame_row<3, VERIFY>(p, i, gl);
      else
        tcp4_tas_frame<U, VERIFY>(p, i, gl, gbase);
    }
  }
}

// FLOW (RX, with VERIFY): the frames' flow lookup (fast_flows_packet_fss,
// tas/fast/fast_flows.c:1084-1163) in the same launch.
//  kFlowSplitX (round 3, the product for the row forms; kFlowSplitX2 for a
//   uniform received length): the split grid with the lookup blocks first, one
//   frame per lane, each lookup block taking the frames of the 16 verify blocks
//   that land on its own XCD (blocks are placed round-robin over the 8 XCDs
//   by blockIdx; the lookup block count is a multiple of 8, so verify block vb
//   keeps vb % 8).  The lookup's dependent chain (key -> bucket -> flow key)
//   is the long one, so its blocks start first and overlap the verify rows
//   instead of forming the grid's tail; its plain key load leaves the frame's
//   first line in that XCD's L2, where the verify row's chunk-0 load then
//   finds it.  kFlowSplitX2: the same with two frames per lookup lane (32
//   verify blocks per lookup block).
//  Measured and not taken (profiles/r02-r04; gone from the source in round 6):
//   the lookup inside the verify rows, lookup blocks over consecutive frames
//   (the round-2 product) or interleaved with the verify blocks, hint
//   prefetch, line-paired generations, issue priority, streamed flow-state keys.
enum { kFlowNone = 0, kFlowSplitX = 5, kFlowSplitX2 = 6 };
// lookup blocks of a kFlowSplitX* grid over nv verify blocks (16 F of them per lookup block)
template <uint32_t F>
__host__ __device__ constexpr uint32_t splitx_lookup_blocks(uint32_t nv) { return ((nv + 16u * F - 1u) / (16u * F) + 7u) & ~7u; }
template <int U, int MODE, bool VERIFY = false, int WPE = 1, bool OFFS = false, int FLOW = kFlowNone>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void tcp4_tas14_kernel(tasx_tcp4_params p)
{
  constexpr int BS = kBlock;
  static_assert(U == 6, "one round of 96 chunks covers the 1522-byte datagram bound");
  static_assert(!(OFFS && MODE == kHint), "uniform hints are a stride-mode form");
  static_assert(FLOW == kFlowNone || VERIFY, "the fused flow lookup is an RX form");
  const int gl = threadIdx.x & 15;
  // this block's verify block (split grids: below); large batches XCD-ordered
  uint32_t vb = FLOW == kFlowNone ? xcd_run(blockIdx.x, gridDim.x, p.xrun) : blockIdx.x;
  if constexpr (FLOW == kFlowSplitX || FLOW == kFlowSplitX2) {
    static_assert(BS == 256, "16 verify rows per block, one lookup lane per row of 16 blocks");
    constexpr uint32_t kF = FLOW == kFlowSplitX2 ? 2u : 1u;
    const uint32_t nl = splitx_lookup_blocks<kF>((uint32_t) (((uint64_t) p.n + BS / 16 - 1u) / (BS / 16)));
    if (blockIdx.x < nl) {
      // lane t, frame f: row t % 16 of verify block 8 (16 F (b / 8) + 16 f + t / 16) + b % 8 (past the batch: no store)
      const uint32_t b = blockIdx.x;
      uint32_t i0[kF];
#pragma unroll
      for (uint32_t f = 0; f < kF; ++f) {
        const uint32_t vbk = 8u * (16u * kF * (b / 8u) + 16u * f + threadIdx.x / 16u) + (b & 7u);
        i0[f] = vbk * (BS / 16) + (threadIdx.x & 15u);
      }
      flow_lookup_lanes_at<kF, BS>(p, i0);
      return;
    }
    vb = blockIdx.x - nl;
  }
  const uint32_t i = vb * (BS / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return;
  const uint8_t *fb = p.base; // loads at fb + 32-bit offsets
  uint32_t a0;
  bool row_ok = true;
  if constexpr (OFFS) {
    const uint64_t fo = (uint64_t) (uintptr_t) p.base + ldg(p.off, i) + (p.ip_off & ~15u);
    row_ok = (fo & 15u) == 0u;
    fb = (const uint8_t *) (uintptr_t) (row_ok ? fo : ((fo + 14u) & ~15ull)); // else: the chunk holding ip[0]
    a0 = 0;
  } else {
    a0 = i * (uint32_t) p.stride + (p.ip_off & ~15u);
  }
  // RX: datagram bytes this row may read (rx_bound); TX trusts total_length
  uint32_t have = 65535u;
  if constexpr (VERIFY && MODE != kHint) {
    const uint32_t b = rx_bound(p, p.flen ? ldg(p.flen, i) : p.flen0);
    have = b > p.ip_off + 20u ? min(b - p.ip_off, 65535u) : 20u;
  }
  // the datagram [ip, ip + hend): uniform from the hint, or per row from the
  // frame's own total_length; loads clamped to its last chunk (kRoom: to the room)
  const uint32_t lo = a0 + 16u * (uint32_t) gl;
  uint32_t hend;
  bool in_range = true;
  u32x4 v[U];
  if constexpr (MODE == kHint) {
    hend = p.flen0 - p.ip_off;
    const uint32_t lastoff = a0 + 16u * ((14u + hend - 1u) >> 4);
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt_off(fb, min(lo + 256u * u, lastoff));
  } else if constexpr (MODE == kTlFirst) {
    const uint32_t tl0 = bswap16(ld16nt_off(fb, a0 + (row_ok ? 16u : 0u)).x & 0xffffu);
    // from 38 (tcp.chksum inside the datagram, so the last chunk's bytes past
    // the end never include the masked field; pure ACKs, ip.len 52, qualify)
    // to 1522 (96 chunks)
    in_range = row_ok && tl0 >= 38u && tl0 <= 1522u && tl0 <= have;
    // out of range: the header only, then the general body (a misaligned row: chunk 0 only)
    hend = in_range ? tl0 : (row_ok ? 20u : 1u);
    const uint32_t lastoff = a0 + 16u * ((14u + hend - 1u) >> 4);
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt_off(fb, min(lo + 256u * u, lastoff));
  } else if constexpr (MODE == kHintArr) {
    // the row's own hint (mbuf data_len) fixes its geometry; lane 15 checks
    // it against total_length afterwards, as kHint does for a uniform hint
    const uint32_t h = ldg(p.flen, i);
    const uint32_t hl = h > p.ip_off ? h - p.ip_off : 0u;
    in_range = row_ok && hl >= 38u && hl <= 1522u && h <= slot_bound(p); // reads stay inside the room / slot
    hend = in_range ? hl : (row_ok ? 20u : 1u);
    const uint32_t last = (14u + hend - 1u) >> 4, lastoff = a0 + 16u * last;
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt_off(fb, min(lo + 256u * u, lastoff));
  } else { // kRoom
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt_off(fb, row_ok ? lo + 256u * u : a0);
    const uint32_t tl0 = bswap16(row_newbcast<1>(v[0].x) & 0xffffu);
    in_range = row_ok && tl0 >= 38u && tl0 <= 1522u && tl0 <= have;
    hend = in_range ? tl0 : (row_ok ? 20u : 1u);
  }
  tas14_finish<U, MODE, VERIFY, OFFS>(p, i, gl, fb, a0, hend, in_range, v);
}

// Dynamic LDS reserved (never used) by the v_sad_u16 kernels to cap residency
// at 5 blocks = 20 waves per CU: with ~100 VALU per wave they would otherwise
// run 8 waves per SIMD, and the extra bytes in flight only lengthen the queue
// (interleaved sweeps: 64K TAS frames -0.4%, 64K x 1500 B RAW -1%, 8M x 1500 B
// RAW -1.5%; profiles/r01_sweeps_s2.jsonl).
constexpr uint32_t kOccLds = 30u * 1024u;

// raw_wave_kernel: chunks per lane per round and the LDS reservation
#ifndef TASX_WAVE_U
#define TASX_WAVE_U 6
#endif
#ifndef TASX_WAVE_LDS
#define TASX_WAVE_LDS kOccLds
#endif


// XCD-ordered grids (xcd_run, round 5): from 16,384 blocks (a batch of 256K
// frames or packets and up) each XCD works through runs of 256 consecutive
// blocks (6 MB of 1500-byte packets), the 8 runs of a window adjacent.  In grid
// order the 8 XCDs spread their L2 misses over every DRAM page in flight; in
// runs each XCD's misses stay on few pages: 8M x 1500 B RAW 1.74-1.77 ms
// against 1.87-2.00, the L2's DRAM credit stalls 0.25M against 1.48M and tag
// stalls 0.29M against 1.52M per launch, translation misses about the same
// (28K against 32K; profiles/r05/INDEX.md r05a-r05c, r05z).  64K-frame batches
// (the headline) are neutral to slower in any XCD order and stay in grid order.
constexpr uint32_t kXrunMinBlocks = 16384u;
constexpr uint32_t kXrun = 9u; // runs of 2^(9 - 1) = 256 blocks


static uint32_t xrun_for(uint64_t blocks)
{
  return blocks >= kXrunMinBlocks ? kXrun : 0u;
}

template <typename K, typename Prm>
int launch_groups(const char *name, K kern, const Prm &p, hipStream_t s, uint32_t lds = 0)
{
  // one 16-lane group per packet, kBlock / 16 groups per block: the grid
  // covers the batch once (measured faster than persistent grids at these
  // batch sizes: no uneven drain, the dispatcher refills CUs within ~0.5 us)
  constexpr int BS = kBlock;
  constexpr uint64_t fpb = BS / 16;
  const uint64_t blocks = ((uint64_t) p.n + fpb - 1) / fpb;
  if (blocks == 0)
    return 0;
  if (blocks > 0x7fffffffull)
    return -2;
  Prm q = p;
  q.xrun = xrun_for(blocks);
  tasx_note_kernel(name);
  hipLaunchKernelGGL(kern, dim3((uint32_t) blocks), dim3(BS), lds, s, q);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}


} // namespace

// tcp4_tas_kernel preconditions: TAS layout, 16-byte aligned base, stride mode,
// every frame within 4 GiB of the base (32-bit offsets)
static bool tas_kernel_ok(const tasx_tcp4_params &p)
{
  return p.l4_off == p.ip_off + 20 && ((uintptr_t) p.base & 15u) == 0 && p.off == nullptr &&
         (uint64_t) p.n * p.stride + 65536u + p.ip_off < (1ull << 32);
}

// tcp4_tas14_kernel in stride mode: in addition the IPv4 header at 14 mod 16
// in every frame (a 16-byte multiple stride)
static bool tas14_stride_ok(const tasx_tcp4_params &p)
{
  return tas_kernel_ok(p) && (p.ip_off & 15u) == 14u && (p.stride & 15u) == 0;
}

// ... with one uniform hint whose datagram spans 5..96 chunks and covers tcp.chksum
static bool tas14_ok(const tasx_tcp4_params &p)
{
  if (!tas14_stride_ok(p) || p.flen || !p.flen0)
    return false;
  if (p.flen0 < p.ip_off + 64u || p.flen0 - p.ip_off > 65535u)
    return false;
  return ((14u + (p.flen0 - p.ip_off) + 15u) >> 4) <= 16u * 6u;
}

// ... without a uniform hint (per-frame hints only steer reads: a row's
// results follow its own total_length), stride mode or frames by an offsets array (IPv4 at 14
// mod 16 from the frame start; frames not 16-byte aligned are checked per row)
static bool tas14_nohint_ok(const tasx_tcp4_params &p)
{
  return tas14_stride_ok(p) && !p.flen0;
}
static bool tas14_offs_ok(const tasx_tcp4_params &p)
{
  return p.off != nullptr && p.l4_off == p.ip_off + 20 && (p.ip_off & 15u) == 14u && !p.flen0;
}

// Row mode without a uniform hint.  A room covering a full-MTU frame lets rows
// of a batch that carries no per-frame lengths load the whole MTU at once
// (bulk TX batches: 64K MTU frames 15.9 us against 16.9 us total_length
// first).  Batches with per-frame hints are data/ACK mixes, where whole-room
// reads cost every ACK row 1.5 KB (16.0 us at any ACK share) and total_length
// first wins (25 / 50 / 75 % ACKs: 13.6 / 10.6 / 8.5 us); the head-5 mode
// (an ACK's 80 bytes with the total_length) lost to it everywhere but all-ACK
// batches (6.3 against 6.8 us).  With per-frame
// hints each row takes its own hint as its geometry (kHintArr: no dependent
// total_length read; 0 / 25 / 50 / 75 % ACKs 16.5 / 13.2 / 10.4-10.5 / 8.3 us
// against 17.0 / 13.6-13.7 / 10.6-10.8 / 8.6 us, all-ACK 7.2 against 6.9).
// tools/ackmix_probe.py, profiles/r02/r02d_ackmix_modes.jsonl, r02o.
static int tas14_mode(const tasx_tcp4_params &p)
{
  const uint32_t from_a0 = p.room > (p.ip_off & ~15u) ? p.room - (p.ip_off & ~15u) : 0u;
  if (p.flen)
    return kHintArr;
  return from_a0 >= 1536u ? kRoom : kTlFirst;
}

template <bool OFFS>
static int launch_tas14_verify(const tasx_tcp4_params &p, int mode, hipStream_t s)
{
  const uint32_t lds = 0u;
  switch (mode) {
  case kHintArr:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<hints,verify,offs>" : "tcp4_tas14_kernel<hints,verify>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, OFFS>, p, s, lds);
  default:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<tl_first,verify,offs>" : "tcp4_tas14_kernel<tl_first,verify>",
                         tcp4_tas14_kernel<6, kTlFirst, true, 8, OFFS>, p, s, lds);
  }
}

// the grid of tcp4_tas14_kernel<..., kFlowSplitX*>: the XCD-matched lookup blocks, then the verify blocks
template <uint32_t F = 1, typename K>
static int launch_splitx(const char *name, K kern, const tasx_tcp4_params &p, hipStream_t s, uint32_t lds)
{
  const uint64_t nv = ((uint64_t) p.n + kBlock / 16 - 1) / (kBlock / 16);
  if (nv == 0)
    return 0;
  const uint64_t blocks = nv + splitx_lookup_blocks<F>((uint32_t) nv);
  if (blocks > 0x7fffffffull)
    return -2;
  tasx_note_kernel(name);
  hipLaunchKernelGGL(kern, dim3((uint32_t) blocks), dim3(kBlock), lds, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the RX pass's row forms (no uniform received length): one lookup lane per
// frame (kFlowSplitX)
template <bool OFFS, int MODE>
static int launch_rx_rows(const tasx_tcp4_params &p, hipStream_t s)
{
  static const char *const names[2][2] = {
      {"tcp4_tas14_kernel<tl_first,verify,flow>", "tcp4_tas14_kernel<tl_first,verify,offs,flow>"},
      {"tcp4_tas14_kernel<hints,verify,flow>", "tcp4_tas14_kernel<hints,verify,offs,flow>"}};
  return launch_splitx<1u>(names[MODE == kHintArr][OFFS], tcp4_tas14_kernel<6, MODE, true, 8, OFFS, kFlowSplitX>, p,
                           s, 0u);
}

// tcp4_tas14_kernel without a uniform hint, in the mode the room allows.  Built for 8 waves per SIMD (64 VGPRs; the
// spills are confined to the general-body fallback after the fast path's
// stores): data/ACK mixes are latency-bound and gain from the residency (64K
// frames at 50 / 75 / 100 % ACKs: 11.2 / 9.3-9.9 / 7.38 -> 10.8 / 8.6 / 6.97
// us; uniform MTU 17.05 -> 17.0; profiles/r01_ackmix_wpe_ab.txt).
template <bool OFFS>
static int launch_tas14_rows(const tasx_tcp4_params &p, int mode, hipStream_t s)
{
  const uint32_t lds = 0u;
  switch (mode) {
  case kHintArr:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<hints,offs>" : "tcp4_tas14_kernel<hints>",
                         tcp4_tas14_kernel<6, kHintArr, false, 8, OFFS>, p, s, lds);
  case kRoom:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<room,offs>" : "tcp4_tas14_kernel<room>",
                         tcp4_tas14_kernel<6, kRoom, false, 8, OFFS>, p, s, lds);
  default:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<tl_first,offs>" : "tcp4_tas14_kernel<tl_first>",
                         tcp4_tas14_kernel<6, kTlFirst, false, 8, OFFS>, p, s, lds);
  }
}

#endif
