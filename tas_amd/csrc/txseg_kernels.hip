// txseg_kernels.hip -- fused TX segment build for gfx950 (SURVEY.md section 8f
// row 1): the payload copy of flow_tx_segment() (flow_tx_read() from the
// flow's circular TX buffer, /root/reference/tas/fast/fast_flows.c:833-846 and
// :930-933, dma_read tas/fast/dma.h:39-53) fused with the tcp_checksums() that
// follows it (:936 -> :1058-1069).  TAS reads the payload twice (rte_memcpy,
// then the checksum loop); here each payload byte is read once from the TX
// buffer, written once into the frame, and summed from registers.
//
// Layout: one 16-lane group (a DPP row) per segment, as in the checksum
// kernels.  The group walks the frame's address-aligned 16-byte chunks
// covering [l4_off, hdrs_len + payload).  For a chunk that holds payload bytes
// the lane loads the two aligned source chunks spanning the payload bytes'
// window in the TX buffer (clamped so both hold valid bytes: they cannot
// fault), funnel-shifts them into frame alignment (v_alignbyte_b32), writes
// them (one dwordx4 store, byte stores at the two partial ends) and sums the
// chunk value the frame will hold.  Header chunks (before hdrs_len) are read
// from the frame.  A chunk whose payload window straddles the end of the
// circular buffer (at most one per segment) is gathered byte by byte.  Bytes
// the IPv4 total_length covers beyond hdrs_len + payload (never produced by
// flow_tx_segment, :897) are summed from the frame in a second pass.  The
// arithmetic (exact 64-bit dword sums, end-around folds, residues) is the
// checksum kernels' (xsum_kernels.hip header comment).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"
#include "xsum_device.h"

namespace {


// 16 bytes starting at byte s (0..15) of the 32-byte pair (a, b)
__device__ __forceinline__ u32x4 funnel16(u32x4 a, u32x4 b, int s)
{
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const int q = s >> 2;
  const uint32_t r = (uint32_t) (s & 3);
  uint32_t o[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const uint32_t w0 = w[t], w1 = w[t + 1], w2 = w[t + 2];
    const uint32_t w3 = (t + 3 < 8) ? w[t + 3] : 0u;
    o[t] = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
  }
  return u32x4{__builtin_amdgcn_alignbyte(o[1], o[0], r), __builtin_amdgcn_alignbyte(o[2], o[1], r),
               __builtin_amdgcn_alignbyte(o[3], o[2], r), __builtin_amdgcn_alignbyte(o[4], o[3], r)};
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

// byte b of v set to x (no-op unless 0 <= b < 16)
__device__ __forceinline__ u32x4 put_byte(u32x4 v, int b, uint32_t x)
{
  const uint32_t sh = 8u * (uint32_t) (b & 3), m = ~(0xffu << sh), y = (x & 0xffu) << sh;
  const int j = b >> 2;
  return u32x4{j == 0 ? (v.x & m) | y : v.x, j == 1 ? (v.y & m) | y : v.y, j == 2 ? (v.z & m) | y : v.z,
               j == 3 ? (v.w & m) | y : v.w};
}

// store bytes [lo, hi) of v into the 16-byte aligned chunk at cp: whole
// dwords as dword stores, the rest as byte stores (constant offsets from one
// address)
__device__ __forceinline__ void store_range(uint8_t *cp, u32x4 v, int lo, int hi, bool nt = true)
{
  if (lo >= hi)
    return;
  if (lo == 0 && hi == 16) {
    if (nt)
      __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
    else
      *(__attribute__((address_space(1))) u32x4 *) cp = v;
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (lo <= 4 * j && 4 * j + 4 <= hi) {
      stg((uint32_t *) cp, (uint32_t) j, w[j]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * j + q >= lo && 4 * j + q < hi)
          st8(cp + 4 * j + q, w[j] >> (8 * q));
    }
  }
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
// bit 1 = temporal instead of non-temporal stores.
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
  const uintptr_t s1 = (uintptr_t) p.shm + tx_base + pos; // payload byte j at s1 + j (j < wrap)
  const uintptr_t s2 = s1 - tx_len;                       // ... or at s2 + j (j >= wrap)
  // the chunk holding payload bytes from both sides of the wrap, if any
  const int pw = dlo + wrap;
  const uint32_t cs = (wrap < (int) pay && ((head + pw) & 15)) ? (uint32_t) ((head + pw) >> 4) : 0xffffffffu;

  // ---- loads, all unconditional (clamped to valid addresses) so that none is
  // sunk into a branch: header bytes, header chunks, the straddle chunk's
  // second piece
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
  const bool own_cs = cs != 0xffffffffu && ((cs - cp0) & 15u) == (uint32_t) gl;
  const u32x4 *xpa = f0p, *xpb = f0p;
  {
    const int o = 16 * (int) cs - head, j0 = o - dlo;
    const u32x4 *pa, *pb;
    window_pair(s2 + (intptr_t) j0, wrap - j0, min(dhi - o, 16), pa, pb);
    xpa = own_cs ? pa : xpa;
    xpb = own_cs ? pb : xpb;
  }
  const u32x4 xa = ld16nt(xpa, 0), xb = ld16nt(xpb, 0);
  const uint32_t len = tl >= 20 ? tl - 20 : 0;
  const int send = min((int) len, dhi);

  // ---- payload chunks: gather, store, sum
  uint64_t acc = 0;
  u32x4 vfirst = u32x4{0, 0, 0, 0}, vlast = vfirst;
  for (uint32_t base = cp0; base < nend; base += 16u * U) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { // clamped: lanes past the end re-read the last chunk
      const uint32_t cc = min(base + (uint32_t) gl + 16u * u, nend - 1);
      const int o = 16 * (int) cc - head, j0 = o - dlo;
      const int blo = max(-j0, 0), bhi = min(dhi - o, 16);
      const bool p2 = j0 + blo >= wrap;
      const int hi = p2 ? bhi : min(bhi, wrap - j0); // wanted bytes in this piece
      const u32x4 *pa, *pb;
      window_pair((p2 ? s2 : s1) + (intptr_t) j0, blo, hi, pa, pb);
      a[u] = ld16nt(pa, 0);
      b[u] = ld16nt(pb, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = base + (uint32_t) gl + 16u * u;
      const bool valid = c < nend;
      const uint32_t cc = valid ? c : nend - 1;
      const int o = 16 * (int) cc - head, j0 = o - dlo;
      const int blo = max(-j0, 0), bhi = min(dhi - o, 16);
      const bool p2 = j0 + blo >= wrap;
      u32x4 v = funnel16(a[u], b[u], (int) (((p2 ? s2 : s1) + (intptr_t) j0) & 15));
      if (cc == cs) // bytes from the wrap on come from the buffer start
        v = merge_at(v, funnel16(xa, xb, (int) ((s2 + (intptr_t) j0) & 15)), wrap - j0);
      uint8_t *const cp = (uint8_t *) (c0p + cc);
      if (valid && blo == 0 && bhi == 16) {
        if (MODE & 2)
          *(__attribute__((address_space(1))) u32x4 *) cp = v;
        else if (!(MODE & 1))
          __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
      }
      // the (at most two) partial payload chunks are stored after the loop
      if (valid && cc == cp0)
        vfirst = v;
      if (valid && cc == nend - 1)
        vlast = v;
      const int sh = valid ? min(bhi, send - o) : blo; // summed: [blo, sh)
      if (blo > 0 || sh < 16)
        v = mask_chunk(v, blo, max(sh, blo));
      acc += (uint64_t) v.x + v.y + v.z + v.w;
    }
  }
  if (nend > cp0) {
    // partial first / last payload chunks (lanes 0 and (nend - 1 - cp0) % 16)
    if (gl == 0) {
      const int o = 16 * (int) cp0 - head;
      store_range((uint8_t *) (c0p + cp0), vfirst, max(dlo - o, 0), min(dhi - o, 16));
    }
    if (((nend - 1 - cp0) & 15u) == (uint32_t) gl && nend - 1 > cp0) {
      const int o = 16 * (int) (nend - 1) - head;
      if (MODE & 4) { // diagnostic: pad the frame's last cache line (needs room)
        uint8_t *e = (uint8_t *) (c0p + (nend - 1));
        store_range(e, vlast, 0, 16);
        for (e += 16; ((uintptr_t) e & 127) != 0; e += 16)
          store_range(e, u32x4{0, 0, 0, 0}, 0, 16);
      } else {
        store_range((uint8_t *) (c0p + (nend - 1)), vlast, 0, min(dhi - o, 16));
      }
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

} // namespace

extern "C" int tasx_launch_txseg(const tasx_txseg_params *p, void *stream)
{
  constexpr uint64_t spb = kBlock / 16;
  const uint64_t blocks = ((uint64_t) p->n + spb - 1) / spb;
  if (blocks == 0)
    return 0;
  const dim3 grid((uint32_t) blocks), block(kBlock);
  hipStream_t s = (hipStream_t) stream;
  switch (p->dbg) {
  case 1: hipLaunchKernelGGL((tx_segment_kernel<3, 1>), grid, block, 0, s, *p); break;
  case 2: hipLaunchKernelGGL((tx_segment_kernel<3, 2>), grid, block, 0, s, *p); break;
  case 3: hipLaunchKernelGGL((tx_segment_kernel<2, 0>), grid, block, 0, s, *p); break;
  case 4: hipLaunchKernelGGL((tx_segment_kernel<4, 0>), grid, block, 0, s, *p); break;
  case 5: hipLaunchKernelGGL((tx_segment_kernel<6, 0>), grid, block, 0, s, *p); break;
  case 6: hipLaunchKernelGGL((tx_segment_kernel<1, 0>), grid, block, 0, s, *p); break;
  case 7: hipLaunchKernelGGL((tx_segment_kernel<6, 4>), grid, block, 0, s, *p); break;
  default: hipLaunchKernelGGL((tx_segment_kernel<3, 0>), grid, block, 0, s, *p); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
