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

// store bytes [lo, hi) of v into the 16-byte aligned chunk at cp
__device__ __forceinline__ void store_range(uint8_t *cp, u32x4 v, int lo, int hi)
{
  if (lo == 0 && hi == 16) {
    __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int l = min(max(lo - 4 * j, 0), 4), h = min(max(hi - 4 * j, 0), 4);
    if (l == 0 && h == 4)
      stg((uint32_t *) cp, (uint32_t) j, w[j]);
    else
      for (int b = l; b < h; ++b)
        st8(cp + 4 * j + b, w[j] >> (8 * b));
  }
}

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
  uint8_t *f = p.frames + frame_off;
  uint8_t *ip = f + p.ip_off;
  uint8_t *l4 = f + p.l4_off;
  const uint8_t *src = p.shm + tx_base; // the flow's TX buffer
  // header words (bytes never written by this kernel before the final stores)
  const uint32_t tl = (ld8(ip + 2) << 8) | ld8(ip + 3);
  uint32_t w = 0;
  if (gl < 10)
    w = ld8(ip + 2 * gl) | (ld8(ip + 2 * gl + 1) << 8);
  // l4-relative coordinates: payload D = [dlo, dhi), checksummed S = [0, slen)
  const int dlo = (int) (hl - p.l4_off), dhi = dlo + (int) pay;
  const Chunks<U> r = chunk_range<U>(l4, (uint32_t) dhi);
  const int wrap = (int) (tx_len - pos); // payload index of the buffer wrap
  const uintptr_t s1 = (uintptr_t) src + pos;      // payload byte j at s1 + j (j < wrap)
  const uintptr_t s2 = (uintptr_t) src - wrap;     // ... or at s2 + j (j >= wrap)
  const uint32_t len = tl >= 20 ? tl - 20 : 0;
  const int send = min((int) len, dhi); // main pass sums [0, send)
  const int p16 = r.head + 16;          // chunk position of tcp.chksum

  uint64_t acc = 0;
  for (uint32_t c = (uint32_t) gl; c < r.nch; c += 16u * U) {
    u32x4 fa[U], sa[U], sb[U];
    // issue every load of this round first
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + 16u * u;
      const int o = 16 * (int) cc - r.head; // l4-relative offset of chunk byte 0
      const int blo = min(max(dlo - o, 0), 16), bhi = min(max(dhi - o, 0), 16);
      fa[u] = sa[u] = sb[u] = u32x4{0, 0, 0, 0};
      if (cc < r.nch && o < dlo)
        fa[u] = ld16nt(r.c0p, cc);
      if (cc < r.nch && blo < bhi) {
        const int j0 = o - dlo;
        const bool p2 = j0 + blo >= wrap;
        const uintptr_t S = (p2 ? s2 : s1) + (intptr_t) j0;
        const uintptr_t ca = S & ~(uintptr_t) 15;
        // a window straddling the buffer end is byte-gathered below; its
        // chunk loads stay inside the first piece
        const int bh = (!p2 && j0 + bhi > wrap) ? wrap - j0 : bhi;
        const uintptr_t lo_c = (S + blo) & ~(uintptr_t) 15, hi_c = (S + bh - 1) & ~(uintptr_t) 15;
        sa[u] = ld16nt((const u32x4 *) lo_c, 0);
        sb[u] = ld16nt((const u32x4 *) (ca + 16 < hi_c ? ca + 16 : hi_c), 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + 16u * u;
      if (cc >= r.nch)
        continue;
      const int o = 16 * (int) cc - r.head;
      const int blo = min(max(dlo - o, 0), 16), bhi = min(max(dhi - o, 0), 16);
      u32x4 val = fa[u];
      if (blo < bhi) {
        const int j0 = o - dlo;
        u32x4 g;
        if (j0 + blo < wrap && j0 + bhi > wrap) {
          // the window straddles the end of the circular buffer: byte gather
          uint32_t gw[4] = {0, 0, 0, 0};
#pragma unroll
          for (int b = 0; b < 16; ++b) {
            const int j = j0 + b;
            if (b >= blo && b < bhi)
              gw[b >> 2] |= ld8((const uint8_t *) ((j < wrap ? s1 : s2) + (intptr_t) j)) << (8 * (b & 3));
          }
          g = u32x4{gw[0], gw[1], gw[2], gw[3]};
        } else {
          const uintptr_t S = ((j0 + blo >= wrap) ? s2 : s1) + (intptr_t) j0;
          g = funnel16(sa[u], sb[u], (int) (S & 15));
        }
        store_range((uint8_t *) (r.c0p + cc), g, blo, bhi);
        val = merge_at(val, g, blo);
      }
      // checksummed bytes of this chunk: [0, send), tcp.chksum taken as zero
      const int lo = min(max(-o, 0), 16), hi = min(max(send - o, 0), 16);
      if (lo > 0 || hi < 16)
        val = mask_chunk(val, lo, hi);
      if ((int) cc == (p16 >> 4))
        val = clear_byte(val, p16 & 15);
      if ((int) cc == ((p16 + 1) >> 4))
        val = clear_byte(val, (p16 + 1) & 15);
      acc += (uint64_t) val.x + val.y + val.z + val.w;
    }
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
  if (gl == 15) {
    const uint32_t ipc = inv_result(residue(fold32_to_16(s_ip)));
    uint32_t tcpc = 0;
    if (tl >= 20) {
      uint32_t r4 = fold32_to_16(part);
      if (r.head & 1)
        r4 = bswap16(r4);
      tcpc = inv_result(residue(fold32_to_16(r4 + s_ph + bswap16(len))));
    }
    st8(ip + 10, ipc);
    st8(ip + 11, ipc >> 8);
    st8(l4 + 16, tcpc);
    st8(l4 + 17, tcpc >> 8);
    if (p.out)
      stg(p.out, i, ipc | (tcpc << 16));
  }
}

} // namespace

extern "C" int tasx_launch_txseg(const tasx_txseg_params *p, void *stream)
{
  constexpr uint64_t spb = kBlock / 16;
  const uint64_t blocks = ((uint64_t) p->n + spb - 1) / spb;
  if (blocks == 0)
    return 0;
  hipLaunchKernelGGL(tx_segment_kernel<6>, dim3((uint32_t) blocks), dim3(kBlock), 0,
                     (hipStream_t) stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
