// xsum_kernels.hip -- CDNA4 (gfx950) kernels for TAS's software TCP/IP checksum
// path (the --fp-no-xsumoffload branch of tcp_checksums(),
// /root/reference/tas/fast/fast_flows.c:1058-1069).
//
// Bandwidth-bound integer fold, no MFMA.  Layout and arithmetic:
//   * A packet (RAW payload, or the L4 segment of a TCP4 frame) is covered by
//     the naturally aligned 16-byte chunks [start & ~15, end rounded up).  Each
//     lane of a G-lane packet group loads whole chunks with global_load_dwordx4
//     (1 KiB per wave instruction, fully coalesced); only the first and the last
//     chunk are byte-masked.  Reading an aligned chunk that contains a valid
//     byte never crosses a page, so it cannot fault.
//   * Sums are taken over ADDRESS-aligned LE 16-bit words.  DPDK sums words
//     counted from the buffer start; for an odd start the two frames differ by
//     a byte swap of the folded result (RFC 1071 section 2(B)), applied at the end.
//   * Each lane accumulates the 32-bit words of its chunks in 64 bits (exact:
//     never wraps for packets < 2^32 words).  Because 2^16 == 1 (mod 0xffff),
//     the dword sum is congruent to the 16-bit word sum, and every end-around
//     fold keeps both the residue mod 0xffff and "zero iff all words zero" --
//     which is exactly what rte_raw_cksum returns.
//   * Group reduction: xor-shuffles inside the G-lane group.
//   * TCP4 (rte_ipv4_cksum + rte_ipv4_udptcp_cksum) depends only on the
//     residue mod 0xffff of (header sum) and of (L4 sum + pseudo-header), so the
//     zeroed checksum fields are handled by subtracting their bytes modulo
//     0xffff instead of masking the loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"

namespace {

constexpr int kBlock = 256;

// Global-address-space views: plain pointers taken from a by-value struct are
// generic to the compiler and would lower to flat_load; these lower to
// global_load_dwordx4 / global_load_ubyte / global_store_*.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gcu4;
typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ u32x4 ld16(const u32x4 *p, uint32_t i) { return ((gcu4 *) p)[i]; }
__device__ __forceinline__ uint32_t ld8(const uint8_t *p) { return *(gcu8 *) p; }
__device__ __forceinline__ void st8(uint8_t *p, uint32_t v) { *(gu8 *) p = (uint8_t) v; }
template <typename T>
__device__ __forceinline__ T ldg(const T *p, uint32_t i) { return ((__attribute__((address_space(1))) const T *) p)[i]; }
template <typename T>
__device__ __forceinline__ void stg(T *p, uint32_t i, T v) { ((__attribute__((address_space(1))) T *) p)[i] = v; }

// ---------------------------------------------------------------------------
// small integer helpers

__device__ __forceinline__ uint32_t fold64_to_18(uint64_t a)
{
  // 64 -> <= 2^33 -> < 2^18, congruent mod 0xffff, positive iff a > 0
  a = (a & 0xffffffffull) + (a >> 32);
  a = (a & 0xffffull) + (a >> 16);
  return (uint32_t) a;
}

__device__ __forceinline__ uint32_t fold32_to_16(uint32_t x)
{
  // x < 2^24 -> [0, 0xffff], 0 iff x == 0
  x = (x & 0xffffu) + (x >> 16);
  x = (x & 0xffffu) + (x >> 16);
  return x;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x)
{
  return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

// residue in [0, 0xfffe] of a folded value in [0, 0xffff]
__device__ __forceinline__ uint32_t residue(uint32_t f)
{
  return f == 0xffffu ? 0u : f;
}

// DPDK's inverted results (rte_ipv4_cksum, rte_ipv4_udptcp_cksum) as a
// function of the residue r of their folded sum: 0xffff when r == 0, else ~r.
__device__ __forceinline__ uint32_t inv_result(uint32_t r)
{
  return r == 0u ? 0xffffu : (0xffffu - r);
}

// keep bytes [lo, hi) (0 <= lo <= hi <= 16) of a 16-byte chunk
__device__ __forceinline__ u32x4 mask_chunk(u32x4 v, int lo, int hi)
{
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int l = min(max(lo - 4 * j, 0), 4);
    int h = min(max(hi - 4 * j, 0), 4);
    uint64_t mh = (1ull << (8 * h)) - 1ull;
    uint64_t ml = (1ull << (8 * l)) - 1ull;
    w[j] &= (uint32_t) (mh & ~ml);
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ uint64_t add_chunk(uint64_t acc, u32x4 v)
{
  acc += v.x;
  acc += v.y;
  acc += v.z;
  acc += v.w;
  return acc;
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v)
{
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1)
    v += __shfl_xor(v, m, 64);
  return v;
}

// Sum of the aligned-word frame over bytes [start, start + len), spread over
// the G lanes of a group (lane gl), U chunks per lane per iteration.  Returns
// this lane's partial (not yet reduced), < 2^18.
template <int G, int U>
__device__ __forceinline__ uint32_t lane_partial(const uint8_t *start, uint32_t len, int gl)
{
  if (len == 0)
    return 0;
  const uintptr_t a0 = (uintptr_t) start;
  const uintptr_t a1 = a0 + len;
  const u32x4 *c0p = (const u32x4 *) (a0 & ~(uintptr_t) 15);
  const uint32_t nch = (uint32_t) (((a1 + 15) & ~(uintptr_t) 15) - (a0 & ~(uintptr_t) 15)) >> 4;
  const int head = (int) (a0 & 15);                 // bytes to drop in chunk 0
  const int tail = (int) (a1 - ((a1 - 1) & ~(uintptr_t) 15)); // bytes kept in last chunk (1..16)
  uint64_t acc = 0;

  for (uint32_t c = (uint32_t) gl; c < nch; c += (uint32_t) (G * U)) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t) (u * G);
      if (cc < nch)
        v[u] = ld16(c0p, cc);
      else
        v[u] = u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t) (u * G);
      if (cc == 0 || cc == nch - 1) {
        const int lo = (cc == 0) ? head : 0;
        const int hi = (cc == nch - 1) ? tail : 16;
        v[u] = mask_chunk(v[u], lo, hi);
      }
      acc = add_chunk(acc, v[u]);
    }
  }
  return fold64_to_18(acc);
}

__device__ __forceinline__ uint64_t pkt_offset(const uint64_t *off, uint64_t stride, uint32_t i)
{
  return off ? ldg(off, i) : (uint64_t) i * stride;
}

// ---------------------------------------------------------------------------
// RAW: out[i] = rte_raw_cksum(base + off_i, len_i)   

template <int G, int U>
__global__ __launch_bounds__(kBlock) void raw_cksum_kernel(tasx_raw_params p)
{
  const int gl = threadIdx.x & (G - 1);
  const uint32_t gpb = kBlock / G;
  const uint32_t ngroups = gridDim.x * gpb;
  for (uint32_t i = blockIdx.x * gpb + threadIdx.x / G; i < p.n; i += ngroups) {
    const uint8_t *s = p.base + pkt_offset(p.off, p.stride, i);
    const uint32_t len = p.len ? ldg(p.len, i) : p.len0;
    uint32_t part = lane_partial<G, U>(s, len, gl);
    uint32_t tot = group_sum<G>(part);
    if (gl == 0) {
      uint32_t f = fold32_to_16(tot);
      if (((uintptr_t) s) & 1)
        f = bswap16(f);
      stg(p.out, i, (uint16_t) f);
    }
  }
}

// ---------------------------------------------------------------------------
// TCP4: per frame, tcp_checksums() flag-off branch:
//   ip.chksum  = rte_ipv4_cksum(ip)            (ip.chksum taken as 0)
//   tcp.chksum = rte_ipv4_udptcp_cksum(ip, l4) (tcp.chksum taken as 0)
// out[2i] = ip.chksum, out[2i+1] = tcp.chksum (native u16, as TAS stores them)

template <int G, int U>
__global__ __launch_bounds__(kBlock) void tcp4_cksum_kernel(tasx_tcp4_params p)
{
  static_assert(G >= 16, "header needs 11 lanes");
  const int gl = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1); // first lane of the group in the wave
  const uint32_t gpb = kBlock / G;
  const uint32_t ngroups = gridDim.x * gpb;

  for (uint32_t i = blockIdx.x * gpb + threadIdx.x / G; i < p.n; i += ngroups) {
    uint8_t *f = p.base + pkt_offset(p.off, p.stride, i);
    uint8_t *ip = f + p.ip_off;
    uint8_t *l4 = f + p.l4_off;

    // header words, relative to the header start: lanes 0..9 hold ip word gl
    uint32_t w = 0;
    if (gl < 10)
      w = ld8(ip + 2 * gl) | (ld8(ip + 2 * gl + 1) << 8);
    // total_length = bswap(word 1)
    const uint32_t w1 = (uint32_t) __shfl(w, gbase + 1, 64);
    const uint32_t tl = bswap16(w1);
    const uint32_t l4len = tl >= 20 ? tl - 20 : 0;

    // checksum field bytes of the L4 header, inside the summed range only
    uint32_t fix = 0;
    if (gl == 10 && l4len > 16) {
      uint32_t fw = ld8(l4 + 16);
      if (l4len > 17)
        fw |= ld8(l4 + 17) << 8;
      fix = (~fw) & 0xffffu; // -fw mod 0xffff, L4-start frame
    }

    // header channels: ip sum (words 0..9 but 5) and pseudo header
    // (src/dst words 6..9, proto<<8 from word 4)
    uint32_t c_ip = (gl < 10 && gl != 5) ? w : 0;
    uint32_t c_ph = (gl >= 6 && gl < 10) ? w : (gl == 4 ? (w & 0xff00u) : 0);

    uint32_t part = lane_partial<G, U>(l4, l4len, gl);

    c_ip = group_sum<G>(c_ip);
    c_ph = group_sum<G>(c_ph);
    part = group_sum<G>(part);
    fix = group_sum<G>(fix);

    if (gl == 0) {
      const uint32_t ipc = inv_result(residue(fold32_to_16(c_ip)));
      uint32_t tcpc = 0;
      if (tl >= 20) {
        uint32_t r4 = fold32_to_16(part);
        if (((uintptr_t) l4) & 1)
          r4 = bswap16(r4);
        const uint32_t lw = bswap16(l4len); // htons(l4len) as a LE word
        uint32_t s = r4 + fix + c_ph + lw;
        tcpc = inv_result(residue(fold32_to_16(s)));
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
}

template <typename K, typename P>
int launch(K kern, const P &p, uint32_t groups_per_block, int max_blocks, hipStream_t s)
{
  uint64_t blocks = ((uint64_t) p.n + groups_per_block - 1) / groups_per_block;
  if (blocks > (uint64_t) max_blocks)
    blocks = (uint64_t) max_blocks;
  if (blocks == 0)
    return 0;
  hipLaunchKernelGGL(kern, dim3((uint32_t) blocks), dim3(kBlock), 0, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace

// ---------------------------------------------------------------------------
// launchers (C ABI, internal to libtasx)

extern "C" int tasx_launch_raw(const tasx_raw_params *p, int group, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  const int maxb = 256 * 64;
  switch (group) {
  case 16: return launch(raw_cksum_kernel<16, 8>, *p, kBlock / 16, maxb, s);
  case 32: return launch(raw_cksum_kernel<32, 4>, *p, kBlock / 32, maxb, s);
  case 64: return launch(raw_cksum_kernel<64, 4>, *p, kBlock / 64, maxb, s);
  default: return -2;
  }
}

extern "C" int tasx_launch_tcp4(const tasx_tcp4_params *p, int group, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  const int maxb = 256 * 64;
  switch (group) {
  case 16: return launch(tcp4_cksum_kernel<16, 8>, *p, kBlock / 16, maxb, s);
  case 32: return launch(tcp4_cksum_kernel<32, 4>, *p, kBlock / 32, maxb, s);
  case 64: return launch(tcp4_cksum_kernel<64, 4>, *p, kBlock / 64, maxb, s);
  default: return -2;
  }
}
