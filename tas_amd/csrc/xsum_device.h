// xsum_device.h -- device helpers shared by the gfx950 checksum kernels
// (xsum_kernels.hip, txseg_kernels.hip): global-address-space loads/stores,
// exact end-around-carry folds, 16-byte chunk ranges and the 16-lane DPP
// group reduction.  See xsum_kernels.hip for the arithmetic argument.
#ifndef TASX_XSUM_DEVICE_H_
#define TASX_XSUM_DEVICE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {


constexpr int kBlock = 256;

// Global-address-space views: plain pointers taken from a by-value struct are
// generic to the compiler and would lower to flat_load; these lower to
// global_load_dwordx4 / global_load_ubyte / global_store_*.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x3u __attribute__((ext_vector_type(3), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4 gcu4;
typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ u32x4 ld16(const u32x4 *p, uint32_t i) { return ((gcu4 *) p)[i]; }
// streaming (non-temporal) 16-byte load: packet bytes are read exactly once
// (MI355X_MICROARCH.md nt-weights: nt cuts issue->landed latency ~18%)
__device__ __forceinline__ u32x4 ld16nt(const u32x4 *p, uint32_t i)
{
  return __builtin_nontemporal_load(&((gcu4 *) p)[i]);
}
// the same at a 32-bit byte offset from a uniform base: global_load_dwordx4
// v, v_off, s[base] (one VGPR per address)
__device__ __forceinline__ u32x4 ld16nt_off(const uint8_t *base, uint32_t off)
{
  return __builtin_nontemporal_load((gcu4 *) (base + off));
}
// the same, L2-allocating (lines that neighbouring loads share are fetched once)
__device__ __forceinline__ u32x4 ld16_off(const uint8_t *base, uint32_t off) { return *(gcu4 *) (base + off); }
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

// The logical block of hardware block b in a grid of nb, XCD-ordered: the
// dispatcher places blocks round-robin over the 8 XCDs (b -> XCD b % 8); in
// every window of 8 S consecutive blocks (S = 2^(xrun - 1)) XCD x takes the S
// consecutive logical blocks [x S, x S + S) of the window, in order, so each
// XCD streams its own contiguous run while the 8 runs stay adjacent.  Blocks
// past the last whole window, and every block when xrun = 0, keep grid order.
// A bijection on [0, nb); xrun is uniform (a kernel argument).
__device__ __forceinline__ uint32_t xcd_run(uint32_t b, uint32_t nb, uint32_t xrun)
{
  if (xrun == 0u)
    return b;
  const uint32_t sh = xrun - 1u, wmask = (8u << sh) - 1u;
  if (b >= (nb & ~wmask))
    return b;
  const uint32_t o = b & wmask;
  return (b & ~wmask) + ((o & 7u) << sh) + (o >> 3);
}

// ---------------------------------------------------------------------------
// 16-lane packet groups (one DPP row each), one block per 16 packets.

__device__ __forceinline__ uint32_t row_sum16(uint32_t v)
{
  // Hillis-Steele inclusive scan inside each 16-lane DPP row; lane 15 = row sum
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, false); // row_shr:1
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, false); // row_shr:2
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, false); // row_shr:4
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, false); // row_shr:8
  return v;
}

// G-lane group total (G = 16, 32, 64; groups aligned in the wave) in the
// group's last lane: DPP row scan, then row_bcast15 / row_bcast31 across rows
template <int G>
__device__ __forceinline__ uint32_t group_total(uint32_t v)
{
  v = row_sum16(v);
  if constexpr (G >= 32) // rows 1, 3 += lane 15 of rows 0, 2
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false);
  if constexpr (G == 64) // rows 2, 3 += lane 31
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false);
  return v;
}

// acc + both LE 16-bit words of w (v_sad_u16 against 0): the address-aligned
// 16-bit word sum in one VALU op per dword, exact in 32 bits
__device__ __forceinline__ uint32_t sadw(uint32_t w, uint32_t acc)
{
  return __builtin_amdgcn_sad_u16(w, 0u, acc);
}

__device__ __forceinline__ uint32_t sad4(u32x4 v, uint32_t acc)
{
  return sadw(v.w, sadw(v.z, sadw(v.y, sadw(v.x, acc))));
}

// DPP lane moves inside 16-lane rows (lanes without a source get 0)
template <int K>
__device__ __forceinline__ uint32_t row_shr(uint32_t v)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x110 + K, 0xf, 0xf, false);
}
template <int K>
__device__ __forceinline__ uint32_t row_shl(uint32_t v)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x100 + K, 0xf, 0xf, false);
}

// lane K of each 16-lane row broadcast to the whole row (DPP row_newbcast)
template <int K>
__device__ __forceinline__ uint32_t row_newbcast(uint32_t v)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x150 + K, 0xf, 0xf, false);
}

// byte mask of [0, h) over a 16-byte chunk as two qwords (0 <= h <= 16)
__device__ __forceinline__ void below_mask(uint32_t h, uint64_t &lo, uint64_t &hi)
{
  const uint64_t a = ~(~0ull << (8u * (h & 7u))); // bytes [0, h mod 8)
  lo = h >= 8u ? ~0ull : a;
  hi = h >= 16u ? ~0ull : (h >= 8u ? a : 0ull);
}

// word sum (sad) of the bytes [0, h) / [h, 16) of a 16-byte chunk (0 <= h <= 16)
__device__ __forceinline__ uint32_t sad_below(u32x4 v, uint32_t h)
{
  uint64_t lo, hi;
  below_mask(h, lo, hi);
  return sad4(u32x4{v.x & (uint32_t) lo, v.y & (uint32_t) (lo >> 32), v.z & (uint32_t) hi,
                    v.w & (uint32_t) (hi >> 32)}, 0u);
}
__device__ __forceinline__ uint32_t sad_from(u32x4 v, uint32_t h)
{
  uint64_t lo, hi;
  below_mask(h, lo, hi);
  return sad4(u32x4{v.x & ~(uint32_t) lo, v.y & ~(uint32_t) (lo >> 32), v.z & ~(uint32_t) hi,
                    v.w & ~(uint32_t) (hi >> 32)}, 0u);
}

// sum of the dwords of chunk v restricted to bytes [0, h) (0 <= h <= 16)
__device__ __forceinline__ uint64_t chunk_prefix_sum(u32x4 v, int h)
{
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = min(max(h - 4 * j, 0), 4);
    s += w[j] & (uint32_t) ((1ull << (8 * b)) - 1ull);
  }
  return s;
}

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

// byte b (0..15) of a 16-byte chunk
__device__ __forceinline__ uint32_t chunk_byte(u32x4 v, int b)
{
  const uint32_t w = (b < 4) ? v.x : (b < 8) ? v.y : (b < 12) ? v.z : v.w;
  return (w >> (8 * (b & 3))) & 0xffu;
}

template <int U>
struct Chunks {
  const u32x4 *c0p;
  uint32_t nch;
  int head, tail; // bytes dropped at the start of chunk 0 / kept in chunk nch-1
};

template <int U>
__device__ __forceinline__ Chunks<U> chunk_range(const uint8_t *start, uint32_t len)
{
  Chunks<U> r;
  const uintptr_t a0 = (uintptr_t) start, a1 = a0 + len;
  r.c0p = (const u32x4 *) (a0 & ~(uintptr_t) 15);
  r.nch = len ? (uint32_t) ((((a1 + 15) & ~(uintptr_t) 15) - (a0 & ~(uintptr_t) 15)) >> 4) : 0u;
  r.head = (int) (a0 & 15);
  r.tail = (int) (a1 - ((a1 - 1) & ~(uintptr_t) 15));
  return r;
}

// this lane's exact partial over the group's chunks gl, gl+G, ... (G lanes)
template <int U, int G = 16>
__device__ __forceinline__ uint32_t group_lane_sum(const Chunks<U> &r, int gl)
{
  static_assert(G * U >= 8, "the 128-byte phase lies in the first round");
  uint64_t acc = 0;
  if (r.nch == 0)
    return 0;
  // Rounds start on 128-byte lines: the range is indexed from the line holding
  // chunk 0 (ph chunks earlier, same line, never loaded past).  With rounds at
  // the range's own 16-byte phase, the line a round ends in is the next one's
  // first line, and the non-temporal loads fetch it twice (a 64 KB TSO segment:
  // ~43 extra lines).
  const uint32_t ph = (uint32_t) (((uintptr_t) r.c0p >> 4) & 7u);
  const u32x4 *cp = r.c0p - ph;
  const uint32_t n = r.nch + ph;
  for (uint32_t c = (uint32_t) gl; c < n; c += (uint32_t) G * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld16nt(cp, max(min(c + (uint32_t) G * u, n - 1), ph));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = c + (uint32_t) G * u;
      const bool keep = k >= ph && k < n;
      acc += keep ? (uint64_t) v[u].x + v[u].y + v[u].z + v[u].w : 0ull;
    }
    // boundary fix-ups: drop bytes [0, head) of chunk 0 (index ph), [tail, 16) of chunk nch-1
    if (r.head && c == ph % G) {
      u32x4 h = v[0];
#pragma unroll
      for (int u = 1; u < U; ++u)
        if (ph / G == (uint32_t) u)
          h = v[u];
      acc -= chunk_prefix_sum(h, r.head);
    }
    const uint32_t last = n - 1;
    if (last >= c && last < c + (uint32_t) G * U && ((last - c) % G) == 0 && r.tail < 16) {
      const uint32_t ut = (last - c) / G;
      u32x4 t = v[0];
#pragma unroll
      for (int u = 1; u < U; ++u)
        if (ut == (uint32_t) u)
          t = v[u];
      acc -= (uint64_t) t.x + t.y + t.z + t.w - chunk_prefix_sum(t, r.tail);
    }
  }
  return fold64_to_18(acc);
}

// flow_hash (tas/fast/fast_flows.c:1078-1082): SSE4.2 crc32 semantics,
// crc32c_sse42_u32(ports, crc32c_sse42_u64(lip | rip << 32, 0)), bit by bit on
// the VALU (the same arithmetic as flow_kernels.hip's product form)
__device__ __forceinline__ uint32_t crc32c_u32(uint32_t crc, uint32_t w)
{
  crc ^= w;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    crc = (crc >> 1) ^ (0x82f63b78u & (0u - (crc & 1u)));
  return crc;
}
__device__ __forceinline__ uint32_t tas_flow_hash(uint32_t lip, uint32_t rip, uint32_t ports)
{
  return crc32c_u32(crc32c_u32(crc32c_u32(0u, lip), rip), ports);
}

constexpr uint32_t kPoly = 0x82f63b78u; // CRC32C (Castagnoli), reflected

// SSE4.2 crc32 on one 32-bit little-endian word from slice-by-4 tables in LDS
// (t[k][x] = CRC of byte x followed by k zero bytes, init 0)
__device__ __forceinline__ uint32_t crc32c_u32_tab(const uint32_t (*t)[256], uint32_t crc, uint32_t w)
{
  crc ^= w;
  return t[3][crc & 0xffu] ^ t[2][(crc >> 8) & 0xffu] ^ t[1][(crc >> 16) & 0xffu] ^ t[0][crc >> 24];
}

// fast_flows_packet_fss lookups (fast_flows.c:1084-1163), F frames per lane:
// lookup block `blk` of BS lanes takes frames blk * BS * F + f * BS + lane,
// TAS's header layout (l4_off == ip_off + 20: the 12 key bytes in one
// unaligned dwordx3 load), every load of a level issued for all F frames
// before any is used.  The split-grid blocks of tcp4_tas14_kernel<...,flow>
// (xsum_kernels.hip) run it; flow_kernels.hip's flow_lookup_kernel is the same
// arithmetic for any layout.  P: tasx_tcp4_params or tasx_flow_params.
template <int F, int BS, typename P>
__device__ __forceinline__ void flow_lookup_lanes_at(const P &p, const uint32_t (&i0)[F])
{
  static_assert(BS == 256, "one table entry per lane");
  constexpr uint32_t kNb = TASX_FLOWHT_NBSZ;
  // the CRC32C slice-by-4 tables in LDS (4 KiB; ~300 VALU per frame less than
  // the bitwise CRC, which cost the one-pass RX kernel 0.7 us per 64K frames)
  __shared__ uint32_t lt[4][256];
  uint32_t i[F], rip[F], lip[F], ports[F], h[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    i[f] = min(i0[f], p.n - 1u); // lanes past the batch repeat the last frame (no store)
    const uint8_t *fr = p.base + pkt_offset(p.off, p.stride, i[f]);
    const u32x3u k = *(__attribute__((address_space(1))) const u32x3u *) (fr + p.ip_off + 12);
    rip[f] = k.x;
    lip[f] = k.y;
    ports[f] = (k.z >> 16) | (k.z << 16); // tcp.dest | tcp.src << 16
  }
  // the tables built while the key loads are in flight (no memory in the
  // chain): T0 by eight bit steps, Tk[x] = T(k-1)[x] >> 8 ^ T0[T(k-1)[x] & 0xff]
  {
    uint32_t c = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    lt[0][threadIdx.x] = c;
    __syncthreads();
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      c = (c >> 8) ^ lt[0][c & 0xffu];
      lt[k][threadIdx.x] = c;
    }
    __syncthreads();
  }
#pragma unroll
  for (int f = 0; f < F; ++f)
    h[f] = crc32c_u32_tab(lt, crc32c_u32_tab(lt, crc32c_u32_tab(lt, 0u, lip[f]), rip[f]), ports[f]);
  uint64_t e[F][kNb];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (uint32_t j = 0; j < kNb; ++j)
      e[f][j] = ldg((const uint64_t *) p.flowht, (h[f] + j) % p.ht_entries);
  bool cand[F][kNb];
  uint32_t fid[F][kNb];
  u32x3 key[F][kNb];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (uint32_t j = 0; j < kNb; ++j) {
      const uint32_t ef = (uint32_t) e[f][j], eh = (uint32_t) (e[f][j] >> 32);
      fid[f][j] = ef & ((1u << TASX_FLOWHTE_POSSHIFT) - 1u);
      cand[f][j] = (ef & TASX_FLOWHTE_VALID) && eh == h[f] && fid[f][j] < p.fs_num;
      const uint8_t *fsk = p.flowst + (uint64_t) (cand[f][j] ? fid[f][j] : 0u) * p.fs_stride + p.fs_key_off;
      key[f][j] = *(__attribute__((address_space(1))) const u32x3 *) fsk;
    }
#pragma unroll
  for (int f = 0; f < F; ++f) {
    uint32_t res = TASX_FLOW_NONE;
#pragma unroll
    for (int j = (int) kNb - 1; j >= 0; --j) // first match wins
      if (cand[f][j] && key[f][j].x == lip[f] && key[f][j].y == rip[f] && key[f][j].z == ports[f])
        res = fid[f][j];
    if (i0[f] < p.n) {
      stg(p.fid_out, i[f], res);
      if (p.hash_out)
        stg(p.hash_out, i[f], h[f]);
    }
  }
}

} // namespace
#endif
