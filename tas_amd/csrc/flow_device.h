// flow_device.h -- the RX flow lookup's device code (SURVEY.md section 8f
// row 4: the batch part of fast_flows_packet_fss(),
// /root/reference/tas/fast/fast_flows.c:1084-1163), shared by the product
// launcher (flow_kernels.hip, which describes the layout) and the A/B build's
// variants (ab/ab_flow.hip).
#ifndef TASX_FLOW_DEVICE_H_
#define TASX_FLOW_DEVICE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"
#include "xsum_device.h"

namespace {

// CRC32C slice-by-4 tables: CrcTables / make_crc_tables / kCrc (xsum_device.h)

// byte-position tables for the whole 12-byte key: CRC32C from state 0 is
// linear, so flow_hash = XOR over key byte positions p of b[p][key[p]], with
// b[p][x] = CRC of byte x followed by 11 - p zero bytes: 12 independent LDS
// reads instead of a 96-step dependent chain
struct CrcKeyTables {
  uint32_t t[12][256];
};

constexpr CrcKeyTables make_crc_key_tables()
{
  CrcKeyTables T{};
  const CrcTables S = make_crc_tables();
  for (uint32_t i = 0; i < 256; ++i)
    T.t[11][i] = S.t[0][i];
  for (int p = 10; p >= 0; --p)
    for (uint32_t i = 0; i < 256; ++i)
      T.t[p][i] = (T.t[p + 1][i] >> 8) ^ S.t[0][T.t[p + 1][i] & 0xffu];
  return T;
}

__constant__ CrcKeyTables kCrcKey = make_crc_key_tables();

// SSE4.2 crc32 on one 32-bit little-endian word (crc32c_sse42_u32(w, crc)):
// slice-by-4 from the LDS copy of the tables, or bit by bit on the VALU
template <bool TAB>
__device__ __forceinline__ uint32_t crc32c_word(const uint32_t (*t)[256], uint32_t crc, uint32_t w)
{
  if constexpr (TAB)
    return crc32c_u32_tab(t, crc, w);
  return crc32c_u32(crc, w);
}

__device__ __forceinline__ uint32_t ld32b(const uint8_t *p)
{
  return ld8(p) | (ld8(p + 1) << 8) | (ld8(p + 2) << 16) | (ld8(p + 3) << 24);
}

// the 16 bytes starting at address x, from the one or two aligned chunks that
// hold its first n (<= 16) bytes (a second chunk is loaded only if needed)
__device__ __forceinline__ u32x4 load_window(const uint8_t *x, int n)
{
  const uintptr_t a = (uintptr_t) x;
  const u32x4 *c0 = (const u32x4 *) (a & ~(uintptr_t) 15);
  const u32x4 *c1 = (const u32x4 *) ((a + (uintptr_t) n - 1) & ~(uintptr_t) 15);
  return funnel16(ld16(c0, 0), ld16(c1, 0), (int) (a & 15));
}


// CRC: 0 bitwise on the VALU, 1 slice-by-4 from LDS, 2 byte-position tables
// from LDS (3: no CRC, a diagnostic build only -- wrong flow ids); CHUNK: key
// fields from 16-byte chunk loads (else byte loads)
enum { kCrcBitwise = 0, kCrcSlice4 = 1, kCrcKeyTab = 2, kCrcNone = 3 };
constexpr int kFlowFramesPerLane = 2; // the product's frames per lane

// F frames per lane (frames blockIdx.x * 256 F + f * 256 + lane): every
// level's loads of all F frames are issued together, so each lane keeps F
// dependent chains in flight -- at 8 waves per SIMD one frame per lane leaves
// 256K frames two generations of waves deep, each paying the whole chain.
// NTKEY (round 4, the product): the frame-key loads non-temporal, so the
// 33.5 MB of streamed frame lines per 256K-frame launch do not evict the
// table lines from the XCDs' L2s between launches: 256K
// lookups 11.67-11.73 us against 12.17-12.29 with L2-allocating key loads (A/B
// 9 now), the same box (profiles/r04/INDEX.md r04d).  NTFS (A/B 10): the
// flow-state key loads non-temporal too, so that the 2 MiB bucket table alone
// competes for each XCD's 4 MiB L2: slower (13.33-13.37 us)
// KPOL >= 0 (A/B 12, 13): the frame keys by a raw buffer load with that
// cache policy (aux bits: 1 sc0, 2 nt, 16 sc1) -- do uncached forms move fewer
// bytes per 12-byte key than the non-temporal global load?
template <int CRC, bool CHUNK, int F = 1, bool NTKEY = false, bool NTFS = false, int KPOL = -1>
__global__ __launch_bounds__(256) void flow_lookup_kernel(tasx_flow_params p)
{
  constexpr bool TAB = CRC == kCrcSlice4;
  __shared__ uint32_t lt[TAB ? 4 : 1][256];
  __shared__ uint32_t kt[CRC == kCrcKeyTab ? 12 : 1][256];
  uint32_t i0[F], i[F], rip[F], lip[F], l4x[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    i0[f] = blockIdx.x * (256u * F) + 256u * (uint32_t) f + threadIdx.x;
    i[f] = min(i0[f], p.n - 1u); // lanes past the batch repeat the last frame (no store)
    const uint8_t *fr = p.base + pkt_offset(p.off, p.stride, i[f]);
    // key = (local = destination, remote = source), network byte order:
    // ip.src/ip.dst are bytes [12, 20) of the IPv4 header, the ports bytes
    // [0, 4) of the TCP header
    if constexpr (CHUNK) {
      const u32x4 ipw = load_window(fr + p.ip_off + 12, 8), l4w = load_window(fr + p.l4_off, 4);
      rip[f] = ipw.x;
      lip[f] = ipw.y;
      l4x[f] = l4w.x;
    } else if (p.l4_off == p.ip_off + 20u) {
      // TAS's layout: ip.src, ip.dst and the ports are 12 contiguous bytes, one
      // unaligned dwordx3 load (gfx950 global loads take any byte address)
      u32x3u k;
      if constexpr (KPOL >= 0) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *) p.base, 0, -1, 0x00020000);
        const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(rs, (uint32_t) (fr - p.base) + p.ip_off + 12u, 0, KPOL);
        k = u32x3u{w.x, w.y, w.z};
      } else if constexpr (NTKEY) {
        k = __builtin_nontemporal_load((__attribute__((address_space(1))) const u32x3u *) (fr + p.ip_off + 12));
      } else {
        k = *(__attribute__((address_space(1))) const u32x3u *) (fr + p.ip_off + 12);
      }
      rip[f] = k.x;
      lip[f] = k.y;
      l4x[f] = k.z;
    } else {
      rip[f] = ld32b(fr + p.ip_off + 12);
      lip[f] = ld32b(fr + p.ip_off + 16);
      l4x[f] = ld32b(fr + p.l4_off);
    }
  }
  // tables into LDS while the key loads are in flight
  if constexpr (TAB) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      lt[k][threadIdx.x] = kCrc.t[k][threadIdx.x];
  }
  if constexpr (CRC == kCrcKeyTab) {
#pragma unroll
    for (int k = 0; k < 12; ++k)
      kt[k][threadIdx.x] = kCrcKey.t[k][threadIdx.x];
  }
  if constexpr (TAB || CRC == kCrcKeyTab)
    __syncthreads();
  // flow_hash: crc32c_sse42_u32(ports, crc32c_sse42_u64(lip | rip << 32, 0))
  uint32_t ports[F], h[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    ports[f] = (l4x[f] >> 16) | (l4x[f] << 16); // tcp.dest | tcp.src << 16
    if constexpr (CRC == kCrcKeyTab) {
      h[f] = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b)
        h[f] ^= kt[b][(lip[f] >> (8 * b)) & 0xffu] ^ kt[4 + b][(rip[f] >> (8 * b)) & 0xffu] ^
                kt[8 + b][(ports[f] >> (8 * b)) & 0xffu];
    } else if constexpr (CRC == kCrcNone) {
      h[f] = lip[f] ^ rip[f] ^ ports[f];
    } else {
      h[f] = crc32c_word<TAB>(lt, crc32c_word<TAB>(lt, crc32c_word<TAB>(lt, 0u, lip[f]), rip[f]), ports[f]);
    }
  }
  // buckets: entries (h + j) % ht_entries, j < NBSZ, all frames' loaded together
  uint64_t e[F][TASX_FLOWHT_NBSZ];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j)
      e[f][j] = ldg((const uint64_t *) p.flowht, (h[f] + j) % p.ht_entries);
  // candidates' keys, loaded together (non-candidates read flow 0)
  bool cand[F][TASX_FLOWHT_NBSZ];
  uint32_t fid[F][TASX_FLOWHT_NBSZ];
  u32x3 key[F][TASX_FLOWHT_NBSZ];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j) {
      const uint32_t ffid = (uint32_t) e[f][j], eh = (uint32_t) (e[f][j] >> 32);
      fid[f][j] = ffid & ((1u << TASX_FLOWHTE_POSSHIFT) - 1u);
      cand[f][j] = (ffid & TASX_FLOWHTE_VALID) && eh == h[f] && fid[f][j] < p.fs_num;
      const uint8_t *fsk = p.flowst + (uint64_t) (cand[f][j] ? fid[f][j] : 0u) * p.fs_stride + p.fs_key_off;
      if constexpr (NTFS)
        key[f][j] = __builtin_nontemporal_load((__attribute__((address_space(1))) const u32x3 *) fsk);
      else
        key[f][j] = *(__attribute__((address_space(1))) const u32x3 *) fsk;
    }
#pragma unroll
  for (int f = 0; f < F; ++f) {
    uint32_t res = TASX_FLOW_NONE;
#pragma unroll
    for (int j = (int) TASX_FLOWHT_NBSZ - 1; j >= 0; --j) // first match wins
      if (cand[f][j] && key[f][j].x == lip[f] && key[f][j].y == rip[f] && key[f][j].z == ports[f])
        res = fid[f][j];
    if (i0[f] < p.n) {
      stg(p.fid_out, i[f], res);
      if (p.hash_out)
        stg(p.hash_out, i[f], h[f]);
    }
  }
}

template <int F, bool NTKEY = false, bool NTFS = false, int KPOL = -1>
int launch_flow_f(const char *name, const tasx_flow_params *p, hipStream_t s)
{
  const uint64_t blocks = ((uint64_t) p->n + 256u * F - 1) / (256u * F);
  tasx_note_kernel(name);
  hipLaunchKernelGGL((flow_lookup_kernel<kCrcBitwise, false, F, NTKEY, NTFS, KPOL>), dim3((uint32_t) blocks), dim3(256), 0, s, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace
#endif
