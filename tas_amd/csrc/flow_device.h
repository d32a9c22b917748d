// flow_device.h -- the RX flow lookup's device code (SURVEY.md section 8f
// row 4: the batch part of fast_flows_packet_fss(),
// /root/reference/tas/fast/fast_flows.c:1084-1163), launched by
// flow_kernels.hip (which describes the layout); the comparison build's bare
// access pattern (ab/ab_flow.hip) shares kFlowFramesPerLane.
#ifndef TASX_FLOW_DEVICE_H_
#define TASX_FLOW_DEVICE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"
#include "xsum_device.h"

namespace {

__device__ __forceinline__ uint32_t ld32b(const uint8_t *p)
{
  return ld8(p) | (ld8(p + 1) << 8) | (ld8(p + 2) << 16) | (ld8(p + 3) << 24);
}

constexpr int kFlowFramesPerLane = 2; // the product's frames per lane

// F frames per lane (frames blockIdx.x * 256 F + f * 256 + lane): every
// level's loads of all F frames are issued together, so each lane keeps F
// dependent chains in flight -- at 8 waves per SIMD one frame per lane leaves
// 256K frames two generations of waves deep, each paying the whole chain.
// The frame-key loads are non-temporal (round 4), so the 33.5 MB of streamed
// frame lines per 256K-frame launch do not evict the table lines from the
// XCDs' L2s between launches: 256K lookups 11.67-11.73 us
// against 12.17-12.29 with L2-allocating key loads, the same box
// (profiles/r04/INDEX.md r04d).  CRC32C bit by bit on the VALU: slice-by-4
// and byte-position tables from LDS measured the same (the CRC is off the
// critical path); non-temporal flow-state keys, raw buffer key loads and the
// hash-range-partitioned lookup lost (profiles/r01_flow_variants.jsonl,
// profiles/r04/INDEX.md r04i) and are gone from the source (round 6).
template <int F>
__global__ __launch_bounds__(256) void flow_lookup_kernel(tasx_flow_params p)
{
  uint32_t i0[F], i[F], rip[F], lip[F], l4x[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    i0[f] = blockIdx.x * (256u * F) + 256u * (uint32_t) f + threadIdx.x;
    i[f] = min(i0[f], p.n - 1u); // lanes past the batch repeat the last frame (no store)
    const uint8_t *fr = p.base + pkt_offset(p.off, p.stride, i[f]);
    // key = (local = destination, remote = source), network byte order:
    // ip.src/ip.dst are bytes [12, 20) of the IPv4 header, the ports bytes
    // [0, 4) of the TCP header
    if (p.l4_off == p.ip_off + 20u) {
      // TAS's layout: ip.src, ip.dst and the ports are 12 contiguous bytes, one
      // unaligned dwordx3 load (gfx950 global loads take any byte address)
      const u32x3u k = __builtin_nontemporal_load((__attribute__((address_space(1))) const u32x3u *) (fr + p.ip_off + 12));
      rip[f] = k.x;
      lip[f] = k.y;
      l4x[f] = k.z;
    } else {
      rip[f] = ld32b(fr + p.ip_off + 12);
      lip[f] = ld32b(fr + p.ip_off + 16);
      l4x[f] = ld32b(fr + p.l4_off);
    }
  }
  // flow_hash: crc32c_sse42_u32(ports, crc32c_sse42_u64(lip | rip << 32, 0))
  uint32_t ports[F], h[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    ports[f] = (l4x[f] >> 16) | (l4x[f] << 16); // tcp.dest | tcp.src << 16
    h[f] = crc32c_u32(crc32c_u32(crc32c_u32(0u, lip[f]), rip[f]), ports[f]);
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

template <int F>
int launch_flow_f(const char *name, const tasx_flow_params *p, hipStream_t s)
{
  const uint64_t blocks = ((uint64_t) p->n + 256u * F - 1) / (256u * F);
  tasx_note_kernel(name);
  hipLaunchKernelGGL((flow_lookup_kernel<F>), dim3((uint32_t) blocks), dim3(256), 0, s, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace
#endif
