// ab/ab_flow.hip -- A/B build only (libtasx_ab.so): the RX flow lookup's
// variants kept for comparisons (tools/flow_probe.py, tools/flow_ab.sh;
// profiles/r01_flow_variants.jsonl, profiles/r04/INDEX.md r04i) and the bare
// access pattern bench.py prices the lookup against.  None of it is in the
// product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../tasx_kernels.h"
#include "../flow_device.h"

namespace {
// The lookup's access pattern with no hashing or key logic (the ceiling its
// dependent chain allows, tools/flow_ceiling.hip): the 12-byte key of each
// frame (HBM), then its 4-entry bucket (flowht), then the candidate flow's key
// line plus three reads of flow 0 (flowst), each level dependent on the last.
__device__ __forceinline__ uint32_t mix32(uint32_t x)
{
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  return x;
}

__global__ __launch_bounds__(256) void flow_pattern_kernel(tasx_flow_params p)
{
  constexpr int F = kFlowFramesPerLane; // the product's frames per lane
  uint32_t i0[F], i[F], h[F], r[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    i0[f] = blockIdx.x * (256u * F) + 256u * (uint32_t) f + threadIdx.x;
    i[f] = min(i0[f], p.n - 1u);
    const uint8_t *fr = p.base + pkt_offset(p.off, p.stride, i[f]);
    // the product's key load (non-temporal since round 4)
    const u32x3u k = __builtin_nontemporal_load((__attribute__((address_space(1))) const u32x3u *) (fr + p.ip_off + 12));
    h[f] = mix32(k.x ^ k.y ^ k.z);
  }
  uint64_t e[F][TASX_FLOWHT_NBSZ];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j)
      e[f][j] = ldg((const uint64_t *) p.flowht, (h[f] + j) % p.ht_entries);
#pragma unroll
  for (int f = 0; f < F; ++f) {
    r[f] = 0;
#pragma unroll
    for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j)
      r[f] += (uint32_t) e[f][j] ^ (uint32_t) (e[f][j] >> 32);
  }
  u32x3 key[F][TASX_FLOWHT_NBSZ];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j) {
      const uint32_t fid = j == 0 ? mix32(h[f] ^ r[f]) % p.fs_num : 0u;
      key[f][j] = *(__attribute__((address_space(1))) const u32x3 *) (p.flowst + (uint64_t) fid * p.fs_stride +
                                                                      p.fs_key_off);
    }
#pragma unroll
  for (int f = 0; f < F; ++f) {
#pragma unroll
    for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j)
      r[f] ^= key[f][j].x ^ key[f][j].y ^ key[f][j].z;
    if (i0[f] < p.n)
      stg(p.fid_out, i[f], r[f]);
  }
}

// A/B 11: the hash-range-partitioned lookup, two
// launches.  flow_route_kernel: per frame the key (non-temporal) and its hash
// (hash_out in frame order), then a 16-byte record {key, frame index} into
// the region of (bucket slice x = (h mod entries) / (entries / 8), route
// block) -- LDS counters, no global atomics.  flow_probe_kernel: workgroup b
// serves slice b mod 8, so (with the observed round-robin placement) every
// slice's bucket lines are read on one XCD and that XCD's L2 serves its
// 1/8 of flowht (256 KiB in TAS's table) to all its lookups; then the
// flow-state check as the product does it (flowst unpartitioned) and fid_out
// by frame index.
constexpr uint32_t kRouteFrames = 512;  // frames per route block = records per region
constexpr uint32_t kProbeRegions = 8;   // regions per probe block

__global__ __launch_bounds__(256) void flow_route_kernel(tasx_flow_params p, u32x4 *rec, uint32_t *cnt)
{
  __shared__ uint32_t s_cnt[8];
  if (threadIdx.x < 8)
    s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t slice = (p.ht_entries + 7u) / 8u;
  u32x3u k[2];
  uint32_t i0[2], i[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    i0[f] = blockIdx.x * kRouteFrames + 256u * (uint32_t) f + threadIdx.x;
    i[f] = min(i0[f], p.n - 1u);
    const uint8_t *fr = p.base + pkt_offset(p.off, p.stride, i[f]);
    k[f] = __builtin_nontemporal_load((__attribute__((address_space(1))) const u32x3u *) (fr + p.ip_off + 12));
  }
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const uint32_t ports = (k[f].z >> 16) | (k[f].z << 16);
    const uint32_t h = tas_flow_hash(k[f].y, k[f].x, ports);
    if (i0[f] < p.n) {
      if (p.hash_out)
        stg(p.hash_out, i[f], h);
      const uint32_t x = min((h % p.ht_entries) / slice, 7u);
      const uint32_t pos = atomicAdd(&s_cnt[x], 1u);
      rec[(uint64_t) (x * gridDim.x + blockIdx.x) * kRouteFrames + pos] = u32x4{k[f].x, k[f].y, k[f].z, i[f]};
    }
  }
  __syncthreads();
  if (threadIdx.x < 8)
    cnt[threadIdx.x * gridDim.x + blockIdx.x] = s_cnt[threadIdx.x];
}

__global__ __launch_bounds__(256) void flow_probe_kernel(tasx_flow_params p, const u32x4 *rec, const uint32_t *cnt,
                                                         uint32_t nrb, uint32_t M)
{
  __shared__ uint32_t s_pre[kProbeRegions + 1];
  const uint32_t g = blockIdx.x % 8u, m = blockIdx.x / 8u;
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (uint32_t j = 0; j < kProbeRegions; ++j) {
      s_pre[j] = a;
      const uint32_t r = m + j * M;
      a += r < nrb ? cnt[g * nrb + r] : 0u;
    }
    s_pre[kProbeRegions] = a;
  }
  __syncthreads();
  const uint32_t total = s_pre[kProbeRegions];
  for (uint32_t base = 0; base < total; base += 512u) {
    uint32_t t[2], idx[2], lip[2], rip[2], ports[2], h[2];
    bool live[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      t[f] = base + 256u * (uint32_t) f + threadIdx.x;
      live[f] = t[f] < total;
      const uint32_t tt = live[f] ? t[f] : 0u;
      uint32_t j = 0;
#pragma unroll
      for (uint32_t q = 1; q < kProbeRegions; ++q)
        j += tt >= s_pre[q] ? 1u : 0u;
      const u32x4 v = live[f] ? rec[(uint64_t) (g * nrb + m + j * M) * kRouteFrames + (tt - s_pre[j])]
                              : u32x4{0u, 0u, 0u, 0u};
      rip[f] = v.x;
      lip[f] = v.y;
      ports[f] = (v.z >> 16) | (v.z << 16);
      idx[f] = v.w;
      h[f] = tas_flow_hash(lip[f], rip[f], ports[f]);
    }
    uint64_t e[2][TASX_FLOWHT_NBSZ];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j)
        e[f][j] = ldg((const uint64_t *) p.flowht, (h[f] + j) % p.ht_entries);
    bool cand[2][TASX_FLOWHT_NBSZ];
    uint32_t fid[2][TASX_FLOWHT_NBSZ];
    u32x3 key[2][TASX_FLOWHT_NBSZ];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j) {
        const uint32_t ffid = (uint32_t) e[f][j], eh = (uint32_t) (e[f][j] >> 32);
        fid[f][j] = ffid & ((1u << TASX_FLOWHTE_POSSHIFT) - 1u);
        cand[f][j] = (ffid & TASX_FLOWHTE_VALID) && eh == h[f] && fid[f][j] < p.fs_num;
        key[f][j] = *(__attribute__((address_space(1))) const u32x3 *) (p.flowst +
            (uint64_t) (cand[f][j] ? fid[f][j] : 0u) * p.fs_stride + p.fs_key_off);
      }
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      uint32_t res = TASX_FLOW_NONE;
#pragma unroll
      for (int j = (int) TASX_FLOWHT_NBSZ - 1; j >= 0; --j)
        if (cand[f][j] && key[f][j].x == lip[f] && key[f][j].y == rip[f] && key[f][j].z == ports[f])
          res = fid[f][j];
      if (live[f])
        stg(p.fid_out, idx[f], res);
    }
  }
}
} // namespace

// A/B 11's scratch: records and region counts, grown on demand, never freed
static u32x4 *g_part_rec;
static uint32_t *g_part_cnt;
static size_t g_part_blocks;

static int launch_flow_partitioned(const tasx_flow_params *p, hipStream_t s)
{
  const uint32_t nrb = (p->n + kRouteFrames - 1) / kRouteFrames;
  if (nrb > g_part_blocks) {
    if (hipMalloc((void **) &g_part_rec, (size_t) 8 * nrb * kRouteFrames * sizeof(u32x4)) != hipSuccess ||
        hipMalloc((void **) &g_part_cnt, (size_t) 8 * nrb * sizeof(uint32_t)) != hipSuccess)
      return -1;
    g_part_blocks = nrb;
  }
  const uint32_t M = (nrb + kProbeRegions - 1) / kProbeRegions;
  tasx_note_kernel("flow_route_kernel + flow_probe_kernel");
  hipLaunchKernelGGL(flow_route_kernel, dim3(nrb), dim3(256), 0, s, *p, g_part_rec, g_part_cnt);
  hipLaunchKernelGGL(flow_probe_kernel, dim3(8u * M), dim3(256), 0, s, *p, (const u32x4 *) g_part_rec,
                     (const uint32_t *) g_part_cnt, nrb, M);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A/B build only (include/tasx_ext.h): the flow lookup's bare access pattern
extern "C" int tasx_ab_flow_pattern(const void *base, uint64_t stride, uint32_t n, uint32_t ip_off,
    const void *flowht, uint32_t ht_entries, const void *flowst, uint32_t fs_num, uint32_t fs_stride,
    uint32_t fs_key_off, uint32_t *out, void *stream)
{
  tasx_flow_params p = {};
  p.base = (const uint8_t *) base;
  p.stride = stride;
  p.n = n;
  p.ip_off = ip_off;
  p.flowht = (const uint32_t *) flowht;
  p.ht_entries = ht_entries;
  p.flowst = (const uint8_t *) flowst;
  p.fs_num = fs_num;
  p.fs_stride = fs_stride;
  p.fs_key_off = fs_key_off;
  p.fid_out = out;
  if (n == 0)
    return 0;
  tasx_note_kernel("flow_pattern_kernel");
  hipLaunchKernelGGL(flow_pattern_kernel, dim3((n + 256u * kFlowFramesPerLane - 1) / (256u * kFlowFramesPerLane)),
                     dim3(256), 0, (hipStream_t) stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the variants of tasx_launch_flow_lookup this build adds (TASX_EXT_PASS: the product's)
extern "C" TASX_INTERNAL int ab_launch_flow_lookup(const tasx_flow_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  const dim3 g((uint32_t) (((uint64_t) p->n + 255) / 256)), b(256); // one frame per lane
  switch (variant) {
  case 2: tasx_note_kernel("flow_lookup_kernel<bitwise,chunk>"); hipLaunchKernelGGL((flow_lookup_kernel<kCrcBitwise, true>), g, b, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 3: tasx_note_kernel("flow_lookup_kernel<slice4>"); hipLaunchKernelGGL((flow_lookup_kernel<kCrcSlice4, false>), g, b, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 4: tasx_note_kernel("flow_lookup_kernel<slice4,chunk>"); hipLaunchKernelGGL((flow_lookup_kernel<kCrcSlice4, true>), g, b, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
#ifdef TASX_FLOW_NOCRC_DIAG
  case 5: tasx_note_kernel("flow_lookup_kernel<nocrc>"); hipLaunchKernelGGL((flow_lookup_kernel<kCrcNone, false>), g, b, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
#else
  case 5: tasx_note_kernel("flow_lookup_kernel<keytab>"); hipLaunchKernelGGL((flow_lookup_kernel<kCrcKeyTab, false>), g, b, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
#endif
  case 6: return launch_flow_f<1>("flow_lookup_kernel<f1>", p, s); // 1 / 4 frames per lane
  case 7: return launch_flow_f<4>("flow_lookup_kernel<f4>", p, s);
  case 8: return launch_flow_f<3>("flow_lookup_kernel<f3>", p, s);
  case 9: return launch_flow_f<kFlowFramesPerLane, false>("flow_lookup_kernel<l2key>", p, s); // the round-3 product
  case 10: return launch_flow_f<kFlowFramesPerLane, true, true>("flow_lookup_kernel<ntfs>", p, s);
  case 12: case 13: // keys by raw buffer loads: stride mode within 4 GiB, TAS layout
    if (!p->off && p->l4_off == p->ip_off + 20u && (uint64_t) p->n * p->stride < (1ull << 32)) {
      if (variant == 12)
        return launch_flow_f<kFlowFramesPerLane, false, false, 1 | 16>("flow_lookup_kernel<key sc0 sc1>", p, s);
      return launch_flow_f<kFlowFramesPerLane, false, false, 16 | 2>("flow_lookup_kernel<key sc1 nt>", p, s);
    }
    break;
  case 11: // TAS layout only (one 12-byte key load); other layouts take the product
    if (p->l4_off == p->ip_off + 20u)
      return launch_flow_partitioned(p, s);
    break;
  default: break;
  }
  return TASX_EXT_PASS;
}
