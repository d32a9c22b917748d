// ab/ab_flow.hip -- comparison build only (libtasx_ab.so): the RX flow lookup's
// bare access pattern, which bench.py prices the lookup against.  The lookup's
// retired variants (CRC forms, frames per lane, key cache policies, the
// hash-range-partitioned lookup: profiles/r01_flow_variants.jsonl,
// profiles/r04/INDEX.md r04i) are gone from the source (round 6).
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

} // namespace

// the flow lookup's bare access pattern (include/tasx_ab.h)
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
