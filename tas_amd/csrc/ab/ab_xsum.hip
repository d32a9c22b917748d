// ab/ab_xsum.hip -- comparison build only (libtasx_ab.so): the access-pattern
// kernels bench.py prices the checksum kernels against (tasx_ab_tcp4_pattern,
// tasx_ab_tcp4_mix_pattern; include/tasx_ab.h).  The checksum kernels' retired
// variants (the first-generation group-per-packet kernels, wave-timeline
// stamps, 32- and 64-lane groups, tcp4_wave_kernel, tcp4_mix_kernel, forced
// row modes, block sizes, persistent rows, the RX pass's other grids and its
// timing ablations) were measured in rounds 1-5 (profiles/r01_*,
// profiles/r02-r05/INDEX.md) and are gone from the source (round 6).
#include <errno.h>
#include <string.h>

#include "../xsum_rows.h"

// The headline kernel's access pattern with no checksum logic: the same rows,
// the same 6 clamped chunk loads per lane at 32-bit offsets from the SGPR
// base, the same 4-byte result store per frame and LDS reservation; the
// loaded words are only xor-folded.  bench.py times it beside the headline
// (its pattern_ceiling).
namespace {
__global__ __launch_bounds__(kBlock) void tcp4_pattern_kernel(tasx_tcp4_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return;
  const uint32_t a0 = i * (uint32_t) p.stride + (p.ip_off & ~15u), hend = p.flen0 - p.ip_off;
  const uint32_t lastoff = a0 + 16u * ((14u + hend - 1u) >> 4), lo = a0 + 16u * (uint32_t) gl;
  u32x4 v[6];
#pragma unroll
  for (int u = 0; u < 6; ++u)
    v[u] = ld16nt_off(p.base, min(lo + 256u * u, lastoff));
  uint32_t x = 0;
#pragma unroll
  for (int u = 0; u < 6; ++u)
    x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  x = row_sum16(x);
  if (gl == 15)
    stg((uint32_t *) p.out, i, x);
}

// The data/ACK mix's access pattern (tcp4_tas14_kernel<hints>, the flush_mix
// leg) with no checksum logic, for its latency roofline (bench.py
// mix_bounds): each row reads its hint, then (CHAIN = 0) the same clamped
// chunk loads as the product, xor-folded, or (CHAIN = 1) only the chunk
// holding the frame's end on lane 15 -- the row's dependent chain (hint ->
// frame -> result store) with almost no bytes behind it; 8 waves per SIMD as
// the product.
template <int CHAIN>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void tcp4_mix_pattern_kernel(tasx_tcp4_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if constexpr (CHAIN == 2) {
    // two frames per row, i and i + n / 2 (rounded up): both hints, then both
    // frames' chunk loads, one generation of resident rows for 64K frames
    const uint32_t half = (p.n + 1u) / 2u;
    if (i >= half)
      return;
    const uint32_t i2 = min(i + half, p.n - 1u);
    const uint32_t h1 = ldg(p.flen, i), h2 = ldg(p.flen, i2);
    uint32_t x1 = 0, x2 = 0;
    u32x4 v1[6], v2[6];
    {
      const uint32_t a1 = i * (uint32_t) p.stride + (p.ip_off & ~15u), a2 = i2 * (uint32_t) p.stride + (p.ip_off & ~15u);
      const uint32_t hl1 = h1 > p.ip_off + 20u ? min(h1 - p.ip_off, 1522u) : 20u;
      const uint32_t hl2 = h2 > p.ip_off + 20u ? min(h2 - p.ip_off, 1522u) : 20u;
      const uint32_t l1 = a1 + 16u * ((14u + hl1 - 1u) >> 4), l2 = a2 + 16u * ((14u + hl2 - 1u) >> 4);
#pragma unroll
      for (int u = 0; u < 6; ++u)
        v1[u] = ld16nt_off(p.base, min(a1 + 16u * (uint32_t) gl + 256u * u, l1));
#pragma unroll
      for (int u = 0; u < 6; ++u)
        v2[u] = ld16nt_off(p.base, min(a2 + 16u * (uint32_t) gl + 256u * u, l2));
    }
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      x1 ^= v1[u].x ^ v1[u].y ^ v1[u].z ^ v1[u].w;
      x2 ^= v2[u].x ^ v2[u].y ^ v2[u].z ^ v2[u].w;
    }
    x1 = row_sum16(x1);
    x2 = row_sum16(x2);
    if (gl == 15) {
      stg((uint32_t *) p.out, i, x1);
      if (i + half < p.n)
        stg((uint32_t *) p.out, i2, x2);
    }
    return;
  }
  if (i >= p.n)
    return;
  const uint32_t a0 = i * (uint32_t) p.stride + (p.ip_off & ~15u);
  const uint32_t h = ldg(p.flen, i);
  const uint32_t hl = h > p.ip_off + 20u ? min(h - p.ip_off, 1522u) : 20u;
  const uint32_t lastoff = a0 + 16u * ((14u + hl - 1u) >> 4), lo = a0 + 16u * (uint32_t) gl;
  uint32_t x = 0;
  if constexpr (CHAIN) {
    if (gl == 15) {
      const u32x4 t = ld16nt_off(p.base, lastoff);
      x = t.x ^ t.y ^ t.z ^ t.w;
    }
  } else {
    u32x4 v[6];
#pragma unroll
    for (int u = 0; u < 6; ++u)
      v[u] = ld16nt_off(p.base, min(lo + 256u * u, lastoff));
#pragma unroll
    for (int u = 0; u < 6; ++u)
      x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  x = row_sum16(x);
  if (gl == 15)
    stg((uint32_t *) p.out, i, x);
}
} // namespace

extern "C" int tasx_ab_tcp4_mix_pattern(const void *base, uint64_t stride, uint32_t n, const uint32_t *flen,
                                        uint32_t ip_off, int chain, uint32_t *out, void *stream)
{
  tasx_tcp4_params p;
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.stride = stride;
  p.n = n;
  p.flen = flen;
  p.ip_off = ip_off;
  p.l4_off = ip_off + 20u;
  p.out = (uint16_t *) out;
  // the product's own geometry checks: 16-byte aligned rooms of at least 1536 bytes, 32-bit offsets
  if (!out || !flen || !base || (ip_off & 15u) != 14u || (stride & 15u) || stride < 1536u ||
      (uint64_t) n * stride > 0xffffffffull || ((uintptr_t) base & 15u))
    return -EINVAL;
  if (chain == 2) { // two frames per row: half the rows
    tasx_tcp4_params q = p;
    q.n = (n + 1u) / 2u;
    const uint64_t blocks = ((uint64_t) q.n + kBlock / 16 - 1) / (kBlock / 16);
    if (blocks == 0)
      return 0;
    tasx_note_kernel("tcp4_mix_pattern_kernel<pair>");
    hipLaunchKernelGGL(tcp4_mix_pattern_kernel<2>, dim3((uint32_t) blocks), dim3(kBlock), 0, (hipStream_t) stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  return chain ? launch_groups("tcp4_mix_pattern_kernel<chain>", tcp4_mix_pattern_kernel<1>, p, (hipStream_t) stream, 0u)
               : launch_groups("tcp4_mix_pattern_kernel", tcp4_mix_pattern_kernel<0>, p, (hipStream_t) stream, 0u);
}

extern "C" int tasx_ab_tcp4_pattern(const void *base, uint64_t stride, uint32_t n, uint32_t flen0, uint32_t ip_off,
                                    uint32_t *out, void *stream)
{
  tasx_tcp4_params p;
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.stride = stride;
  p.n = n;
  p.flen0 = flen0;
  p.ip_off = ip_off;
  p.l4_off = ip_off + 20u;
  p.out = (uint16_t *) out;
  if (!out || !tas14_ok(p))
    return -EINVAL;
  return launch_groups("tcp4_pattern_kernel", tcp4_pattern_kernel, p, (hipStream_t) stream, kOccLds);
}
