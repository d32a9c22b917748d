// copy_pattern.hip -- copy ceilings for the TX segment build's memory pattern
// (diagnostic; not part of libtasx).  Each case copies N segments of LEN bytes
// from a packed source into frames at a 2048-byte stride, one 16-lane group
// per segment, 16-byte lanes, non-temporal loads and stores, and reports the
// event-timed average over rotating buffers.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/copy_pattern tools/copy_pattern.hip
//   tools/bin/copy_pattern
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu4;

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// contiguous copy, 16 B per lane per step
__global__ void copy_contig(const u32x4 *src, u32x4 *dst, uint64_t n16)
{
  for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < n16; k += (uint64_t) gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load((const gu4 *) src + k), (gu4 *) dst + k);
}

// segment copy: chunks of 16 B; source segment i at i * sstride (16-aligned),
// destination at frame i * 2048 + doff (16-aligned), nch chunks each.  U
// chunks per lane, all loads first.
template <int U>
__global__ __launch_bounds__(256) void copy_seg(const uint8_t *src, uint8_t *dst, uint32_t n, uint32_t sstride,
                                                uint32_t doff, uint32_t nch)
{
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16, gl = threadIdx.x & 15;
  if (i >= n)
    return;
  const gu4 *s = (const gu4 *) (src + (uint64_t) i * sstride);
  gu4 *d = (gu4 *) (dst + (uint64_t) i * 2048 + doff);
  for (uint32_t base = 0; base < nch; base += 16 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_nontemporal_load(s + min(base + gl + 16 * u, nch - 1));
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + gl + 16 * u < nch)
        __builtin_nontemporal_store(v[u], d + base + gl + 16 * u);
  }
}

__device__ __forceinline__ u32x4 funnel16(u32x4 a, u32x4 b, int s)
{
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const int q = s >> 2;
  const uint32_t r = (uint32_t) (s & 3);
  uint32_t o[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const uint32_t w3 = (t + 3 < 8) ? w[t + 3] : 0u;
    o[t] = q == 0 ? w[t] : q == 1 ? w[t + 1] : q == 2 ? w[t + 2] : w3;
  }
  return u32x4{__builtin_amdgcn_alignbyte(o[1], o[0], r), __builtin_amdgcn_alignbyte(o[2], o[1], r),
               __builtin_amdgcn_alignbyte(o[3], o[2], r), __builtin_amdgcn_alignbyte(o[4], o[3], r)};
}

// unaligned-source segment copy: source segment i at soff_i (any alignment),
// two aligned loads + funnel per destination chunk.  desc != 0: the source
// offset comes from a per-segment descriptor array (a dependent load).
template <int U>
__global__ __launch_bounds__(256) void copy_seg_unal(const uint8_t *src, uint8_t *dst, uint32_t n,
                                                     uint32_t sstride, uint32_t sshift, uint32_t doff,
                                                     uint32_t nch, const uint64_t *desc)
{
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16, gl = threadIdx.x & 15;
  if (i >= n)
    return;
  const uint64_t so = desc ? desc[i] : (uint64_t) i * sstride + sshift;
  const uintptr_t S0 = (uintptr_t) src + so;
  gu4 *d = (gu4 *) (dst + (uint64_t) i * 2048 + doff);
  for (uint32_t base = 0; base < nch; base += 16 * U) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uintptr_t S = S0 + 16 * min(base + gl + 16 * u, nch - 1);
      a[u] = __builtin_nontemporal_load((const gu4 *) (S & ~(uintptr_t) 15));
      b[u] = __builtin_nontemporal_load((const gu4 *) ((S + 15) & ~(uintptr_t) 15));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + gl + 16 * u < nch)
        __builtin_nontemporal_store(funnel16(a[u], b[u], (int) (S0 & 15)), d + base + gl + 16 * u);
  }
}

// same, reading only (sum into one dword per segment)
template <int U>
__global__ __launch_bounds__(256) void read_seg(const uint8_t *src, uint32_t *out, uint32_t n, uint32_t sstride,
                                                uint32_t nch)
{
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16, gl = threadIdx.x & 15;
  if (i >= n)
    return;
  const gu4 *s = (const gu4 *) (src + (uint64_t) i * sstride);
  uint32_t acc = 0;
  for (uint32_t base = 0; base < nch; base += 16 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_nontemporal_load(s + min(base + gl + 16 * u, nch - 1));
#pragma unroll
    for (int u = 0; u < U; ++u)
      acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u)
    out[i] = acc;
}

int main()
{
  const uint32_t N = 65536, R = 8, STEPS = 100;
  const size_t sbytes = (size_t) N * 2048, dbytes = (size_t) N * 2048;
  uint8_t *src[R], *dst[R];
  uint32_t *out;
  for (uint32_t r = 0; r < R; ++r) {
    CHK(hipMalloc(&src[r], sbytes));
    CHK(hipMalloc(&dst[r], dbytes));
    CHK(hipMemset(src[r], (int) r + 1, sbytes));
    CHK(hipMemset(dst[r], 0, dbytes));
  }
  CHK(hipMalloc(&out, N * 4));
  uint64_t *desc, *hd = (uint64_t *) malloc(N * 8);
  for (uint32_t i = 0; i < N; ++i)
    hd[i] = (uint64_t) i * 1456 + 3;
  CHK(hipMalloc(&desc, N * 8));
  CHK(hipMemcpy(desc, hd, N * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  struct Case {
    const char *name;
    int kind; // 0 contig, 1 seg copy, 2 seg read, 3 unaligned seg copy, 4 same via descriptors
    uint32_t sstride, doff, nch;
  } cases[] = {
      {"contig copy 95MB", 0, 0, 0, 0},
      {"seg copy 1456B src packed, dst frame+64 (last line partial)", 1, 1456, 64, 91},
      {"seg copy 1472B src packed, dst frame+64 (full lines)", 1, 1472, 64, 92},
      {"seg copy 1456B src 2048 stride, dst frame+64", 1, 2048, 64, 91},
      {"seg copy 1536B src packed, dst frame+0 (full lines)", 1, 1536, 0, 96},
      {"seg read 1456B src packed", 2, 1456, 0, 91},
      {"seg copy unaligned src (+3, 2 loads+funnel), dst frame+64", 3, 1456, 64, 91},
      {"seg copy unaligned src via descriptor array, dst frame+64", 4, 1456, 64, 91},
      {"seg copy aligned src via 2-load path (+0), dst frame+64", 5, 1456, 64, 91},
      {"seg read 1456B src 2048 stride", 2, 2048, 0, 91},
  };
  for (const Case &c : cases) {
    auto launch = [&](uint32_t k) {
      const uint32_t r = k % R;
      if (c.kind == 0)
        hipLaunchKernelGGL(copy_contig, dim3(4096), dim3(256), 0, 0, (const u32x4 *) src[r], (u32x4 *) dst[r],
                           (uint64_t) N * 1448 / 16);
      else if (c.kind == 1)
        hipLaunchKernelGGL(copy_seg<6>, dim3(N / 16), dim3(256), 0, 0, src[r], dst[r], N, c.sstride, c.doff,
                           c.nch);
      else if (c.kind >= 3)
        hipLaunchKernelGGL(copy_seg_unal<6>, dim3(N / 16), dim3(256), 0, 0, src[r], dst[r], N, c.sstride,
                           c.kind == 5 ? 0u : 3u, c.doff, c.nch, c.kind == 4 ? (const uint64_t *) desc : nullptr);
      else
        hipLaunchKernelGGL(read_seg<6>, dim3(N / 16), dim3(256), 0, 0, src[r], out, N, c.sstride, c.nch);
    };
    for (uint32_t k = 0; k < 3 * R; ++k)
      launch(k);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    for (uint32_t k = 0; k < STEPS; ++k)
      launch(k);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / STEPS;
    const double bytes = c.kind == 0 ? 2.0 * N * 1448 : (c.kind == 2 ? 1.0 : 2.0) * N * 16.0 * c.nch;
    printf("%-62s %8.2f us  %7.1f GB/s\n", c.name, us, bytes / us / 1e3);
  }
  return 0;
}
