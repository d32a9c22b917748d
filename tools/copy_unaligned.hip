// copy_unaligned.hip -- probe for the fused TX segment build (not a product
// kernel): can one UNALIGNED 16-byte global load per destination chunk replace
// the aligned two-chunk gather + funnel shift?  65,536 segments of 1,456 B
// (91 chunks, the TAS data segment's payload chunks) copied from random byte
// offsets in 8,192 16 KiB flow buffers into frames at a 2048 B stride
// (destination chunk-aligned, as the kernel stores whole frame chunks), summed
// on the way.  Variants: source offsets forced to 16-byte alignment
// (ceiling), unaligned single loads, and reads only / writes only.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/copy_unaligned tools/copy_unaligned.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4u gcu4u;
typedef __attribute__((address_space(1))) const u32x4 gcu4;
typedef __attribute__((address_space(1))) u32x4 gu4;

constexpr int NCH = 91;

// MODE: 0 = copy, 1 = loads only (sum), 2 = stores only (constant data)
// NT: non-temporal loads; NTS: non-temporal stores; DS: destination stride
// X: bit 0 = the offset comes from a 32-byte descriptor read by all 16 lanes
// (as the TX segment kernel's), bit 1 = also read the frame's header chunk and
// two header half-words from the destination frame
template <int U, int MODE, bool NT, bool NTS = true, uint32_t DS = 2048, uint32_t DO = 64, int X = 0>
__global__ __launch_bounds__(256) void seg_copy(const uint8_t *src, const uint32_t *soff, uint8_t *dst, uint32_t n,
                                                uint32_t *out)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16;
  if (i >= n)
    return;
  uint32_t so;
  if (X & 1) {
    const u32x4 d0 = *(gcu4 *) (soff + 8 * i), d1 = *(gcu4 *) (soff + 8 * i + 4);
    so = d0.x + d1.w;
  } else {
    so = soff[i];
  }
  const uint32_t dbase = i * DS + DO;
  uint32_t acc = 0;
  if (X & 2) {
    const u32x4 h = *(gcu4 *) (dst + i * DS + 16u * min(gl, 4));
    const uint32_t t = *(__attribute__((address_space(1))) const uint16_t *) (dst + i * DS + 16);
    const uint32_t t2 = *(__attribute__((address_space(1))) const uint16_t *) (dst + i * DS + 14 + 2 * min(gl, 9));
    acc = h.x + h.w + t + t2;
  }
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = min((uint32_t) (gl + 16 * u), (uint32_t) NCH - 1);
    if (MODE != 2)
      v[u] = NT ? __builtin_nontemporal_load((gcu4u *) (src + so + 16u * c)) : *(gcu4u *) (src + so + 16u * c);
    else
      v[u] = u32x4{so, c, 1u, 2u};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = gl + 16 * u;
    if (c < NCH) {
      if (MODE != 1) {
        if (NTS)
          __builtin_nontemporal_store(v[u], (gu4 *) (dst + dbase + 16u * c));
        else
          *(gu4 *) (dst + dbase + 16u * c) = v[u];
      }
      acc = __builtin_amdgcn_sad_u16(v[u].x, 0, __builtin_amdgcn_sad_u16(v[u].y, 0, __builtin_amdgcn_sad_u16(v[u].z, 0, __builtin_amdgcn_sad_u16(v[u].w, 0, acc))));
    }
  }
  if (acc == 0x12345678u)
    out[0] = acc;
}

// One segment per WAVE, aligned loads only: the segment's start shift sh is
// wave-uniform, lane L loads aligned chunks L and L + 64 of the source span,
// gets aligned chunk L + 1 from lane L + 1 by DPP wave_rol:1 (lane 63: lane
// 0's second chunk by readlane) and funnel-shifts the pair by sh (a uniform
// dword select + v_alignbyte).  NCH + 1 aligned chunks cover the 16 * NCH
// bytes at any shift.
__device__ __forceinline__ uint32_t wave_rol1(uint32_t x)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x134, 0xf, 0xf, false); // wave_rol:1
}
__device__ __forceinline__ u32x4 funnel_u(const u32x4 a, const u32x4 b, uint32_t q, uint32_t r8)
{
  // bytes [4q + r8, 4q + r8 + 16) of a:b, q and r8 wave-uniform
  uint32_t w0, w1, w2, w3, w4;
  switch (q) {
  case 0: w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; break;
  case 1: w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; break;
  case 2: w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; break;
  default: w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; break;
  }
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, r8), __builtin_amdgcn_alignbyte(w2, w1, r8),
               __builtin_amdgcn_alignbyte(w3, w2, r8), __builtin_amdgcn_alignbyte(w4, w3, r8)};
}
__global__ __launch_bounds__(256) void seg_copy_wave(const uint8_t *src, const uint32_t *soff, uint8_t *dst, uint32_t n,
                                                     uint32_t *out)
{
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * 4u + threadIdx.x / 64u;
  if (i >= n)
    return;
  const uint32_t so = __builtin_amdgcn_readfirstlane(soff[i]);
  const uint32_t A = so & ~15u, q = (so >> 2) & 3u, r8 = so & 3u;
  const uint8_t *sa = src + A;
  const u32x4 v0 = __builtin_nontemporal_load((gcu4 *) (sa + 16u * lane));
  const u32x4 v1 = __builtin_nontemporal_load((gcu4 *) (sa + 16u * min(lane + 64u, (uint32_t) NCH)));
  u32x4 n0, n1;
  n0.x = wave_rol1(v0.x); n0.y = wave_rol1(v0.y); n0.z = wave_rol1(v0.z); n0.w = wave_rol1(v0.w);
  n1.x = wave_rol1(v1.x); n1.y = wave_rol1(v1.y); n1.z = wave_rol1(v1.z); n1.w = wave_rol1(v1.w);
  const u32x4 l0 = {(uint32_t) __builtin_amdgcn_readlane((int) v1.x, 0), (uint32_t) __builtin_amdgcn_readlane((int) v1.y, 0),
                    (uint32_t) __builtin_amdgcn_readlane((int) v1.z, 0), (uint32_t) __builtin_amdgcn_readlane((int) v1.w, 0)};
  if (lane == 63u)
    n0 = l0;
  const u32x4 o0 = funnel_u(v0, n0, q, r8), o1 = funnel_u(v1, n1, q, r8);
  uint8_t *d = dst + i * 2048u + 64u;
  __builtin_nontemporal_store(o0, (gu4 *) (d + 16u * lane));
  if (lane + 64u < (uint32_t) NCH)
    __builtin_nontemporal_store(o1, (gu4 *) (d + 16u * (lane + 64u)));
  uint32_t acc = __builtin_amdgcn_sad_u16(o0.x, 0, __builtin_amdgcn_sad_u16(o0.y, 0, o0.z + o0.w));
  if (acc == 0x12345678u)
    out[0] = acc;
}

// 16-lane rows (one segment per row, four per wave) reading ALIGNED chunks:
// lane gl holds aligned chunks gl + 16u, gets chunk + 1 from lane gl + 1 by
// DPP row_ror:15 (lane 15: lane 0's next round), and funnel-shifts by the
// row's own shift (per-lane dword select + v_alignbyte)
__device__ __forceinline__ uint32_t ror15(uint32_t x)
{
  return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x12F, 0xf, 0xf, false); // row_ror:15
}
__device__ __forceinline__ u32x4 funnel_lane(const u32x4 a, const u32x4 b, uint32_t sh)
{
  const uint32_t q = sh >> 2, r8 = sh & 3u;
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t o[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const uint32_t lo = (q & 1u) ? w[j + 1] : w[j], hi = (q & 1u) ? w[j + 3] : w[j + 2];
    o[j] = (q & 2u) ? hi : lo;
  }
  return u32x4{__builtin_amdgcn_alignbyte(o[1], o[0], r8), __builtin_amdgcn_alignbyte(o[2], o[1], r8),
               __builtin_amdgcn_alignbyte(o[3], o[2], r8), __builtin_amdgcn_alignbyte(o[4], o[3], r8)};
}
template <int U>
__global__ __launch_bounds__(256) void seg_copy_row_aligned(const uint8_t *src, const uint32_t *soff, uint8_t *dst,
                                                            uint32_t n, uint32_t *out)
{
  const uint32_t gl = threadIdx.x & 15u;
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16;
  if (i >= n)
    return;
  const uint32_t so = soff[i], A = so & ~15u, sh = so & 15u;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = __builtin_nontemporal_load((gcu4 *) (src + A + 16u * min(gl + 16u * u, (uint32_t) NCH)));
  uint32_t acc = 0;
  const uint32_t dbase = i * 2048u + 64u;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    u32x4 nx = {ror15(v[u].x), ror15(v[u].y), ror15(v[u].z), ror15(v[u].w)};
    if (u + 1 < U) {
      const u32x4 nn = {ror15(v[u + 1].x), ror15(v[u + 1].y), ror15(v[u + 1].z), ror15(v[u + 1].w)};
      if (gl == 15u)
        nx = nn;
    }
    const u32x4 o = funnel_lane(v[u], nx, sh);
    const uint32_t c = gl + 16u * u;
    if (c < (uint32_t) NCH) {
      __builtin_nontemporal_store(o, (gu4 *) (dst + dbase + 16u * c));
      acc = __builtin_amdgcn_sad_u16(o.x, 0, __builtin_amdgcn_sad_u16(o.y, 0, __builtin_amdgcn_sad_u16(o.z, 0, __builtin_amdgcn_sad_u16(o.w, 0, acc))));
    }
  }
  if (acc == 0x12345678u)
    out[0] = acc;
}

struct Res { double min_us, med_us; };

template <typename F>
Res run(F launch, int R, int K, hipStream_t s)
{
  hipEvent_t t0, t1; CHK(hipEventCreate(&t0)); CHK(hipEventCreate(&t1));
  for (int k = 0; k < 4 * R; ++k) launch(k % R);
  CHK(hipStreamSynchronize(s));
  std::vector<float> w;
  for (int rep = 0; rep < 5; ++rep) {
    CHK(hipEventRecord(t0, s));
    for (int k = 0; k < K; ++k) launch(k % R);
    CHK(hipEventRecord(t1, s));
    CHK(hipEventSynchronize(t1));
    float tot; CHK(hipEventElapsedTime(&tot, t0, t1));
    w.push_back(tot * 1e3f / K);
  }
  std::sort(w.begin(), w.end());
  return {w[0], w[2]};
}

int main(int argc, char **argv)
{
  const int R = argc > 1 ? atoi(argv[1]) : 8;
  const int K = argc > 2 ? atoi(argv[2]) : 100;
  const uint32_t n = 65536, flows = 8192;
  const size_t shm = (size_t) flows * 16384 + 64, fr = (size_t) n * 2048;
  std::vector<uint8_t *> src(R), dst(R);
  for (int r = 0; r < R; ++r) {
    CHK(hipMalloc(&src[r], shm));
    CHK(hipMalloc(&dst[r], fr));
    CHK(hipMemset(src[r], 0x11 + r, shm));
    CHK(hipMemset(dst[r], 0, fr));
  }
  // segment i: flow (i * 2654435761) % flows, random start inside its buffer
  std::vector<uint32_t> h_un(n), h_al(n);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < n; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    const uint32_t f = (uint32_t) ((i * 2654435761ull) % flows);
    const uint32_t pos = (uint32_t) (x % (16384 - 1456 - 16));
    h_un[i] = f * 16384u + pos;
    h_al[i] = f * 16384u + (pos & ~15u);
  }
  std::vector<uint32_t> h_desc(8 * (size_t) n, 0u);
  for (uint32_t i = 0; i < n; ++i)
    h_desc[8 * i] = h_un[i];
  uint32_t *d_desc;
  CHK(hipMalloc(&d_desc, 32 * (size_t) n));
  CHK(hipMemcpy(d_desc, h_desc.data(), 32 * (size_t) n, hipMemcpyHostToDevice));
  uint32_t *d_un, *d_al, *out;
  CHK(hipMalloc(&d_un, n * 4)); CHK(hipMalloc(&d_al, n * 4)); CHK(hipMalloc(&out, 64));
  CHK(hipMemcpy(d_un, h_un.data(), n * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_al, h_al.data(), n * 4, hipMemcpyHostToDevice));
  hipStream_t s; CHK(hipStreamCreate(&s));
  const double bytes = (double) n * NCH * 16 * 2;
  printf("65536 segments x 91 chunks (1456 B) read + written = %.1f MB per launch, %d rotations\n", bytes / 1e6, R);
  auto rep = [&](const char *nm, Res r, double b) {
    printf("%-44s min %7.2f us median %7.2f us  %6.0f GB/s\n", nm, r.min_us, r.med_us, b / r.med_us / 1e3);
    fflush(stdout);
  };
  const dim3 g(n / 16), b(256);
  hipFuncAttributes fa;
  CHK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(seg_copy<6, 0, false, true, 2048, 64, 3>)));
  printf("seg_copy<+both>: %d VGPRs\n", fa.numRegs);
  { // the wave form copies the same bytes as seg_copy<6, 0, false> (checked once)
    std::vector<uint8_t> h(n * 2048), h2(n * 2048);
    for (uint32_t k = 0; k < 64; ++k) // a source with a byte pattern
      ;
    std::vector<uint8_t> pat(shm);
    for (size_t k = 0; k < shm; ++k) pat[k] = (uint8_t) (k * 131u + (k >> 9));
    CHK(hipMemcpy(src[0], pat.data(), shm, hipMemcpyHostToDevice));
    CHK(hipMemset(dst[0], 0, fr)); CHK(hipMemset(dst[1 % R], 0, fr));
    hipLaunchKernelGGL((seg_copy<6, 0, false>), g, b, 0, s, src[0], d_un, dst[0], n, out);
    hipLaunchKernelGGL(seg_copy_wave, dim3(n / 4), b, 0, s, src[0], d_un, dst[1 % R], n, out);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpy(h.data(), dst[0], fr, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(h2.data(), dst[1 % R], fr, hipMemcpyDeviceToHost));
    printf("wave form copies the same bytes: %s\n", h == h2 ? "yes" : "NO");
    CHK(hipMemset(dst[1 % R], 0, fr));
    hipLaunchKernelGGL((seg_copy_row_aligned<6>), g, b, 0, s, src[0], d_un, dst[1 % R], n, out);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpy(h2.data(), dst[1 % R], fr, hipMemcpyDeviceToHost));
    printf("aligned row form copies the same bytes: %s\n", h == h2 ? "yes" : "NO");
  }
  for (int pass = 0; pass < 2; ++pass) {
    rep("one segment per wave, aligned loads + DPP funnel", run([&](int r) { hipLaunchKernelGGL(seg_copy_wave, dim3(n / 4), b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes);
    rep("16-lane rows, aligned loads + DPP funnel", run([&](int r) { hipLaunchKernelGGL((seg_copy_row_aligned<6>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes);
    rep("unaligned src, copy", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes);
    rep("  + 32 B descriptor", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 1>), g, b, 0, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes);
    rep("  + frame header reads", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 2>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes);
    rep("  + both", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 3>), g, b, 0, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes);
    // residency: the same "+ both" copy with blocks per CU capped by reserved
    // LDS (160 KiB per CU): 5 / 4 / 3 blocks = 5 / 4 / 3 waves per SIMD, the
    // TX segment kernel holding 105 VGPRs runs at 4
    for (uint32_t lds_kib : {32u, 36u, 48u}) {
      char nm[64];
      snprintf(nm, sizeof nm, "  + both, %u KiB LDS reserved (%u blocks/CU)", lds_kib, 160u / lds_kib);
      rep(nm, run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 3>), g, b, lds_kib * 1024u, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes);
    }
    rep("loads only", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 1, false>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes / 2);
    rep("loads only + both", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 1, false, true, 2048, 64, 3>), g, b, 0, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes / 2);
  }
  return 0;
}
