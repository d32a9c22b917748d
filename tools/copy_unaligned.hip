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
  for (int pass = 0; pass < 2; ++pass) {
    rep("unaligned src, copy", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes);
    rep("  + 32 B descriptor", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 1>), g, b, 0, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes);
    rep("  + frame header reads", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 2>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes);
    rep("  + both", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 0, false, true, 2048, 64, 3>), g, b, 0, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes);
    rep("loads only", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 1, false>), g, b, 0, s, src[r], d_un, dst[r], n, out); }, R, K, s), bytes / 2);
    rep("loads only + both", run([&](int r) { hipLaunchKernelGGL((seg_copy<6, 1, false, true, 2048, 64, 3>), g, b, 0, s, src[r], d_desc, dst[r], n, out); }, R, K, s), bytes / 2);
  }
  return 0;
}
