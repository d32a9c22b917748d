// pattern_ceiling.hip -- practical HBM read ceiling for the headline ACCESS
// PATTERN (not a product kernel): 65,536 frames at a 2048 B stride, the first
// 1,520 B of each read (the aligned chunks of a 1500 B IPv4 datagram at frame
// offset 14), summed with no checksum logic.  Compared against the same bytes
// packed contiguously and against a 2048 B full read, so the cost of the
// mbuf-stride layout and of the kernel's own logic can be separated.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/pattern_ceiling tools/pattern_ceiling.hip
//   tools/bin/pattern_ceiling [rotations] [launches]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gcu4;

__device__ __forceinline__ u32x4 ldnt(const uint8_t *base, uint32_t off)
{
  return __builtin_nontemporal_load((gcu4 *) (base + off));
}

// G lanes per frame, FPR frames per group (sequential, all loads issued first),
// NCH chunks per frame, stride S bytes, block BS threads
// EXTRA: independent VALU ops per lane after the loads land (4 sad chains)
template <int G, int FPR, int NCH, int BS, int EXTRA = 0, int SALU = 0>
__global__ __launch_bounds__(BS) void frames(const uint8_t *base, uint32_t n, uint32_t stride, uint32_t *out)
{
  extern __shared__ uint32_t lds_cap[]; // dynamic LDS only to cap blocks per CU

  constexpr int U = (NCH + G - 1) / G;
  const int gl = threadIdx.x & (G - 1);
  const uint32_t grp = blockIdx.x * (BS / G) + threadIdx.x / G;
  uint64_t acc = 0;
  u32x4 v[FPR][U];
#pragma unroll
  for (int f = 0; f < FPR; ++f) {
    const uint32_t i = min(grp * FPR + f, n - 1);
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[f][u] = ldnt(base, i * stride + 16u * min(gl + G * u, NCH - 1));
  }
#pragma unroll
  for (int f = 0; f < FPR; ++f)
#pragma unroll
    for (int u = 0; u < U; ++u)
      acc += (gl + G * u < NCH) ? (uint64_t) v[f][u].x + v[f][u].y + v[f][u].z + v[f][u].w : 0ull;
  uint32_t r = (uint32_t) acc + (uint32_t) (acc >> 32);
  if constexpr (EXTRA > 0) {
    uint32_t c0 = r, c1 = r ^ 1u, c2 = r ^ 2u, c3 = r ^ 3u;
#pragma unroll
    for (int e = 0; e < EXTRA / 4; ++e) {
      c0 = __builtin_amdgcn_sad_u16(v[0][0].x, (uint32_t) e, c0);
      c1 = __builtin_amdgcn_sad_u16(v[0][0].y, (uint32_t) e, c1);
      c2 = __builtin_amdgcn_sad_u16(v[0][0].z, (uint32_t) e, c2);
      c3 = __builtin_amdgcn_sad_u16(v[0][0].w, (uint32_t) e, c3);
    }
    r += c0 + c1 + c2 + c3;
  }
  if constexpr (SALU > 0) { // wave-uniform scalar work (a frame's final folds on the SALU)
    uint32_t q = __builtin_amdgcn_readfirstlane(r);
#pragma unroll
    for (int e = 0; e < SALU / 3; ++e) {
      q = (q & 0xffffu) + (q >> 16) + (uint32_t) e;
      asm volatile("" : "+s"(q));
    }
    r += q;
  }
  if (r == 0x12345678u)
    out[0] = r;
}

struct Res { double ev_us, wall_us; };

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
  (void) hipEventDestroy(t0); (void) hipEventDestroy(t1);
  return {w[0], w[2]};
}

static void report(const char *name, double bytes, Res r)
{
  printf("%-52s wall/K min %7.2f us median %7.2f us  %6.0f GB/s (of the bytes read)\n", name, r.ev_us, r.wall_us,
         bytes / r.wall_us / 1e3);
  fflush(stdout);
}

template <int G, int FPR, int NCH, int BS, int EXTRA = 0, int SALU = 0>
void fcase(const char *tag, std::vector<uint8_t *> &buf, uint32_t n, uint32_t stride, uint32_t *out, int R, int K,
           hipStream_t s, uint32_t lds = 0)
{
  const uint32_t groups = (n + FPR - 1) / FPR;
  const uint32_t grid = (groups + BS / G - 1) / (BS / G);
  char nm[128];
  snprintf(nm, sizeof nm, "%s G=%d FPR=%d NCH=%d BS=%d stride=%u extra=%d salu=%d lds=%u", tag, G, FPR, NCH, BS,
           stride, EXTRA, SALU, lds);
  report(nm, (double) n * NCH * 16,
         run([&](int r) { hipLaunchKernelGGL((frames<G, FPR, NCH, BS, EXTRA, SALU>), dim3(grid), dim3(BS), lds, s, buf[r], n, stride, out); },
             R, K, s));
}

int main(int argc, char **argv)
{
  int R = argc > 1 ? atoi(argv[1]) : 16;
  int K = argc > 2 ? atoi(argv[2]) : 200;
  const uint32_t n = 65536;
  const size_t B = (size_t) n * 2048;
  std::vector<uint8_t *> buf(R);
  for (int r = 0; r < R; ++r) {
    CHK(hipMalloc(&buf[r], B));
    CHK(hipMemset(buf[r], 0x5a + r, B));
  }
  uint32_t *out; CHK(hipMalloc(&out, 64));
  hipStream_t s; CHK(hipStreamCreate(&s));
  printf("65536 frames, %d rotating buffers of %zu B, %d launches x 5 reps\n", R, B, K);
  for (int rep = 0; rep < 2; ++rep) {
    fcase<16, 1, 95, 256>("mbuf", buf, n, 2048, out, R, K, s);    // the headline pattern
    fcase<16, 1, 95, 256, 96>("mbuf", buf, n, 2048, out, R, K, s, 30 * 1024);
    fcase<64, 1, 95, 256>("mbuf", buf, n, 2048, out, R, K, s);
    fcase<64, 1, 95, 256, 24, 45>("mbuf", buf, n, 2048, out, R, K, s);
    fcase<64, 1, 95, 256, 44, 45>("mbuf", buf, n, 2048, out, R, K, s);
    fcase<64, 1, 95, 256, 44, 90>("mbuf", buf, n, 2048, out, R, K, s);
    fcase<64, 1, 95, 256, 44, 45>("mbuf", buf, n, 2048, out, R, K, s, 30 * 1024);
    fcase<64, 1, 95, 256, 64, 0>("mbuf", buf, n, 2048, out, R, K, s);
  }
  return 0;
}
