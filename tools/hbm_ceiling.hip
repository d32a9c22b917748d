// hbm_ceiling.hip -- practical HBM read ceiling on this MI355X for the batch
// sizes the checksum path sees (a known-good reference measured on the same
// hardware, cdna_hip_programming.md section 5.4 rule 10).  Not part of the product.
//
// Pure streaming read + integer fold (the same VALU work per byte as the
// checksum, no packet structure), over R rotating buffers of B bytes each so
// every launch reads HBM.  Reports per-launch time (hipEvents around each
// launch, and total / K) for several launch shapes.
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_ceiling tools/hbm_ceiling.hip
//   ./hbm_ceiling [bytes_per_launch] [rotations] [launches]
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

// grid-stride: each thread U chunks in flight per iteration
template <int U>
__global__ __launch_bounds__(256) void stream_gs(const u32x4 *p, uint64_t nchunks, uint32_t *out)
{
  const gcu4 *g = (const gcu4 *) p;
  uint64_t acc = 0;
  const uint64_t T = (uint64_t) gridDim.x * blockDim.x;
  uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * T < nchunks; i += U * T) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = g[i + u * T];
#pragma unroll
    for (int u = 0; u < U; ++u) { acc += v[u].x; acc += v[u].y; acc += v[u].z; acc += v[u].w; }
  }
  for (; i < nchunks; i += T) { u32x4 v = g[i]; acc += v.x; acc += v.y; acc += v.z; acc += v.w; }
  uint32_t r = (uint32_t) acc + (uint32_t) (acc >> 32);
  if (r == 0x12345678u) out[0] = r;  // keep live, never true for random data
}

// one-shot: block b reads a contiguous span of 256*U chunks, wave-contiguous 1 KiB per load
template <int U>
__global__ __launch_bounds__(256) void stream_blk(const u32x4 *p, uint64_t nchunks, uint32_t *out)
{
  const gcu4 *g = (const gcu4 *) p;
  uint64_t base = (uint64_t) blockIdx.x * 256 * U;
  uint64_t acc = 0;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    uint64_t i = base + (uint64_t) u * 256 + threadIdx.x;
    v[u] = i < nchunks ? g[i] : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) { acc += v[u].x; acc += v[u].y; acc += v[u].z; acc += v[u].w; }
  uint32_t r = (uint32_t) acc + (uint32_t) (acc >> 32);
  if (r == 0x12345678u) out[0] = r;
}

struct Res { double ev_us, wall_us; };

template <typename F>
Res run(F launch, int R, int K, hipStream_t s)
{
  std::vector<hipEvent_t> a(K), b(K);
  for (int k = 0; k < K; ++k) { CHK(hipEventCreate(&a[k])); CHK(hipEventCreate(&b[k])); }
  hipEvent_t t0, t1; CHK(hipEventCreate(&t0)); CHK(hipEventCreate(&t1));
  for (int k = 0; k < 2 * R; ++k) launch(k % R);
  CHK(hipStreamSynchronize(s));
  // pass 1: wall time over K launches, no per-launch events
  CHK(hipEventRecord(t0, s));
  for (int k = 0; k < K; ++k) launch(k % R);
  CHK(hipEventRecord(t1, s));
  CHK(hipEventSynchronize(t1));
  float tot; CHK(hipEventElapsedTime(&tot, t0, t1));
  // pass 2: per-launch events
  for (int k = 0; k < K; ++k) { CHK(hipEventRecord(a[k], s)); launch(k % R); CHK(hipEventRecord(b[k], s)); }
  CHK(hipStreamSynchronize(s));
  std::vector<float> d(K);
  for (int k = 0; k < K; ++k) CHK(hipEventElapsedTime(&d[k], a[k], b[k]));
  std::sort(d.begin(), d.end());
  for (int k = 0; k < K; ++k) { hipEventDestroy(a[k]); hipEventDestroy(b[k]); }
  return {d[K / 2] * 1e3, tot * 1e3 / K};
}

int main(int argc, char **argv)
{
  uint64_t B = argc > 1 ? strtoull(argv[1], 0, 0) : 98304000ull;
  int R = argc > 2 ? atoi(argv[2]) : 16;
  int K = argc > 3 ? atoi(argv[3]) : 200;
  B &= ~15ull;
  uint64_t nch = B / 16;
  std::vector<u32x4 *> buf(R);
  for (int r = 0; r < R; ++r) {
    CHK(hipMalloc(&buf[r], B));
    CHK(hipMemset(buf[r], 0x5a + r, B));
  }
  uint32_t *out; CHK(hipMalloc(&out, 64));
  hipStream_t s; CHK(hipStreamCreate(&s));
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d, %llu B per launch, %d rotating buffers, %d launches\n",
         prop.name, prop.multiProcessorCount, (unsigned long long) B, R, K);
  auto report = [&](const char *name, Res r) {
    printf("%-34s event-median %8.2f us  %7.0f GB/s | wall/K %8.2f us  %7.0f GB/s\n", name,
           r.ev_us, B / r.ev_us / 1e3, r.wall_us, B / r.wall_us / 1e3);
  };
  for (int blocksPerCU : {2, 4, 8, 16}) {
    int grid = prop.multiProcessorCount * blocksPerCU;
    char nm[64];
    snprintf(nm, sizeof nm, "grid-stride U=4 %d blk/CU", blocksPerCU);
    report(nm, run([&](int r) { hipLaunchKernelGGL(stream_gs<4>, dim3(grid), dim3(256), 0, s, buf[r], nch, out); }, R, K, s));
    snprintf(nm, sizeof nm, "grid-stride U=8 %d blk/CU", blocksPerCU);
    report(nm, run([&](int r) { hipLaunchKernelGGL(stream_gs<8>, dim3(grid), dim3(256), 0, s, buf[r], nch, out); }, R, K, s));
  }
  {
    int grid = (int) ((nch + 256 * 4 - 1) / (256 * 4));
    report("one-shot U=4", run([&](int r) { hipLaunchKernelGGL(stream_blk<4>, dim3(grid), dim3(256), 0, s, buf[r], nch, out); }, R, K, s));
    grid = (int) ((nch + 256 * 8 - 1) / (256 * 8));
    report("one-shot U=8", run([&](int r) { hipLaunchKernelGGL(stream_blk<8>, dim3(grid), dim3(256), 0, s, buf[r], nch, out); }, R, K, s));
    grid = (int) ((nch + 256 * 16 - 1) / (256 * 16));
    report("one-shot U=16", run([&](int r) { hipLaunchKernelGGL(stream_blk<16>, dim3(grid), dim3(256), 0, s, buf[r], nch, out); }, R, K, s));
  }
  return 0;
}
