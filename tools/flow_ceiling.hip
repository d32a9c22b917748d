// flow_ceiling.hip -- access-pattern ceiling of the RX flow lookup (not a
// product kernel): the dependent chain of fast_flows_packet_fss()
// (/root/reference/tas/fast/fast_flows.c:1084-1163) with no hashing or key
// logic, so the cost of the memory pattern itself can be separated from the
// kernel's work.  One lane per frame, 262,144 frames at a 2048 B stride (4
// rotating 512 MB batches, as bench.py's flow_lookup leg):
//   hdr      the 12-byte key at frame + 26 (one 64 B line per frame, from HBM)
//   hdr+b1   + one dependent 8-byte load from a 2 MB table (the flowht bucket)
//   hdr+b4   + four (the 4-entry bucket, consecutive entries)
//   chain    + four bucket entries + one dependent 12-byte load from a 16 MB
//            table (the candidate flow's key in flowst)
//   chain4   + four bucket entries + four 12-byte key loads (as the product
//            kernel issues them: non-candidates read entry 0)
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/flow_ceiling tools/flow_ceiling.hip
//   tools/bin/flow_ceiling [launches]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x3u __attribute__((ext_vector_type(3), aligned(1)));
#define G1(T, p) (*(__attribute__((address_space(1))) const T *) (p))

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void flow_pattern(const uint8_t *frames, uint32_t n, const uint64_t *ht,
                                                    uint32_t ht_n, const uint8_t *fs, uint32_t fs_n,
                                                    uint32_t *out)
{
  const uint32_t i0 = blockIdx.x * 256u + threadIdx.x;
  const uint32_t i = min(i0, n - 1u);
  const u32x3u k = G1(u32x3u, frames + (uint64_t) i * 2048u + 26u);
  uint32_t h = mix(k.x ^ k.y ^ k.z);
  uint32_t r = h;
  if constexpr (MODE >= 1) {
    uint64_t e[4];
    constexpr int NB = MODE >= 2 ? 4 : 1;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      e[j] = G1(uint64_t, ht + (h + j) % ht_n);
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      acc += (uint32_t) e[j] ^ (uint32_t) (e[j] >> 32);
    r = acc;
    if constexpr (MODE >= 3) {
      constexpr int NK = MODE >= 4 ? 4 : 1;
      uint32_t kk = 0;
#pragma unroll
      for (int j = 0; j < NK; ++j) {
        // the first entry's flow is the candidate (a random flow per frame,
        // dependent on the bucket load); the others read flow 0
        const uint32_t fid = j == 0 ? mix(h ^ (uint32_t) e[0]) % fs_n : 0u;
        const u32x3 key = G1(u32x3, fs + (uint64_t) fid * 128u + 32u);
        kk += key.x ^ key.y ^ key.z;
      }
      r ^= kk;
    }
  }
  if (i0 < n)
    out[i0] = r;
}

__global__ void init_keys(uint8_t *fr, uint32_t n, uint32_t r)
{
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n)
    *(uint32_t *) (fr + (size_t) i * 2048 + 28) = i * 2654435761u + r;
}

template <int MODE>
static float run(uint8_t **fr, int R, uint32_t n, const uint64_t *ht, uint32_t ht_n, const uint8_t *fs,
                 uint32_t fs_n, uint32_t *out, int launches)
{
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const dim3 g((n + 255) / 256), bl(256);
  for (int k = 0; k < 20; ++k)
    hipLaunchKernelGGL(flow_pattern<MODE>, g, bl, 0, 0, fr[k % R], n, ht, ht_n, fs, fs_n, out);
  CHK(hipEventRecord(a, 0));
  for (int k = 0; k < launches; ++k)
    hipLaunchKernelGGL(flow_pattern<MODE>, g, bl, 0, 0, fr[k % R], n, ht, ht_n, fs, fs_n, out);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipGetLastError());
  return ms * 1e3f / launches;
}

int main(int argc, char **argv)
{
  const int launches = argc > 1 ? atoi(argv[1]) : 200;
  const uint32_t n = 262144, ht_n = 262144, fs_n = 131072;
  const int R = 4;
  uint8_t *fr[R];
  for (int r = 0; r < R; ++r) {
    CHK(hipMalloc(&fr[r], (size_t) n * 2048));
    CHK(hipMemset(fr[r], 0x11 * (r + 1), (size_t) n * 2048));
  }
  uint64_t *ht;
  uint8_t *fs;
  uint32_t *out;
  CHK(hipMalloc(&ht, (size_t) ht_n * 8));
  CHK(hipMemset(ht, 0x5a, (size_t) ht_n * 8));
  CHK(hipMalloc(&fs, (size_t) fs_n * 128));
  CHK(hipMemset(fs, 0x3c, (size_t) fs_n * 128));
  CHK(hipMalloc(&out, (size_t) n * 4));
  // vary the keys so the hashed indices spread (one word per frame)
  for (int r = 0; r < R; ++r)
    hipLaunchKernelGGL(init_keys, dim3((n + 255) / 256), dim3(256), 0, 0, fr[r], n, (uint32_t) r);
  CHK(hipDeviceSynchronize());
  const char *names[] = {"hdr", "hdr+b1", "hdr+b4", "chain", "chain4"};
  float t[5];
  for (int rep = 0; rep < 3; ++rep) {
    t[0] = run<0>(fr, R, n, ht, ht_n, fs, fs_n, out, launches);
    t[1] = run<1>(fr, R, n, ht, ht_n, fs, fs_n, out, launches);
    t[2] = run<2>(fr, R, n, ht, ht_n, fs, fs_n, out, launches);
    t[3] = run<3>(fr, R, n, ht, ht_n, fs, fs_n, out, launches);
    t[4] = run<4>(fr, R, n, ht, ht_n, fs, fs_n, out, launches);
    for (int m = 0; m < 5; ++m)
      printf("{\"pattern\": \"%s\", \"frames\": %u, \"us\": %.3f, \"rep\": %d}\n", names[m], n, t[m], rep);
  }
  return 0;
}
