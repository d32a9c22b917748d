// copy_ceiling.hip -- the device's read+write streaming rate (not a product
// kernel): hipMemcpyAsync D2D against hand-written grid-stride copies (16 B per
// lane, plain or non-temporal loads/stores), over 4 rotating buffer pairs of
// the TX segment build's block-floor bytes (107 MB each way; 856 MB in all,
// more than the MALL holds).  Prints one JSON line per method.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/copy_ceiling tools/copy_ceiling.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu4;
typedef __attribute__((address_space(1))) const u32x4 gcu4;

// U chunks per lane per iteration, all loads issued before the stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4 *src, u32x4 *dst, size_t nchunks)
{
  const size_t stride = (size_t) gridDim.x * 256u * U;
  for (size_t base = (size_t) blockIdx.x * 256u * U + threadIdx.x; base < nchunks; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t c = base + (size_t) u * 256u;
      if (c < nchunks)
        v[u] = NT ? __builtin_nontemporal_load((gcu4 *) (src + c)) : *(gcu4 *) (src + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t c = base + (size_t) u * 256u;
      if (c < nchunks) {
        if (NT)
          __builtin_nontemporal_store(v[u], (gu4 *) (dst + c));
        else
          *(gu4 *) (dst + c) = v[u];
      }
    }
  }
}

int main(int argc, char **argv)
{
  const size_t bytes = argc > 1 ? strtoull(argv[1], NULL, 10) : 107188032ull;
  const int R = 4, K = 50;
  const size_t nchunks = bytes / 16;
  std::vector<u32x4 *> src(R), dst(R);
  for (int r = 0; r < R; ++r) {
    CHK(hipMalloc(&src[r], bytes));
    CHK(hipMalloc(&dst[r], bytes));
    CHK(hipMemset(src[r], 0x11 + r, bytes));
    CHK(hipMemset(dst[r], 0, bytes));
  }
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch) {
    std::vector<float> w;
    for (int k = 0; k < 8; ++k)
      launch(k % R);
    for (int rep = 0; rep < 5; ++rep) {
      CHK(hipEventRecord(e0, s));
      for (int k = 0; k < K; ++k)
        launch(k % R);
      CHK(hipEventRecord(e1, s));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      w.push_back(ms * 1e3f / K);
    }
    std::sort(w.begin(), w.end());
    printf("{\"method\": \"%s\", \"bytes_each_way\": %zu, \"us_median\": %.3f, \"us_min\": %.3f, "
           "\"GBps_rw\": %.1f, \"frac_of_8TBps\": %.4f}\n",
           name, bytes, w[2], w[0], 2.0 * bytes / w[2] / 1e3, 2.0 * bytes / w[2] / 8e6);
    fflush(stdout);
  };
  int cus = 256;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  timeit("hipMemcpyAsync D2D", [&](int r) { CHK(hipMemcpyAsync(dst[r], src[r], bytes, hipMemcpyDeviceToDevice, s)); });
  for (int g : {cus * 4, cus * 8, cus * 16, (int) ((nchunks + 255) / 256)}) {
    char nm[96];
    snprintf(nm, sizeof nm, "copy_kernel<1, nt> grid %d", g);
    timeit(nm, [&](int r) { hipLaunchKernelGGL((copy_kernel<1, true>), dim3(g), dim3(256), 0, s, src[r], dst[r], nchunks); });
    snprintf(nm, sizeof nm, "copy_kernel<4, nt> grid %d", g);
    timeit(nm, [&](int r) { hipLaunchKernelGGL((copy_kernel<4, true>), dim3(g), dim3(256), 0, s, src[r], dst[r], nchunks); });
    snprintf(nm, sizeof nm, "copy_kernel<4, plain> grid %d", g);
    timeit(nm, [&](int r) { hipLaunchKernelGGL((copy_kernel<4, false>), dim3(g), dim3(256), 0, s, src[r], dst[r], nchunks); });
  }
  return 0;
}
