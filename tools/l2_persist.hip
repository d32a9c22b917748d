// l2_persist.hip -- does a flow table stay in an XCD's L2 from one launch to the
// next, and what evicts it?  Not part of the product (the
// flow tables L2-resident per XCD).
//
// A dependent pointer chase over 128-byte lines of a table of S bytes: every
// lane of every block follows its own random cycle, one load at a time, and
// the kernel reports the mean wall-clock time per step (s_memrealtime, 100 MHz).
// "part" mode: the table is cut into 8 slices and a block chases only the slice
// of the XCD it runs on (HW_REG_XCC_ID), so each XCD touches S/8 bytes;
// "full" mode: every block chases over the whole table.  Sequence per mode:
//   cold     the first chase after a 1 GiB streaming read (caches flushed)
//   again    the same chase, the next launch
//   nt64     after a 64 MiB non-temporal streaming read of another buffer
//   again
//   def64    after a 64 MiB default-policy streaming read
//   again
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/l2_persist tools/l2_persist.hip
//   tools/bin/l2_persist [table_MiB ...]      (default 2 16)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <numeric>
#include <algorithm>
#include <random>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

constexpr int kBlocks = 256 * 2, kThreads = 64, kSteps = 256;

__device__ __forceinline__ uint32_t xcc_id()
{
  // HW_REG_XCC_ID = 20, bits [3:0]
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
}

// next[] holds, per 128-byte line (32 u32), the index of the next line in the
// line's first word; slices of `lines_per_part` lines each form their own cycle
__global__ __launch_bounds__(kThreads) void chase(const uint32_t *tab, uint32_t lines_per_part, int part,
                                                  uint64_t *ticks, uint32_t *sink)
{
  const uint32_t x = part ? xcc_id() : 0u;
  const uint32_t base = x * lines_per_part;
  uint32_t l = base + (uint32_t) ((blockIdx.x * 977u + threadIdx.x * 131u) % lines_per_part);
  const uint64_t t0 = wall_clock64();
  for (int s = 0; s < kSteps; s++)
    l = tab[(uint64_t) l * 32u];
  const uint64_t t1 = wall_clock64();
  if (threadIdx.x == 0)
    atomicAdd((unsigned long long *) ticks, (unsigned long long) (t1 - t0));
  if (l == 0xffffffffu)
    sink[0] = l;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void stream(const u32x4 *p, uint64_t n, uint32_t *sink)
{
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t) gridDim.x * 256u) {
    u32x4 v = NT ? __builtin_nontemporal_load(&p[i]) : p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u)
    sink[1] = acc;
}

int main(int argc, char **argv)
{
  std::vector<int> mibs;
  for (int i = 1; i < argc; i++)
    mibs.push_back(atoi(argv[i]));
  if (mibs.empty())
    mibs = {2, 16};
  int khz = 0;
  CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const size_t big = 1ull << 30, s64 = 64ull << 20;
  u32x4 *flush = nullptr, *other = nullptr;
  uint32_t *sink = nullptr;
  uint64_t *ticks = nullptr;
  CHK(hipMalloc(&flush, big));
  CHK(hipMalloc(&other, s64));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMalloc(&ticks, 8));
  CHK(hipMemset(flush, 1, big));
  CHK(hipMemset(other, 2, s64));
  for (int mib : mibs) {
    const uint32_t lines = (uint32_t) ((size_t) mib << 20) / 128u;
    uint32_t *tab = nullptr;
    CHK(hipMalloc(&tab, (size_t) lines * 128u));
    for (int part = 0; part < 2; part++) {
      const uint32_t lpp = part ? lines / 8u : lines;
      std::vector<uint32_t> h((size_t) lines * 32u, 0u);
      std::mt19937 rng(1234 + mib);
      for (uint32_t pbase = 0; pbase < lines; pbase += lpp) {
        std::vector<uint32_t> perm(lpp);
        std::iota(perm.begin(), perm.end(), 0u);
        std::shuffle(perm.begin(), perm.end(), rng);
        for (uint32_t i = 0; i < lpp; i++)
          h[(size_t) (pbase + perm[i]) * 32u] = pbase + perm[(i + 1) % lpp];
      }
      CHK(hipMemcpy(tab, h.data(), (size_t) lines * 128u, hipMemcpyHostToDevice));
      const char *names[6] = {"cold", "again", "nt64", "again", "def64", "again"};
      printf("{\"table_MiB\": %d, \"mode\": \"%s\"", mib, part ? "part" : "full");
      for (int k = 0; k < 6; k++) {
        if (k == 0)
          hipLaunchKernelGGL(stream<false>, dim3(2048), dim3(256), 0, 0, flush, big / 16, sink);
        if (k == 2)
          hipLaunchKernelGGL(stream<true>, dim3(2048), dim3(256), 0, 0, other, s64 / 16, sink);
        if (k == 4)
          hipLaunchKernelGGL(stream<false>, dim3(2048), dim3(256), 0, 0, other, s64 / 16, sink);
        CHK(hipMemset(ticks, 0, 8));
        hipLaunchKernelGGL(chase, dim3(kBlocks), dim3(kThreads), 0, 0, tab, lpp, part, ticks, sink);
        CHK(hipDeviceSynchronize());
        uint64_t t = 0;
        CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
        const double ns = (double) t / kBlocks / kSteps * 1e6 / khz;
        printf(", \"%s%s\": %.1f", names[k], k == 1 || k == 3 || k == 5 ? (k == 1 ? "" : k == 3 ? "_nt" : "_def") : "", ns);
      }
      printf("}\n");
      fflush(stdout);
    }
    CHK(hipFree(tab));
  }
  return 0;
}
