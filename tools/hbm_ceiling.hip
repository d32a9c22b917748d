// hbm_ceiling.hip -- practical HBM read ceiling on this MI355X for the batch
// sizes the checksum path sees (a known-good reference measured on the same
// hardware, cdna_hip_programming.md section 5.4 rule 10).  Not part of the product.
//
// Pure streaming read + integer fold (the same VALU work per byte as the
// checksum, no packet structure), over R rotating buffers of B bytes each so
// every launch reads HBM.  Reports per-launch time (hipEvents around each
// launch, and total / K back-to-back) for several launch shapes.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/hbm_ceiling tools/hbm_ceiling.hip
//   tools/bin/hbm_ceiling [bytes_per_launch] [rotations] [launches] [all|glds|blk]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <string.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gcu4;

template <bool NT>
__device__ __forceinline__ u32x4 ld(const gcu4 *g, uint64_t i)
{
  if constexpr (NT)
    return __builtin_nontemporal_load(&g[i]);
  else
    return g[i];
}

// grid-stride: each thread U chunks in flight per iteration
template <int U, int BS, bool NT>
__global__ __launch_bounds__(BS) void stream_gs(const u32x4 *p, uint64_t nchunks, uint32_t *out)
{
  const gcu4 *g = (const gcu4 *) p;
  uint64_t acc = 0;
  const uint64_t T = (uint64_t) gridDim.x * BS;
  uint64_t i = (uint64_t) blockIdx.x * BS + threadIdx.x;
  for (; i + (U - 1) * T < nchunks; i += U * T) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(g, i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u) { acc += v[u].x; acc += v[u].y; acc += v[u].z; acc += v[u].w; }
  }
  for (; i < nchunks; i += T) { u32x4 v = ld<NT>(g, i); acc += v.x; acc += v.y; acc += v.z; acc += v.w; }
  uint32_t r = (uint32_t) acc + (uint32_t) (acc >> 32);
  if (r == 0x12345678u) out[0] = r;  // keep live, never true for this data
}

// block-contiguous: block b reads chunks [b*S, (b+1)*S) with S = BS*U*iters,
// wave-contiguous 1 KiB per load, U loads in flight per thread
template <int U, int BS, bool NT>
__global__ __launch_bounds__(BS) void stream_blk(const u32x4 *p, uint64_t nchunks, uint64_t per_block, uint32_t *out)
{
  const gcu4 *g = (const gcu4 *) p;
  const uint64_t b0 = (uint64_t) blockIdx.x * per_block;
  const uint64_t b1 = min(b0 + per_block, nchunks);
  uint64_t acc = 0;
  for (uint64_t base = b0; base < b1; base += (uint64_t) BS * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = base + (uint64_t) u * BS + threadIdx.x;
      v[u] = ld<NT>(g, i < b1 ? i : b0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = base + (uint64_t) u * BS + threadIdx.x;
      if (i < b1) { acc += v[u].x; acc += v[u].y; acc += v[u].z; acc += v[u].w; }
    }
  }
  uint32_t r = (uint32_t) acc + (uint32_t) (acc >> 32);
  if (r == 0x12345678u) out[0] = r;
}

// LDS-DMA (round 4): gfx950's 16-byte global_load_lds_dwordx4
// lands each lane's 16 bytes in LDS with no VGPR destination; one wave-instruction
// writes 1 KiB linearly at M0.  Each wave owns a ring of D 1-KiB slots; group j
// (64 consecutive chunks) goes to slot j % D.  The wave waits for its own oldest
// DMA with a counted vmcnt (same-wave ordering needs no barrier), folds the slot
// with ds_read_b128 + v_sad_u16, then refills it with group j + D.  FOLD = false
// skips the LDS read (pure DMA issue rate).
template <bool NT>
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr)
{
  uint32_t keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_addr) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_addr) : "memory");
}

template <int D, int BS, bool NT, bool FOLD>
__global__ __launch_bounds__(BS) void stream_glds(const u32x4 *p, uint64_t ngroups, uint32_t *out)
{
  __shared__ u32x4 ring[BS / 64][D][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) &ring[wave][0][0]);
  const uint64_t W = (uint64_t) gridDim.x * (BS / 64);
  const uint64_t g0 = __builtin_amdgcn_readfirstlane((uint32_t) (blockIdx.x * (BS / 64) + wave));
  // groups g0, g0 + W, ...: n_it of them for this wave
  const uint64_t n_it = g0 < ngroups ? (ngroups - g0 + W - 1) / W : 0;
  uint32_t acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < n_it) glds16<NT>(p + (g0 + d * W) * 64 + lane, lbase + d * 1024);
  uint64_t it = 0;
  for (; it + D < n_it; ++it) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D - 1) : "memory");
    const int slot = (int) (it % D);
    if constexpr (FOLD) {
      u32x4 v = ring[wave][slot][lane];
      acc = __builtin_amdgcn_sad_u16(v.x, 0, acc);
      acc = __builtin_amdgcn_sad_u16(v.y, 0, acc);
      acc = __builtin_amdgcn_sad_u16(v.z, 0, acc);
      acc = __builtin_amdgcn_sad_u16(v.w, 0, acc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    glds16<NT>(p + (g0 + (it + D) * W) * 64 + lane, lbase + slot * 1024);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (; it < n_it; ++it) {
    if constexpr (FOLD) {
      u32x4 v = ring[wave][it % D][lane];
      acc = __builtin_amdgcn_sad_u16(v.x, 0, acc);
      acc = __builtin_amdgcn_sad_u16(v.y, 0, acc);
      acc = __builtin_amdgcn_sad_u16(v.z, 0, acc);
      acc = __builtin_amdgcn_sad_u16(v.w, 0, acc);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
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
  CHK(hipEventRecord(t0, s));
  for (int k = 0; k < K; ++k) launch(k % R);
  CHK(hipEventRecord(t1, s));
  CHK(hipEventSynchronize(t1));
  float tot; CHK(hipEventElapsedTime(&tot, t0, t1));
  for (int k = 0; k < K; ++k) { CHK(hipEventRecord(a[k], s)); launch(k % R); CHK(hipEventRecord(b[k], s)); }
  CHK(hipStreamSynchronize(s));
  std::vector<float> d(K);
  for (int k = 0; k < K; ++k) CHK(hipEventElapsedTime(&d[k], a[k], b[k]));
  std::sort(d.begin(), d.end());
  for (int k = 0; k < K; ++k) { (void) hipEventDestroy(a[k]); (void) hipEventDestroy(b[k]); }
  (void) hipEventDestroy(t0); (void) hipEventDestroy(t1);
  return {d[K / 2] * 1e3, tot * 1e3 / K};
}

static uint64_t B;
static void report(const char *name, Res r)
{
  printf("%-40s event-median %8.2f us %6.0f GB/s | wall/K %8.2f us %6.0f GB/s\n", name,
         r.ev_us, B / r.ev_us / 1e3, r.wall_us, B / r.wall_us / 1e3);
  fflush(stdout);
}

template <int U, int BS, bool NT>
void gs_case(std::vector<u32x4 *> &buf, uint64_t nch, uint32_t *out, int R, int K, hipStream_t s, int ncu, int bpc)
{
  int grid = ncu * bpc;
  char nm[96];
  snprintf(nm, sizeof nm, "gs U=%d BS=%d %s %d blk/CU", U, BS, NT ? "nt" : "  ", bpc);
  report(nm, run([&](int r) { hipLaunchKernelGGL((stream_gs<U, BS, NT>), dim3(grid), dim3(BS), 0, s, buf[r], nch, out); }, R, K, s));
}

template <int U, int BS, bool NT>
void blk_case(std::vector<u32x4 *> &buf, uint64_t nch, uint32_t *out, int R, int K, hipStream_t s, uint64_t per_block)
{
  int grid = (int) ((nch + per_block - 1) / per_block);
  char nm[96];
  snprintf(nm, sizeof nm, "blk U=%d BS=%d %s %llu KiB/blk (%d blk)", U, BS, NT ? "nt" : "  ",
           (unsigned long long) per_block / 64, grid);
  report(nm, run([&](int r) { hipLaunchKernelGGL((stream_blk<U, BS, NT>), dim3(grid), dim3(BS), 0, s, buf[r], nch, per_block, out); }, R, K, s));
}

template <int D, int BS, bool NT, bool FOLD>
void glds_case(std::vector<u32x4 *> &buf, uint64_t nch, uint32_t *out, int R, int K, hipStream_t s, int ncu, int bpc)
{
  const uint64_t ngroups = nch / 64;  // whole 1-KiB groups (the tail < 1 KiB is not read)
  int grid = ncu * bpc;
  char nm[96];
  snprintf(nm, sizeof nm, "glds D=%d BS=%d %s%s %d blk/CU", D, BS, NT ? "nt" : "  ", FOLD ? "" : " nofold", bpc);
  report(nm, run([&](int r) { hipLaunchKernelGGL((stream_glds<D, BS, NT, FOLD>), dim3(grid), dim3(BS), 0, s, buf[r], ngroups, out); }, R, K, s));
}

int main(int argc, char **argv)
{
  B = argc > 1 ? strtoull(argv[1], 0, 0) : 98304000ull;
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
  int ncu = prop.multiProcessorCount;
  printf("CUs %d, %llu B per launch, %d rotating buffers, %d launches\n", ncu, (unsigned long long) B, R, K);
  const char *mode = argc > 4 ? argv[4] : "all";
  if (!strcmp(mode, "glds") || !strcmp(mode, "all")) {
    // register-load references first, then LDS-DMA rings at several depths / residencies
    gs_case<8, 256, false>(buf, nch, out, R, K, s, ncu, 8);
    gs_case<8, 256, true>(buf, nch, out, R, K, s, ncu, 8);
    gs_case<4, 256, false>(buf, nch, out, R, K, s, ncu, 16);
    for (int bpc : {2, 4, 8}) {
      glds_case<4, 256, false, true>(buf, nch, out, R, K, s, ncu, bpc);
      glds_case<4, 256, true, true>(buf, nch, out, R, K, s, ncu, bpc);
      glds_case<8, 256, false, true>(buf, nch, out, R, K, s, ncu, bpc);
      glds_case<8, 256, true, true>(buf, nch, out, R, K, s, ncu, bpc);
      glds_case<8, 256, true, false>(buf, nch, out, R, K, s, ncu, bpc);
    }
    for (int bpc : {1, 2, 4}) {
      glds_case<16, 256, false, true>(buf, nch, out, R, K, s, ncu, bpc);
      glds_case<16, 256, true, true>(buf, nch, out, R, K, s, ncu, bpc);
      glds_case<16, 512, true, true>(buf, nch, out, R, K, s, ncu, bpc);
    }
    glds_case<4, 1024, true, true>(buf, nch, out, R, K, s, ncu, 1);
    glds_case<4, 1024, true, true>(buf, nch, out, R, K, s, ncu, 2);
    if (!strcmp(mode, "glds")) return 0;
  }
  if (!strcmp(mode, "blk")) {  // the fastest register-load shapes only
    for (uint64_t kib : {8, 16, 32}) {
      blk_case<8, 256, true>(buf, nch, out, R, K, s, kib * 64);
      blk_case<4, 256, true>(buf, nch, out, R, K, s, kib * 64);
    }
    return 0;
  }
  for (int bpc : {2, 4, 8, 16}) {
    gs_case<4, 256, false>(buf, nch, out, R, K, s, ncu, bpc);
    gs_case<8, 256, false>(buf, nch, out, R, K, s, ncu, bpc);
    gs_case<8, 256, true>(buf, nch, out, R, K, s, ncu, bpc);
  }
  for (int bpc : {1, 2, 4}) {
    gs_case<4, 512, false>(buf, nch, out, R, K, s, ncu, bpc);
    gs_case<8, 512, false>(buf, nch, out, R, K, s, ncu, bpc);
    gs_case<4, 1024, false>(buf, nch, out, R, K, s, ncu, bpc);
    gs_case<8, 1024, false>(buf, nch, out, R, K, s, ncu, bpc);
  }
  for (uint64_t kib : {4, 8, 16, 24, 32, 64}) {
    blk_case<4, 256, false>(buf, nch, out, R, K, s, kib * 64);
    blk_case<6, 256, false>(buf, nch, out, R, K, s, kib * 64);
    blk_case<8, 256, false>(buf, nch, out, R, K, s, kib * 64);
    blk_case<8, 256, true>(buf, nch, out, R, K, s, kib * 64);
  }
  return 0;
}
