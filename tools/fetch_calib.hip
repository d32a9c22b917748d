// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE on gfx950 for the access
// widths the TX segment build uses (not a product kernel).  MI355X_MICROARCH.md:
// "FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming
// read ... other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern".  Every kernel reads a known set of 64 B
// lines once (the host counts them) and writes 4 B per segment:
//   stream      95.4 MB contiguous, 16 B per lane (the guide's calibrated case)
//   seg_a64     65,536 segments of 1,456 B (91 chunks) at 64 B aligned offsets
//   seg_a16     the same at 16 B aligned offsets (lines touched: 23 or 24)
//   seg_u       the same at byte offsets, one unaligned 16 B load per chunk
//               (the TX segment kernel's payload window loads)
//   hdr         the frame-header reads of the TX segment kernel alone: chunks
//               0..4 of each 2048 B frame (2 lines)
// Run under `rocprofv3 --pmc FETCH_SIZE` (and `--pmc TCC_EA0_RDREQ_sum ...`);
// compare FETCH_SIZE x 1024 with the touched bytes printed here.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4u gcu4u;
typedef __attribute__((address_space(1))) const u32x4 gcu4;

constexpr int NCH = 91;

__device__ __forceinline__ uint32_t sad4(u32x4 v, uint32_t a)
{
  return __builtin_amdgcn_sad_u16(v.x, 0, __builtin_amdgcn_sad_u16(v.y, 0,
         __builtin_amdgcn_sad_u16(v.z, 0, __builtin_amdgcn_sad_u16(v.w, 0, a))));
}

// one 16-lane row per segment, 6 chunk loads per lane (clamped, as the kernels)
template <bool ALIGNED>
__global__ __launch_bounds__(256) void seg_read(const uint8_t *src, const uint32_t *soff, uint32_t n, uint32_t *out)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16;
  if (i >= n)
    return;
  const uint32_t so = soff[i];
  uint32_t acc = 0;
  u32x4 v[6];
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const uint32_t c = min((uint32_t) (gl + 16 * u), (uint32_t) NCH - 1);
    v[u] = ALIGNED ? __builtin_nontemporal_load((gcu4 *) (src + so + 16u * c))
                   : __builtin_nontemporal_load((gcu4u *) (src + so + 16u * c));
  }
#pragma unroll
  for (int u = 0; u < 6; ++u)
    acc = (gl + 16 * u < NCH) ? sad4(v[u], acc) : acc;
  for (int m = 8; m >= 1; m >>= 1)
    acc += __shfl_xor(acc, m, 16);
  if (gl == 0)
    out[i] = acc;
}

__global__ __launch_bounds__(256) void stream_read(const uint8_t *src, uint32_t nchunks, uint32_t *out)
{
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t c = t; c < nchunks; c += gridDim.x * 256)
    acc = sad4(__builtin_nontemporal_load((gcu4 *) (src + 16u * c)), acc);
  if (acc == 0x12345678u)
    out[0] = acc;
}

__global__ __launch_bounds__(256) void hdr_read(const uint8_t *fr, uint32_t n, uint32_t *out)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * 16 + threadIdx.x / 16;
  if (i >= n)
    return;
  const u32x4 h = __builtin_nontemporal_load((gcu4 *) (fr + (size_t) i * 2048 + 16u * min(gl, 4)));
  uint32_t acc = sad4(h, 0);
  for (int m = 8; m >= 1; m >>= 1)
    acc += __shfl_xor(acc, m, 16);
  if (gl == 0)
    out[i] = acc;
}

static uint64_t lines_bytes(const std::vector<uint32_t> &off, uint32_t len)
{
  uint64_t b = 0;
  for (uint32_t o : off)
    b += 64ull * (((uint64_t) o + len + 63) / 64 - o / 64);
  return b;
}

int main()
{
  const uint32_t n = 65536, flows = 8192;
  const size_t shm = (size_t) flows * 16384 + 64;
  uint8_t *src, *fr;
  uint32_t *out, *d_off[3];
  CHK(hipMalloc(&src, shm));
  CHK(hipMemset(src, 0x5a, shm));
  CHK(hipMalloc(&fr, (size_t) n * 2048));
  CHK(hipMemset(fr, 0x3c, (size_t) n * 2048));
  CHK(hipMalloc(&out, n * 4));
  std::vector<uint32_t> off[3]; // 64-aligned, 16-aligned, byte
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < n; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    const uint32_t f = (uint32_t) ((i * 2654435761ull) % flows);
    const uint32_t pos = (uint32_t) (x % (16384 - 1456 - 64));
    off[0].push_back(f * 16384u + (pos & ~63u));
    off[1].push_back(f * 16384u + (pos & ~15u));
    off[2].push_back(f * 16384u + pos);
  }
  for (int k = 0; k < 3; ++k) {
    CHK(hipMalloc(&d_off[k], n * 4));
    CHK(hipMemcpy(d_off[k], off[k].data(), n * 4, hipMemcpyHostToDevice));
  }
  const uint32_t nchunks = n * NCH;
  // distinct lines of the segment sets (segments of different flows never share
  // a line; two segments of one flow may: count the union)
  auto uniq = [&](const std::vector<uint32_t> &o) {
    std::vector<uint8_t> seen(shm / 64 + 1, 0);
    uint64_t b = 0;
    for (uint32_t s : o)
      for (uint64_t l = s / 64; l <= ((uint64_t) s + 1456 - 1) / 64; ++l)
        if (!seen[l]) { seen[l] = 1; b += 64; }
    return b;
  };
  const dim3 g(n / 16), b(256);
  for (int rep = 0; rep < 4; ++rep) {
    hipLaunchKernelGGL(stream_read, dim3(2048), b, 0, 0, src, nchunks, out);
    hipLaunchKernelGGL(seg_read<true>, g, b, 0, 0, src, d_off[0], n, out);
    hipLaunchKernelGGL(seg_read<true>, g, b, 0, 0, src, d_off[1], n, out);
    hipLaunchKernelGGL(seg_read<false>, g, b, 0, 0, src, d_off[2], n, out);
    hipLaunchKernelGGL(hdr_read, g, b, 0, 0, fr, n, out);
  }
  CHK(hipDeviceSynchronize());
  printf("{\"kernel\": \"stream_read\", \"touched_bytes\": %llu}\n", (unsigned long long) nchunks * 16ull);
  printf("{\"kernel\": \"seg_read<true>#64\", \"touched_bytes\": %llu, \"sum_of_segment_lines\": %llu}\n",
         (unsigned long long) uniq(off[0]), (unsigned long long) lines_bytes(off[0], 1456));
  printf("{\"kernel\": \"seg_read<true>#16\", \"touched_bytes\": %llu, \"sum_of_segment_lines\": %llu}\n",
         (unsigned long long) uniq(off[1]), (unsigned long long) lines_bytes(off[1], 1456));
  printf("{\"kernel\": \"seg_read<false>\", \"touched_bytes\": %llu, \"sum_of_segment_lines\": %llu}\n",
         (unsigned long long) uniq(off[2]), (unsigned long long) lines_bytes(off[2], 1456));
  printf("{\"kernel\": \"hdr_read\", \"touched_bytes\": %llu}\n", (unsigned long long) n * 128ull);
  printf("{\"order\": \"per rep: stream_read, seg_read<true> (64-aligned), seg_read<true> (16-aligned), "
         "seg_read<false>, hdr_read\"}\n");
  return 0;
}
