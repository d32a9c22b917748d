// txseg_lds_probe.hip -- probe (not a product kernel) for the fused TX segment
// build's load scheme, on its exact access pattern: 65,536 segments of 1,448 B
// payload from random positions in 8,192 16 KiB flow buffers (no wraps here)
// into 1514 B frames at a 2048 B stride (payload at frame byte 66), the frame's
// header chunks read and written back, every chunk summed, the two checksum
// fields stored at the end, zeros past the frame to the end of its 128-B block
// (the product's scratch room).  One 16-lane row per segment.
//   A: one unaligned 16-byte window load per frame chunk (the product's scheme)
//   B: aligned 16-byte loads (lane = source chunk), staged in a per-row LDS
//      slice, each lane's window read back as 5 dwords + v_alignbyte
//   C: as B, the window read back by one ds_read_b128 at its byte address
//      (valid only if the LDS runs in unaligned mode: checked)
//   D/E: A/B with SEG segments per row, the next descriptor prefetched
// Every variant's frames are compared with a host-built expectation.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/txseg_lds_probe tools/txseg_lds_probe.hip
//   tools/bin/txseg_lds_probe [launches]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4 gcu4;
typedef __attribute__((address_space(1))) const u32x4u gcu4u;
typedef __attribute__((address_space(1))) u32x4 gu4;

constexpr uint32_t N = 65536, STRIDE = 2048, PAY = 1448, HL = 66, NFLOW = 8192, TXLEN = 16384;
constexpr int K = (HL + PAY + 15) / 16; // 95 frame chunks
constexpr int KEND = 96;                // scratch zeros to the end of the 1536 B block

struct Seg { uint64_t frame_off, s1; }; // 16-byte descriptor: frame offset, payload source offset

__device__ __forceinline__ uint32_t sad4(u32x4 v, uint32_t acc)
{
  acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
  return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}

template <int N_>
__device__ __forceinline__ uint32_t row_ror(uint32_t x)
{
  return (uint32_t) __builtin_amdgcn_update_dpp((int) 0, (int) x, 0x120 + N_, 0xf, 0xf, false);
}

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((gcu4 *) p); }
__device__ __forceinline__ u32x4 ldu(const uint8_t *p) { return __builtin_nontemporal_load((gcu4u *) p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gu4 *) p); }

// bytes [lo, 16) of b over a
__device__ __forceinline__ u32x4 splice_hi(u32x4 a, u32x4 b, int lo)
{
  u32x4 r;
  for (int d = 0; d < 4; ++d) {
    const int s = lo - 4 * d;
    const uint32_t m = s <= 0 ? 0xffffffffu : s >= 4 ? 0u : (0xffffffffu << (8 * s));
    r[d] = (a[d] & ~m) | (b[d] & m);
  }
  return r;
}

// the segment's end: both fields from the row total on the lane holding chunk 1
__device__ __forceinline__ void finish(uint8_t *f, uint32_t acc, int gl, u32x4 h1, uint32_t *out, uint32_t i)
{
  acc += row_ror<8>(acc);
  acc += row_ror<4>(acc);
  acc += row_ror<2>(acc);
  acc += row_ror<1>(acc);
  if (gl == 1) {
    const uint32_t r = acc + h1.x; // stands in for the checksum arithmetic
    *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) r;
    *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) (r >> 16);
    out[i] = r;
  }
}

// A: unaligned windows (TL: temporal window loads)
template <int SEG, bool TL = false>
__global__ __launch_bounds__(256) void k_unaligned(const uint8_t *shm, const Seg *segs, uint8_t *frames, uint32_t *out)
{
  const int gl = threadIdx.x & 15;
  const uint32_t row = blockIdx.x * 16 + threadIdx.x / 16, rows = gridDim.x * 16;
  u32x4 d = *(gcu4 *) (segs + row);
  for (int s = 0; s < SEG; ++s) {
    const uint32_t i = row + s * rows;
    const uint64_t fo = d.x | ((uint64_t) d.y << 32);
    const uint32_t s1 = d.z;
    if (s + 1 < SEG)
      d = *(gcu4 *) (segs + i + rows); // next descriptor in flight during this segment
    uint8_t *f = frames + fo;
    const u32x4 hv = *(gcu4 *) (f + 16 * min(gl, 4));
    const u32x4 w4 = TL ? *(gcu4u *) (shm + s1 - 2) : ldu(shm + s1 - 2);
    u32x4 a[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int k = min(max(gl + 16 * u, 5), K - 1);
      a[u] = TL ? *(gcu4u *) (shm + s1 + 16 * k - HL) : ldu(shm + s1 + 16 * k - HL);
    }
    uint32_t acc = 0;
    if (gl < 5) {
      const u32x4 h = gl == 4 ? splice_hi(hv, w4, 2) : hv;
      *(gu4 *) (f + 16 * gl) = h;
      acc = gl >= 2 ? sad4(h, 0u) : 0u;
    }
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int k = gl + 16 * u;
      if (k >= 5 && k < K) {
        stnt(f + 16 * k, a[u]);
        acc = sad4(a[u], acc);
      } else if (k >= K && k < KEND) {
        stnt(f + 16 * k, u32x4{0u, 0u, 0u, 0u});
      }
    }
    finish(f, acc, gl, hv, out, i);
  }
}

// B / C: aligned loads staged in LDS.  OPT bits: 1 = temporal (not
// non-temporal) source loads; 2 = lanes own source chunks by absolute index
// mod 8 (each load instruction covers whole 128-B lines; 7 rounds); 4 = the
// header chunks go out in round 0's store instruction (one store per line);
// 8 = plain (temporal) frame stores
template <int SEG, bool B128, int OPT = 0>
__global__ __launch_bounds__(256) void k_lds(const uint8_t *shm, const Seg *segs, uint8_t *frames, uint32_t *out)
{
  constexpr int NR = (OPT & 2) ? 7 : 6;         // load rounds
  constexpr int SL = 16 * 16 * NR + 16;         // bytes per row slice
  __shared__ __attribute__((aligned(16))) uint8_t lds[16 * SL];
  const int gl = threadIdx.x & 15;
  const uint32_t rr = threadIdx.x / 16;
  uint8_t *sl = lds + rr * SL;
  const uint32_t row = blockIdx.x * 16 + rr, rows = gridDim.x * 16;
  u32x4 d = *(gcu4 *) (segs + row);
  for (int s = 0; s < SEG; ++s) {
    const uint32_t i = row + s * rows;
    const uint64_t fo = d.x | ((uint64_t) d.y << 32);
    const uint32_t s1 = d.z;
    if (s + 1 < SEG)
      d = *(gcu4 *) (segs + i + rows);
    uint8_t *f = frames + fo;
    const u32x4 hv = *(gcu4 *) (f + 16 * min(gl, 4));
    // first aligned source chunk (chunk 4's window; OPT 2: its 128-B line)
    const uint32_t a0 = (OPT & 2) ? ((s1 - 2u) & ~127u) : ((s1 - 2u) & ~15u);
    // aligned source bytes: through chunk 94's window end (s1 + 16K - HL) plus the 5th dword read
    const uint32_t nsrc = ((s1 + 16u * K - HL + 4u + 15u) & ~15u) - a0;
    u32x4 a[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const uint8_t *src = shm + a0 + min((uint32_t) (16 * (gl + 16 * u)), nsrc - 16u);
      a[u] = (OPT & 1) ? *(gcu4 *) src : ldnt(src);
    }
    if (s > 0)
      __builtin_amdgcn_wave_barrier(); // the previous segment's reads of the slice are done (in order)
#pragma unroll
    for (int u = 0; u < NR; ++u)
      *(u32x4 *) (sl + 16 * (gl + 16 * u)) = a[u];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t sh = s1 - a0; // LDS offset of payload byte 0
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int k = gl + 16 * u;
      if (k >= KEND)
        continue;
      if (k >= K) {
        if (OPT & 8)
          *(gu4 *) (f + 16 * k) = u32x4{0u, 0u, 0u, 0u};
        else
          stnt(f + 16 * k, u32x4{0u, 0u, 0u, 0u});
        continue;
      }
      if (!(OPT & 4) && k < 4)
        continue;
      const uint32_t b = sh + 16 * max(k, 4) - HL; // window's byte offset in the slice
      u32x4 v;
      if (B128) {
        v = *(const u32x4 *) (sl + b);
      } else {
        const uint32_t *w = (const uint32_t *) (sl + (b & ~3u));
        const uint32_t r = b & 3u;
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        v.x = __builtin_amdgcn_alignbyte(w1, w0, r);
        v.y = __builtin_amdgcn_alignbyte(w2, w1, r);
        v.z = __builtin_amdgcn_alignbyte(w3, w2, r);
        v.w = __builtin_amdgcn_alignbyte(w4, w3, r);
      }
      if (k == 4)
        v = splice_hi(hv, v, 2);
      if (k < 4)
        v = hv;
      if (OPT & 8)
        *(gu4 *) (f + 16 * k) = v;
      else if ((OPT & 4) || k > 4)
        stnt(f + 16 * k, v);
      else
        *(gu4 *) (f + 64) = v;
      acc = k >= 2 ? sad4(v, acc) : acc;
    }
    if (!(OPT & 4) && gl < 4) {
      *(gu4 *) (f + 16 * gl) = hv;
      acc = gl >= 2 ? sad4(hv, acc) : acc;
    }
    finish(f, acc, gl, hv, out, i);
  }
}

int main(int argc, char **argv)
{
  const int launches = argc > 1 ? atoi(argv[1]) : 50;
  const int R = argc > 2 ? atoi(argv[2]) : 4; // rotating input sets (each > the MALL)
  const size_t shm_len = (size_t) NFLOW * TXLEN + 64, fr_len = (size_t) N * STRIDE;
  std::vector<uint8_t> hshm(shm_len), hfr(fr_len);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (auto &b : hshm) b = (uint8_t) rnd();
  for (auto &b : hfr) b = (uint8_t) rnd();
  std::vector<Seg> hseg(N);
  for (uint32_t i = 0; i < N; ++i) {
    const uint32_t flow = i % NFLOW;
    hseg[i].frame_off = (uint64_t) i * STRIDE;
    hseg[i].s1 = 16 + (uint64_t) flow * TXLEN + rnd() % (TXLEN - PAY - 32);
  }
  std::vector<uint8_t *> dshm(R), dfr(R);
  Seg *dseg;
  uint32_t *dout;
  for (int r = 0; r < R; ++r) {
    CHK(hipMalloc(&dshm[r], shm_len));
    CHK(hipMalloc(&dfr[r], fr_len));
    CHK(hipMemcpy(dshm[r], hshm.data(), shm_len, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dfr[r], hfr.data(), fr_len, hipMemcpyHostToDevice));
  }
  CHK(hipMalloc(&dseg, N * sizeof(Seg)));
  CHK(hipMemcpy(dseg, hseg.data(), N * sizeof(Seg), hipMemcpyHostToDevice));
  CHK(hipMalloc(&dout, N * 4));
  // the expected frame bytes except the two fields: headers kept, payload copied, zeros to 1536
  std::vector<uint8_t> exp(hfr);
  for (uint32_t i = 0; i < N; ++i) {
    uint8_t *f = exp.data() + (size_t) i * STRIDE;
    memcpy(f + HL, hshm.data() + hseg[i].s1, 16 * K - HL); // the last chunk's window runs 6 B past the payload
    memset(f + 16 * K, 0, (KEND - K) * 16);
  }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  struct V { const char *name; void (*k)(const uint8_t *, const Seg *, uint8_t *, uint32_t *); int seg; };
  V vs[] = {{"A_unaligned", k_unaligned<1>, 1}, {"A1_unaligned_temporal", k_unaligned<1, true>, 1},
            {"B1_temporal_loads", k_lds<1, false, 1>, 1}, {"B5_temporal_header_round0", k_lds<1, false, 5>, 1},
            {"B7_temporal_line_owned_header_round0", k_lds<1, false, 7>, 1},
            {"C5_b128_temporal_header_round0", k_lds<1, true, 5>, 1},
            {"E5_seg2_temporal_header_round0", k_lds<2, false, 5>, 2}, {"A1_again", k_unaligned<1, true>, 1},
            {"B5_again", k_lds<1, false, 5>, 1}};
  std::vector<uint8_t> got(fr_len);
  for (auto &v : vs) {
    const uint32_t grid = N / 16 / v.seg;
    for (int k = 0; k < 3 * R; ++k)
      hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, dshm[k % R], dseg, dfr[k % R], dout);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    for (int k = 0; k < launches; ++k)
      hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, dshm[k % R], dseg, dfr[k % R], dout);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(got.data(), dfr[0], fr_len, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint32_t i = 0; i < N; ++i) {
      const uint8_t *g = got.data() + (size_t) i * STRIDE, *e = exp.data() + (size_t) i * STRIDE;
      for (int b = 0; b < KEND * 16; ++b)
        if (b != 24 && b != 25 && b != 50 && b != 51 && g[b] != e[b]) { ++bad; break; }
    }
    printf("{\"variant\": \"%s\", \"us\": %.3f, \"bad_frames\": %zu}\n", v.name, ms * 1e3 / launches, bad);
    fflush(stdout);
    CHK(hipMemcpy(dfr[0], hfr.data(), fr_len, hipMemcpyHostToDevice));
  }
  return 0;
}
