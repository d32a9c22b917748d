// sync_probe.hip -- what one small launch costs end to end, by the way the
// host learns that it finished (measurement tool for tasx_flush's floor):
//   sync   : hipStreamSynchronize
//   event  : hipEventRecord + spin on hipEventQuery
//   wv32   : hipStreamWriteValue32 into pinned host memory + spin on the word
//   kflag  : the kernel itself stores a sequence number into pinned host
//            memory (system-scope release) + spin on the word
// for an empty kernel and for one that reads NF frames of 1504 B from pinned
// host memory (the zero-copy flush's traffic).
//
//   hipcc --offload-arch=gfx950 -O3 tools/sync_probe.hip -o tools/bin/sync_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void work(const uint4 *frames, uint32_t nf, uint32_t *out, uint32_t *flag, uint32_t *cnt, uint32_t seq)
{
  // one 64-lane wave per frame: 94 x 16 B per 1504 B frame
  const uint32_t f = blockIdx.x;
  uint32_t acc = 0;
  if (f < nf)
    for (uint32_t c = threadIdx.x; c < 94; c += 64) {
      const uint4 v = frames[(size_t) f * 128 + c];
      acc += v.x + v.y + v.z + v.w;
    }
  for (int o = 32; o > 0; o >>= 1)
    acc += __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0 && f < nf)
    out[f] = acc;
  if (flag && !cnt && threadIdx.x == 0)
    __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (flag && cnt && threadIdx.x == 0) {
    // the last block to finish (device-memory counter) posts the host word
    const uint32_t old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void post(uint32_t *flag, uint32_t seq)
{
  __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us()
{
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// bounded spin: a word that never arrives ends the probe instead of hanging it
static void spin_until(const uint32_t *w, uint32_t v, const char *what)
{
  const double t0 = now_us();
  while (*(volatile const uint32_t *) w != v)
    if (now_us() - t0 > 1e6) {
      fprintf(stderr, "%s: completion word never arrived (have %u, want %u)\n", what, *(volatile const uint32_t *) w, v);
      exit(2);
    }
}

int main(int argc, char **argv)
{
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint4 *frames;
  uint32_t *hflag, *out, *dcnt;
  CK(hipHostMalloc((void **) &frames, 512 * 2048, 0));
  CK(hipHostMalloc((void **) &hflag, 64, hipHostMallocCoherent));
  CK(hipMalloc((void **) &out, 4096));
  CK(hipMalloc((void **) &dcnt, 64));
  CK(hipMemset(dcnt, 0, 64));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char *modes[] = {"sync", "event", "wv32", "kflag", "kflag_last", "postk"};
  for (uint32_t nf : {0u, 1u, 32u, 128u}) {
    for (int m = 0; m < 6; ++m) {
      std::vector<double> t;
      uint32_t seq = 0;
      *(volatile uint32_t *) hflag = 0;
      for (int r = 0; r < reps + 50; ++r) {
        const uint32_t blocks = std::max(nf, 1u);
        const double t0 = now_us();
        if (m >= 4)
          ++seq;
        hipLaunchKernelGGL(work, dim3(blocks), dim3(64), 0, st, frames, nf, out, (m == 3 || m == 4) ? hflag : nullptr,
                           m == 4 ? dcnt : nullptr, seq);
        if (m == 0) {
          CK(hipStreamSynchronize(st));
        } else if (m == 1) {
          CK(hipEventRecord(ev, st));
          while (hipEventQuery(ev) == hipErrorNotReady) {
          }
        } else if (m == 2) {
          ++seq;
          CK(hipStreamWriteValue32(st, hflag, seq, 0));
          spin_until(hflag, seq, "wv32");
        } else if (m == 3) {
          seq += blocks;
          spin_until(hflag, seq, "kflag");
        } else if (m == 4) {
          spin_until(hflag, seq, "kflag_last");
        } else {
          hipLaunchKernelGGL(post, dim3(1), dim3(1), 0, st, hflag, seq);
          spin_until(hflag, seq, "postk");
        }
        const double t1 = now_us();
        if (r >= 50)
          t.push_back(t1 - t0);
      }
      CK(hipStreamSynchronize(st));
      std::sort(t.begin(), t.end());
      printf("{\"frames\": %u, \"mode\": \"%s\", \"p50_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", nf,
             modes[m], t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
      fflush(stdout);
    }
  }
  return 0;
}
