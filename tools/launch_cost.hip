// launch_cost.hip -- host-side cost of issuing a flush's GPU work (not a
// product file): two kernel launches (the checksum kernel's shape + a one-lane
// completion kernel) against one hipGraphLaunch of the same two nodes, with
// and without updating the first node's parameters each time (what a flush
// whose batch size changes would need).  Host microseconds per issue, median
// of 5 x 2000 issues (the stream is drained every 64 issues, outside the
// timed calls).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/launch_cost tools/launch_cost.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <time.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); return 1;} } while (0)

struct Args {
  const uint8_t *base;
  const uint64_t *off;
  uint32_t *out;
  uint32_t n, pad[3];
};

__global__ __launch_bounds__(256) void work_kernel(Args a)
{
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < a.n)
    a.out[i] = a.base[a.off[i]];
}

__global__ __launch_bounds__(64) void done_kernel(uint32_t *w, uint32_t v)
{
  if (threadIdx.x == 0)
    __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us()
{
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main()
{
  const uint32_t n = 32;
  uint8_t *base;
  uint64_t *off;
  uint32_t *out, *word;
  CHK(hipMalloc(&base, 1 << 20));
  CHK(hipMalloc(&off, n * 8));
  CHK(hipMemset(off, 0, n * 8));
  CHK(hipMalloc(&out, n * 4));
  CHK(hipHostMalloc(&word, 64, hipHostMallocCoherent));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Args a{base, off, out, n, {0, 0, 0}};

  // the graph: work_kernel -> done_kernel
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(work_kernel, dim3(1), dim3(256), 0, s, a);
  hipLaunchKernelGGL(done_kernel, dim3(1), dim3(64), 0, s, word, 1u);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CHK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CHK(hipGraphGetNodes(g, nodes.data(), &nn));
  hipKernelNodeParams kp;
  hipGraphNode_t work_node = nullptr;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    CHK(hipGraphNodeGetType(nd, &t));
    if (t == hipGraphNodeTypeKernel) {
      CHK(hipGraphKernelNodeGetParams(nd, &kp));
      if (kp.func == (void *) work_kernel) {
        work_node = nd;
        break;
      }
    }
  }
  if (!work_node) {
    fprintf(stderr, "work node not found\n");
    return 1;
  }
  hipKernelNodeParams wp;
  CHK(hipGraphKernelNodeGetParams(work_node, &wp));

  auto bench = [&](const char *name, auto issue) -> int {
    std::vector<double> med;
    for (int rep = 0; rep < 5; ++rep) {
      double tot = 0;
      for (int k = 0; k < 2000; ++k) {
        const double t0 = now_us();
        issue(k);
        tot += now_us() - t0;
        if ((k & 63) == 63)
          CHK(hipStreamSynchronize(s));
      }
      CHK(hipStreamSynchronize(s));
      med.push_back(tot / 2000);
    }
    std::sort(med.begin(), med.end());
    printf("{\"issue\": \"%s\", \"host_us\": %.3f}\n", name, med[2]);
    fflush(stdout);
    return 0;
  };
  bench("two hipLaunchKernelGGL", [&](int k) {
    hipLaunchKernelGGL(work_kernel, dim3(1), dim3(256), 0, s, a);
    hipLaunchKernelGGL(done_kernel, dim3(1), dim3(64), 0, s, word, (uint32_t) k);
  });
  bench("one hipLaunchKernelGGL", [&](int) { hipLaunchKernelGGL(work_kernel, dim3(1), dim3(256), 0, s, a); });
  bench("hipGraphLaunch (fixed params)", [&](int) { (void) hipGraphLaunch(ge, s); });
  Args a2 = a;
  void *argp[] = {&a2};
  bench("hipGraphExecKernelNodeSetParams + hipGraphLaunch", [&](int k) {
    a2.n = n - (uint32_t) (k & 7);
    hipKernelNodeParams p2 = wp;
    p2.kernelParams = argp;
    (void) hipGraphExecKernelNodeSetParams(ge, work_node, &p2);
    (void) hipGraphLaunch(ge, s);
  });
  return 0;
}
