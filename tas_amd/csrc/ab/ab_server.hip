// ab/ab_server.hip -- A/B build only (libtasx_ab.so): the flush server with
// its per-batch timing sums (TASX_SRV_DIAG, tasx_ab_server_diag;
// tools/server_diag.py, profiles/r04/INDEX.md r04m, r04x).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../tasx_kernels.h"
#include "../server_device.h"

extern "C" TASX_INTERNAL int ab_launch_server(const tasx_srv_params *p, void *stream)
{
  hipLaunchKernelGGL(flush_server_kernel<true>, dim3(TASX_MAX_CTX * p->k), dim3(kSrvBlock), 0, (hipStream_t) stream,
                     *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
