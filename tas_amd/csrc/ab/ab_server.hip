// ab/ab_server.hip -- A/B build only (libtasx_ab.so): the flush server's
// other forms -- its per-batch timing sums (TASX_SRV_DIAG, tasx_ab_server_diag;
// tools/server_diag.py, profiles/r04/INDEX.md r04m, r04x, profiles/r05 r05h,
// r05k) and, for pricing what the server costs device-resident work beside it
// only, the per-batch acquire at agent scope or left out (TASX_SRV_ACQ=1 / 2,
// read at each start; profiles/r05 r05l).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "../tasx_kernels.h"
#include "../server_device.h"

template <bool DIAG>
static void launch_acq(int acq, const tasx_srv_params *p, hipStream_t s)
{
  const dim3 grid(TASX_MAX_CTX * p->k), block(kSrvBlock);
  if (acq == 1)
    hipLaunchKernelGGL((flush_server_kernel<DIAG, 1>), grid, block, 0, s, *p);
  else if (acq == 2)
    hipLaunchKernelGGL((flush_server_kernel<DIAG, 2>), grid, block, 0, s, *p);
  else
    hipLaunchKernelGGL((flush_server_kernel<DIAG, 0>), grid, block, 0, s, *p);
}

extern "C" TASX_INTERNAL int ab_launch_server(const tasx_srv_params *p, void *stream)
{
  const char *e = getenv("TASX_SRV_ACQ");
  const int acq = e ? atoi(e) : 0;
  if (!p->diag && acq == 0)
    return TASX_EXT_PASS; // the product's form
  if (p->diag)
    launch_acq<true>(acq, p, (hipStream_t) stream);
  else
    launch_acq<false>(acq, p, (hipStream_t) stream);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
