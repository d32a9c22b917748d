// ab/ab_txseg.hip -- comparison build only (libtasx_ab.so): the TX segment
// build's kept forms (tasx_ab_tx_segment_form: 30 = the round-2 product, run
// beside the product by tests/test_txseg.py; 40 = the product's access pattern
// alone, bench.py's pattern ceiling; ab_txseg_rows.h) and the streaming
// ceilings bench.py prices kernels against (tasx_ab_stream_read,
// tasx_ab_stream_copy).  None of it is in the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "../tasx_kernels.h"
#include "ab_txseg_rows.h"

// The device's read+write streaming rate for the TX segment build's ceiling
// (bench.py copy_ceiling): a grid-stride copy, one non-temporal 16-byte load
// and store per lane, grid of 4 blocks per CU (tools/copy_ceiling.hip: 6.2
// TB/s, against 5.2 for hipMemcpyAsync D2D).
namespace {
__global__ __launch_bounds__(256) void stream_copy_kernel(const u32x4 *src, u32x4 *dst, size_t nchunks)
{
  for (size_t c = (size_t) blockIdx.x * 256u + threadIdx.x; c < nchunks; c += (size_t) gridDim.x * 256u)
    __builtin_nontemporal_store(__builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4 *) (src + c)),
                                (__attribute__((address_space(1))) u32x4 *) (dst + c));
}
// A pure streaming read (round 4; profiles/r04/INDEX.md
// r04a/r04b), the words folded by v_sad_u16 as the checksum kernels do: 8 KiB
// per 256-thread block, two 16-byte non-temporal loads per lane (the fastest
// register shape measured: 15.40 us per 98.3 MB launch; LDS-DMA rings were
// slower at every size)
__global__ __launch_bounds__(256) void stream_read_reg_kernel(const u32x4 *src, size_t nchunks, uint32_t *sink,
                                                             uint32_t xrun)
{
  const size_t c0 = (size_t) xcd_run(blockIdx.x, gridDim.x, xrun) * 512u + threadIdx.x;
  u32x4 a = {0u, 0u, 0u, 0u}, b = a;
  if (c0 < nchunks)
    a = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4 *) (src + c0));
  if (c0 + 256u < nchunks)
    b = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4 *) (src + c0 + 256u));
  const uint32_t acc = sad4(b, sad4(a, 0u));
  if (acc == 0x12345678u)
    sink[0] = acc;
}

} // namespace

extern "C" int tasx_ab_stream_read(const void *src, size_t bytes, int path, uint32_t *sink, void *stream)
{
  // path 0: grid order; 2 + k: XCD runs of 2^k blocks (xcd_run)
  if (!src || !sink || (bytes & 1023) || ((uintptr_t) src & 15) || path < 0 || path == 1 || path > 13)
    return -22;
  hipLaunchKernelGGL(stream_read_reg_kernel, dim3((uint32_t) ((bytes / 16 + 511) / 512)), dim3(256), 0,
                     (hipStream_t) stream, (const u32x4 *) src, bytes / 16, sink, path == 0 ? 0u : (uint32_t) path - 1u);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int tasx_ab_stream_copy(const void *src, void *dst, size_t bytes, void *stream)
{
  if (!src || !dst || (bytes & 15) || ((uintptr_t) src & 15) || ((uintptr_t) dst & 15))
    return -22;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  hipLaunchKernelGGL(stream_copy_kernel, dim3((uint32_t) cus * 4u), dim3(256), 0, (hipStream_t) stream,
                     (const u32x4 *) src, (u32x4 *) dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The kept TX forms on a batch (the same arguments as
// tasx_tx_segment_batch_dev, TAS's layout only): form 30 = the round-2
// product, tx_segment_tas_kernel; form 40 = the product's access pattern
// alone (timing only: results wrong).
extern "C" int tasx_ab_tx_segment_form(int form, const void *shm, uint64_t shm_len, void *frames, const tasx_tx_seg *segs,
                                       uint32_t n, uint32_t ip_off, uint32_t l4_off, uint32_t *out, void *stream)
{
  if (n == 0)
    return 0;
  if (!shm || !frames || !segs || ((uintptr_t) segs & 15u) || ((uintptr_t) out & 3u) || ip_off != 14u || l4_off != 34u ||
      shm_len < 16u || shm_len > 0xffffffffull || (form != 30 && form != 40))
    return -22;
  tasx_txseg_params p = {};
  p.shm = (const uint8_t *) shm;
  p.shm_len = shm_len;
  p.frames = (uint8_t *) frames;
  p.segs = segs;
  p.out = out;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  constexpr uint64_t spb = kBlock / 16;
  const dim3 grid((uint32_t) (((uint64_t) n + spb - 1) / spb)), block(kBlock);
  hipStream_t s = (hipStream_t) stream;
  if (form == 30) { // unaligned non-temporal windows, header-first, DPP tail
    tasx_note_kernel("tx_segment_tas_kernel");
    hipLaunchKernelGGL((tx_segment_tas_kernel<6, true>), grid, block, 0, s, p);
  } else {
    tasx_note_kernel("tx_segment_lds_kernel<pattern>");
    hipLaunchKernelGGL((tx_segment_lds_ab_kernel<true, 6, 1, 8>), grid, block, 0, s, p);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
