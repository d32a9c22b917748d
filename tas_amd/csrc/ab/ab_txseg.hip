// ab/ab_txseg.hip -- A/B build only (libtasx_ab.so): the TX segment build's
// diagnostics forms (TASX_TXSEG_DEBUG, tools/txseg_probe.py, tools/txseg_ab.sh;
// profiles/r01_pmc_txseg, profiles/r03, profiles/r04) and the streaming
// ceilings bench.py prices kernels against (tasx_ab_stream_read,
// tasx_ab_stream_copy).  None of it is in the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "../tasx_kernels.h"
#include "../txseg_rows.h"

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
// The two load paths of a pure streaming read (round 4, VERDICT r03 item 1;
// tools/hbm_ceiling.hip, profiles/r04/INDEX.md r04a/r04b), the words folded by
// v_sad_u16 as the checksum kernels do:
//  register: 8 KiB per 256-thread block, two 16-byte non-temporal loads per
//   lane (the fastest register shape measured: 15.40 us per 98.3 MB launch)
//  LDS-DMA: global_load_lds_dwordx4 (nt) into a 4-slot ring of 1 KiB per
//   wave, 2 blocks per CU, counted vmcnt, ds_read_b128 + v_sad_u16
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

__device__ __forceinline__ void glds16_nt(const void *gsrc, uint32_t lds_addr)
{
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_addr) : "memory");
}

__global__ __launch_bounds__(256) void stream_read_glds_kernel(const u32x4 *src, uint64_t ngroups, uint32_t *sink)
{
  constexpr int D = 4;
  __shared__ u32x4 ring[4][D][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) &ring[wave][0][0]);
  const uint64_t W = (uint64_t) gridDim.x * 4u;
  const uint64_t g0 = (uint64_t) __builtin_amdgcn_readfirstlane((int) (blockIdx.x * 4u + (uint32_t) wave));
  const uint64_t n_it = g0 < ngroups ? (ngroups - g0 + W - 1u) / W : 0u;
  uint32_t acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if ((uint64_t) d < n_it)
      glds16_nt(src + (g0 + d * W) * 64u + lane, lbase + d * 1024u);
  uint64_t it = 0;
  for (; it + D < n_it; ++it) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
    const int slot = (int) (it % D);
    acc = sad4(ring[wave][slot][lane], acc);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    glds16_nt(src + (g0 + (it + D) * W) * 64u + lane, lbase + slot * 1024u);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (; it < n_it; ++it)
    acc = sad4(ring[wave][it % D][lane], acc);
  if (acc == 0x12345678u)
    sink[0] = acc;
}
} // namespace

extern "C" int tasx_ab_stream_read(const void *src, size_t bytes, int path, uint32_t *sink, void *stream)
{
  if (!src || !sink || (bytes & 1023) || ((uintptr_t) src & 15) || path < 0 || path > 13)
    return -22;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (path != 1) // 0: grid order; 2 + k: XCD runs of 2^k blocks (xcd_run)
    hipLaunchKernelGGL(stream_read_reg_kernel, dim3((uint32_t) ((bytes / 16 + 511) / 512)), dim3(256), 0,
                       (hipStream_t) stream, (const u32x4 *) src, bytes / 16, sink, path == 0 ? 0u : (uint32_t) path - 1u);
  else
    hipLaunchKernelGGL(stream_read_glds_kernel, dim3((uint32_t) cus * 2u), dim3(256), 0, (hipStream_t) stream,
                       (const u32x4 *) src, (uint64_t) (bytes / 1024), sink);
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

extern "C" TASX_INTERNAL int ab_launch_txseg(const tasx_txseg_params *p0, void *stream)
{
  // the diagnostics form is read at every launch (tests switch it per case)
  tasx_txseg_params q = *p0;
  const char *e = getenv("TASX_TXSEG_DEBUG");
  q.dbg = e ? (uint32_t) atoi(e) : 0u;
  const tasx_txseg_params *p = &q;
  constexpr uint64_t spb = kBlock / 16;
  const uint64_t blocks = ((uint64_t) p->n + spb - 1) / spb;
  const dim3 grid((uint32_t) blocks), block(kBlock);
  hipStream_t s = (hipStream_t) stream;
  const bool u_ok = p->l4_off + 18u + 15u <= 256u && p->ip_off + 12u + 15u <= 256u && p->shm_len >= 16u;
  const bool tas = p->ip_off == 14u && p->l4_off == 34u;
  if (!u_ok || p->dbg == 0u)
    return TASX_EXT_PASS;
  switch (p->dbg) {
  case 1: tasx_note_kernel("tx_segment_kernel<3>"); hipLaunchKernelGGL((tx_segment_kernel<3, 0>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;  // 3 slots per round
  case 2: tasx_note_kernel("tx_segment_kernel<nostore_full>"); hipLaunchKernelGGL((tx_segment_kernel<6, 1>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;  // no full-chunk stores
  case 3: tasx_note_kernel("tx_segment_kernel<nostore>"); hipLaunchKernelGGL((tx_segment_kernel<6, 25>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; // no stores at all
  case 4: tasx_note_kernel("tx_segment_kernel"); hipLaunchKernelGGL((tx_segment_kernel<6, 0>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;  // aligned-gather kernel
  case 5: tasx_note_kernel("tx_segment_u_kernel"); hipLaunchKernelGGL((tx_segment_u_kernel<6, true>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; // general layout
  case 6: tasx_note_kernel("tx_segment_tas_kernel<plain>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, false, 1, kTxHeaderFirst>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; // plain stores
  case 7: tasx_note_kernel("tx_segment_tas_kernel<wpe6>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 6, kTxHeaderFirst>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; // <= 80 VGPRs
  case 8: tasx_note_kernel("tx_segment_tas_kernel<wpe8>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 8, kTxHeaderFirst>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; // <= 64 VGPRs
  case 15: tasx_note_kernel("tx_segment_tas_kernel<line_keep>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxLineKeep>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 19: tasx_note_kernel("tx_segment_tas_kernel<block_writeback>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, 0>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 17: tasx_note_kernel("tx_segment_tas_kernel<simple>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxSimple>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 18: tasx_note_kernel("tx_segment_tas_kernel<simple,fields_only>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxSimple | kTxFieldsOnly>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 20: tasx_note_kernel("tx_segment_tas_kernel<shfl_tail>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxHeaderFirst>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 21: tasx_note_kernel("tx_segment_tas_kernel<shfl_tail,wpe5>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 5, kTxHeaderFirst>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 22: tasx_note_kernel("tx_segment_tas_kernel<wpe5>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 5>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  // 23-25: the product with residency capped by dynamic LDS (the kernel uses none):
  // 48 KiB -> 3 blocks per CU, 64 KiB -> 2, 40 KiB -> 3 (timing probes)
  case 23: tasx_note_kernel("tx_segment_tas_kernel<shfl_tail,lds48k>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxHeaderFirst>), grid, block, 48u << 10, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 24: tasx_note_kernel("tx_segment_tas_kernel<lds64k>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true>), grid, block, 64u << 10, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 25: tasx_note_kernel("tx_segment_tas_kernel<lds48k>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true>), grid, block, 48u << 10, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  // 26-28: timing-only ablations of the product (results wrong)
  case 26: tasx_note_kernel("tx_segment_tas_kernel<no_header_store>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxHeaderFirst | kTxDppTail | kTxNoHeaderStore>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 27: tasx_note_kernel("tx_segment_tas_kernel<no_fields>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxHeaderFirst | kTxDppTail | kTxNoFields>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 28: tasx_note_kernel("tx_segment_tas_kernel<no_sums>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxHeaderFirst | kTxDppTail | kTxNoSums>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 29: if (tas) { tasx_note_kernel("tx_segment_wave_kernel"); hipLaunchKernelGGL((tx_segment_wave_kernel<true>), dim3((uint32_t) ((p->n + 3u) / 4u)), block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  // 31: the product with 7 load slots (lanes own whole 128-byte source lines)
  case 31: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<slots7>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 7>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  // 32-34: timing-only ablations of the product: no fallback / no wraps / both
  case 32: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<nofb>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 1, 1>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  case 33: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<nowrap>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 1, 2>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  case 34: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<nofb,nowrap>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 1, 3>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  // 42 / 43: the access pattern alone (40) at 8 / 6 waves per SIMD (the pattern uses no LDS)
  case 42: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<pattern,wpe8>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 8, 8>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  case 43: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<pattern,wpe6>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 6, 8>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  case 40: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<pattern>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 1, 8>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  case 39: if (tas) { tasx_note_kernel("tx_segment_lds_kernel<nt_first>"); hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6, 1, 4>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  // 35-38: the product with residency capped by dynamic LDS at 5 / 4 / 3 / 2 blocks per CU
  case 35: case 36: case 37: case 38: if (tas) {
    constexpr uint32_t st = (kBlock / 16) * (uint32_t) lds_slice<6>(); // the kernel's static LDS
    static const uint32_t extra[4] = {163840u / 5u - st - 64u, 163840u / 4u - st - 64u, 163840u / 3u - st - 64u,
                                      163840u / 2u - st - 64u};
    static const char *const names[4] = {"tx_segment_lds_kernel<5blk>", "tx_segment_lds_kernel<4blk>", "tx_segment_lds_kernel<3blk>", "tx_segment_lds_kernel<2blk>"};
    tasx_note_kernel(names[p->dbg - 35]);
    hipLaunchKernelGGL((tx_segment_lds_kernel<true, 6>), grid, block, extra[p->dbg - 35], s, *p);
    return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  // 30: the round-2 product (unaligned non-temporal window loads, header-first, DPP tail)
  case 30: if (tas) { tasx_note_kernel("tx_segment_tas_kernel"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1; } break;
  case 16: tasx_note_kernel("tx_segment_tas_kernel<fields_only>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxFieldsOnly>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  // 9..14: ablations (timing only)
  case 9: tasx_note_kernel("tx_segment_tas_kernel<abl1>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxNoScratch>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 10: tasx_note_kernel("tx_segment_tas_kernel<abl2>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxNoWriteBack>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 11: tasx_note_kernel("tx_segment_tas_kernel<abl4>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxNoWindows>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 12: tasx_note_kernel("tx_segment_tas_kernel<abl8>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxNoFallback>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 13: tasx_note_kernel("tx_segment_tas_kernel<abl15>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, 15>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  case 14: tasx_note_kernel("tx_segment_tas_kernel<abl16>"); hipLaunchKernelGGL((tx_segment_tas_kernel<6, true, 1, kTxNoPayloadStores>), grid, block, 0, s, *p); return hipGetLastError() == hipSuccess ? 0 : -1;
  default: break;
  }
  return TASX_EXT_PASS;
}
