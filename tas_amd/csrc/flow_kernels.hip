// flow_kernels.hip -- RX flow lookup for gfx950:
// the batch part of fast_flows_packet_fss()
// (/root/reference/tas/fast/fast_flows.c:1084-1163): per received frame, the
// CRC32C flow hash of its 4-tuple (flow_hash, :1078-1082) and the probe of
// FLEXNIC_PL_FLOWHT_NBSZ hash-table entries, each candidate confirmed against
// the 4-tuple in its flow state.
//
// Layout: one lane per frame.  The work is latency-bound random access (a
// dependent chain frame header -> bucket -> flow state), not bandwidth: every
// load of a phase is issued before any is used (the four bucket entries
// together, then the four candidates' keys together, clamped to flow 0 when
// not a candidate), and the kernel keeps few registers so many frames are in
// flight per CU.  CRC32C is computed bitwise on the VALU (96 steps, no table
// lookups in the chain).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"
#include "xsum_device.h"

namespace {

constexpr uint32_t kPoly = 0x82f63b78u; // CRC32C (Castagnoli), reflected

// SSE4.2 crc32 on one 32-bit little-endian word: crc32c_sse42_u32(w, crc)
__device__ __forceinline__ uint32_t crc32c_word(uint32_t crc, uint32_t w)
{
  crc ^= w;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    crc = (crc >> 1) ^ (kPoly & (0u - (crc & 1u)));
  return crc;
}

__device__ __forceinline__ uint32_t ld32b(const uint8_t *p)
{
  return ld8(p) | (ld8(p + 1) << 8) | (ld8(p + 2) << 16) | (ld8(p + 3) << 24);
}

__global__ __launch_bounds__(256) void flow_lookup_kernel(tasx_flow_params p)
{
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= p.n)
    return;
  const uint8_t *f = p.base + pkt_offset(p.off, p.stride, i);
  const uint8_t *ip = f + p.ip_off, *l4 = f + p.l4_off;
  // key = (local = destination, remote = source), network byte order
  const uint32_t lip = ld32b(ip + 16), rip = ld32b(ip + 12);
  const uint32_t ports = (ld8(l4 + 2) | (ld8(l4 + 3) << 8)) | ((ld8(l4) | (ld8(l4 + 1) << 8)) << 16);
  // flow_hash: crc32c_sse42_u32(ports, crc32c_sse42_u64(lip | rip << 32, 0))
  const uint32_t h = crc32c_word(crc32c_word(crc32c_word(0u, lip), rip), ports);
  // bucket: entries (h + j) % ht_entries, j < NBSZ
  uint32_t fid[TASX_FLOWHT_NBSZ], ehash[TASX_FLOWHT_NBSZ];
#pragma unroll
  for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j) {
    const uint32_t k = (h + j) % p.ht_entries;
    fid[j] = ldg(p.flowht, 2 * k);
    ehash[j] = ldg(p.flowht, 2 * k + 1);
  }
  // candidates' keys, all loads issued together
  bool cand[TASX_FLOWHT_NBSZ];
  uint32_t klip[TASX_FLOWHT_NBSZ], krip[TASX_FLOWHT_NBSZ], kport[TASX_FLOWHT_NBSZ];
#pragma unroll
  for (uint32_t j = 0; j < TASX_FLOWHT_NBSZ; ++j) {
    const uint32_t id = fid[j] & ((1u << TASX_FLOWHTE_POSSHIFT) - 1u);
    cand[j] = (fid[j] & TASX_FLOWHTE_VALID) && ehash[j] == h && id < p.fs_num;
    fid[j] = id;
    const uint32_t *key = (const uint32_t *) (p.flowst + (uint64_t) (cand[j] ? id : 0u) * p.fs_stride +
                                              p.fs_key_off);
    klip[j] = ldg(key, 0);
    krip[j] = ldg(key, 1);
    kport[j] = ldg(key, 2);
  }
  uint32_t res = TASX_FLOW_NONE;
#pragma unroll
  for (int j = (int) TASX_FLOWHT_NBSZ - 1; j >= 0; --j) // first match wins
    if (cand[j] && klip[j] == lip && krip[j] == rip && kport[j] == ports)
      res = fid[j];
  stg(p.fid_out, i, res);
  if (p.hash_out)
    stg(p.hash_out, i, h);
}

} // namespace

extern "C" int tasx_launch_flow_lookup(const tasx_flow_params *p, void *stream)
{
  const uint64_t blocks = ((uint64_t) p->n + 255) / 256;
  if (blocks == 0)
    return 0;
  hipLaunchKernelGGL(flow_lookup_kernel, dim3((uint32_t) blocks), dim3(256), 0, (hipStream_t) stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
