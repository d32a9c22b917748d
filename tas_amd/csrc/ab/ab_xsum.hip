// ab/ab_xsum.hip -- A/B build only (libtasx_ab.so): the checksum kernels'
// variants kept for comparisons (their numbers are in profiles/r01_*,
// profiles/r02-r05/INDEX.md; tools/sweep.py, tools/ackmix_probe.py,
// tools/rx_probe.py, tools/big_probe.py) and the access-pattern kernels
// bench.py prices the product against (tasx_ab_tcp4_pattern,
// tasx_ab_tcp4_mix_pattern).  Reached through the tasx_ext hooks
// (tasx_kernels.h); none of it is in the product library.  Variant numbers:
// include/tasx_ab.h.
#include "../xsum_rows.h"

namespace {

// ---------------------------------------------------------------------------
// First-generation kernels (variant 1, the A/B baseline): one G-lane group per
// packet, xor-shuffle reductions, byte loads for the TCP4 header.
// RAW: out[i] = rte_raw_cksum(base + off_i, len_i)   

template <int G, int U>
__global__ __launch_bounds__(kBlock) void raw_cksum_kernel(tasx_raw_params p)
{
  const int gl = threadIdx.x & (G - 1);
  const uint32_t gpb = kBlock / G;
  const uint32_t ngroups = gridDim.x * gpb;
  for (uint32_t i = blockIdx.x * gpb + threadIdx.x / G; i < p.n; i += ngroups) {
    const uint8_t *s = p.base + pkt_offset(p.off, p.stride, i);
    const uint32_t len = p.len ? ldg(p.len, i) : p.len0;
    uint32_t part = lane_partial<G, U>(s, len, gl);
    uint32_t tot = group_sum<G>(part);
    if (gl == 0) {
      uint32_t f = fold32_to_16(tot);
      if (((uintptr_t) s) & 1)
        f = bswap16(f);
      stg(p.out, i, (uint16_t) f);
    }
  }
}

// ---------------------------------------------------------------------------
// TCP4: per frame, tcp_checksums() flag-off branch:
//   ip.chksum  = rte_ipv4_cksum(ip)            (ip.chksum taken as 0)
//   tcp.chksum = rte_ipv4_udptcp_cksum(ip, l4) (tcp.chksum taken as 0)
// out[2i] = ip.chksum, out[2i+1] = tcp.chksum (native u16, as TAS stores them)

template <int G, int U>
__global__ __launch_bounds__(kBlock) void tcp4_cksum_kernel(tasx_tcp4_params p)
{
  static_assert(G >= 16, "header needs 11 lanes");
  const int gl = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1); // first lane of the group in the wave
  const uint32_t gpb = kBlock / G;
  const uint32_t ngroups = gridDim.x * gpb;

  for (uint32_t i = blockIdx.x * gpb + threadIdx.x / G; i < p.n; i += ngroups) {
    uint8_t *f = p.base + pkt_offset(p.off, p.stride, i);
    uint8_t *ip = f + p.ip_off;
    uint8_t *l4 = f + p.l4_off;

    // header words, relative to the header start: lanes 0..9 hold ip word gl
    uint32_t w = 0;
    if (gl < 10)
      w = ld8(ip + 2 * gl) | (ld8(ip + 2 * gl + 1) << 8);
    // total_length = bswap(word 1)
    const uint32_t w1 = (uint32_t) __shfl(w, gbase + 1, 64);
    const uint32_t tl = bswap16(w1);
    const uint32_t l4len = tl >= 20 ? tl - 20 : 0;

    // checksum field bytes of the L4 header, inside the summed range only
    uint32_t fix = 0;
    if (gl == 10 && l4len > 16) {
      uint32_t fw = ld8(l4 + 16);
      if (l4len > 17)
        fw |= ld8(l4 + 17) << 8;
      fix = (~fw) & 0xffffu; // -fw mod 0xffff, L4-start frame
    }

    // header channels: ip sum (words 0..9 but 5) and pseudo header
    // (src/dst words 6..9, proto<<8 from word 4)
    uint32_t c_ip = (gl < 10 && gl != 5) ? w : 0;
    uint32_t c_ph = (gl >= 6 && gl < 10) ? w : (gl == 4 ? (w & 0xff00u) : 0);

    uint32_t part = lane_partial<G, U>(l4, l4len, gl);

    c_ip = group_sum<G>(c_ip);
    c_ph = group_sum<G>(c_ph);
    part = group_sum<G>(part);
    fix = group_sum<G>(fix);

    if (gl == 0) {
      const uint32_t ipc = inv_result(residue(fold32_to_16(c_ip)));
      uint32_t tcpc = 0;
      if (tl >= 20) {
        uint32_t r4 = fold32_to_16(part);
        if (((uintptr_t) l4) & 1)
          r4 = bswap16(r4);
        const uint32_t lw = bswap16(l4len); // htons(l4len) as a LE word
        uint32_t s = r4 + fix + c_ph + lw;
        tcpc = inv_result(residue(fold32_to_16(s)));
      }
      if (p.out)
        stg((uint32_t *) p.out, i, ipc | (tcpc << 16));
      if (p.flags & TASX_F_INPLACE) {
        st8(ip + 10, ipc);
        st8(ip + 11, ipc >> 8);
        st8(l4 + 16, tcpc);
        st8(l4 + 17, tcpc >> 8);
      }
    }
  }
}

// RAW, any layout: out[i] = rte_raw_cksum(base + off_i, len_i)
template <int U>
__global__ __launch_bounds__(kBlock) void raw_group_kernel(tasx_raw_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t ngroups = gridDim.x * (kBlock / 16);
  uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  // descriptor prefetch (every lane of the group reads the same word)
  uint64_t off = 0;
  uint32_t len = p.len0;
  if (i < p.n) {
    off = pkt_offset(p.off, p.stride, i);
    if (p.len)
      len = ldg(p.len, i);
  }
  for (; i < p.n; i += ngroups) {
    const uint8_t *s = p.base + off;
    const Chunks<U> r = chunk_range<U>(s, len);
    const uint32_t inext = i + ngroups;
    uint32_t part = group_lane_sum<U>(r, gl);
    if (inext < p.n) {
      off = pkt_offset(p.off, p.stride, inext);
      if (p.len)
        len = ldg(p.len, inext);
    }
    part = row_sum16(part);
    if (gl == 15) {
      uint32_t f = fold32_to_16(part);
      if (r.head & 1)
        f = bswap16(f);
      stg(p.out, i, (uint16_t) f);
    }
  }
}

// TCP4 batches of mixed frame lengths with per-frame hints (a tx_flush batch:
// flow_tx_segment data frames among flow_tx_ack / inject_tcp_ts frames,
// fast_flows.c:877-1030).  One row per frame leaves the rows of short frames
// idle while the wave's longest frame is read; here a wave's 4 frames are one
// flattened chunk sequence, as in raw_wave_kernel: each datagram [ip, ip +
// hint - ip_off) is summed whole (exact 32-bit word sum; the IPv4 header is at
// an even address), then lane k takes frame k's header words off it:
//   L4 sum  = datagram sum - the 10 IPv4 header words - tcp.chksum as stored
//   IP sum  = the IPv4 header words - ip.chksum as stored
// (exact subtractions of words the datagram sum holds; tcp.chksum lies inside
// it because the hint covers ip + 40).  The header words are loaded up front,
// in flight with round 0.  A frame whose ip.total_length is not the hinted
// datagram length, whose hint does not cover ip + 40, or whose header sits at
// an odd address is redone by one 16-lane row (tcp4_frame_row): the results
// always follow ip.total_length, the hint only decides the reads.
// Measured (tools/ackmix_probe.py, profiles/r01_ackmix.jsonl): slower than
// tcp4_tas_kernel's row per frame at every ACK fraction (0 / 25 / 50 / 75 %:
// 18.0 / 15.9 / 14.9 / 14.0 us against 17.2 / 15.0 / 13.8 / 12.7 us for 64K
// frames).  These batches are bound by per-wave dependent latency (hint ->
// data -> store) over ~2.7 generations of resident waves, not by bytes, and
// the flattened pass adds VALU and registers (70 VGPRs against 55 for
// raw_wave_kernel) without removing a dependent step.  Kept as variant 8 (A/B).
template <int U>
__global__ __launch_bounds__(kBlock) void tcp4_wave_kernel(tasx_tcp4_params p)
{
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t i0 = xcd_run(blockIdx.x, gridDim.x, p.xrun) * (kBlock / 16) + (threadIdx.x >> 6) * 4u;
  if (i0 >= p.n) // wave-uniform
    return;
  const uint32_t i = i0 + (lane & 3u);
  uint64_t a = 0;
  uint32_t len = 0;
  if (lane < 8u && i < p.n) {
    const uint32_t h = p.flen ? ldg(p.flen, i) : p.flen0;
    const uint64_t ipa = (uint64_t) (uintptr_t) p.base + pkt_offset(p.off, p.stride, i) + p.ip_off;
    if (h >= p.ip_off + 40u && !(ipa & 1u)) {
      a = ipa;
      len = min(h - p.ip_off, 65535u);
    }
  }
  uint32_t w[10], wt = 0;
#pragma unroll
  for (int j = 0; j < 10; ++j)
    w[j] = 0;
  if (lane < 4u && len) {
    const uint16_t *ip16 = (const uint16_t *) (uintptr_t) a;
#pragma unroll
    for (int j = 0; j < 10; ++j)
      w[j] = ldg(ip16, (uint32_t) j);
    wt = ldg(ip16, 18u); // tcp.chksum: ip + 20 + 16 (l4_off == ip_off + 20)
  }
  const uint32_t s = wave4_sums<U>(lane, a, len);
  bool redo = false;
  if (lane < 4u && i < p.n) {
    const uint32_t tl = bswap16(w[1]);
    redo = len == 0u || tl != len;
    if (!redo) {
      uint32_t ipall = 0;
#pragma unroll
      for (int j = 0; j < 10; ++j)
        ipall += w[j];
      const uint32_t ph = w[6] + w[7] + w[8] + w[9] + (w[4] & 0xff00u); // src, dst, {0, proto}
      const uint32_t ipc = inv_result(residue(fold32_to_16(ipall - w[5])));
      const uint32_t r = fold32_to_16(s - ipall - wt) + fold32_to_16(ph) + bswap16(tl - 20u);
      const uint32_t tcpc = inv_result(residue(fold32_to_16(r)));
      if (p.out)
        stg((uint32_t *) p.out, i, ipc | (tcpc << 16));
      if (p.flags & TASX_F_INPLACE) {
        uint8_t *ip = (uint8_t *) (uintptr_t) a;
        st8(ip + 10, ipc);
        st8(ip + 11, ipc >> 8);
        st8(ip + 36, tcpc);
        st8(ip + 37, tcpc >> 8);
      }
    }
  }
  const uint64_t rb = __builtin_amdgcn_ballot_w64(redo);
  if (rb) { // row r (lanes 16r..16r+15) redoes frame i0 + r
    const uint32_t r = lane >> 4;
    if ((rb >> r) & 1ull)
      tcp4_frame_row<3>(p, i0 + r, (int) (lane & 15u)); // (3 per round: keeps the rare redo below the flattened pass's registers)
  }
}


// A whole short datagram (ip.len 38..66: a pure ACK, flow_tx_ack
// fast_flows.c:957-1030, is 52) in ONE lane: c[] = chunks 0..4 of the frame
// (IPv4 at a0 + 14, tcp4_tas14_kernel's chunk map), both results stored.
__device__ __forceinline__ void tas14_short_lane(const tasx_tcp4_params &p, uint32_t i, const uint8_t *fb, uint32_t a0,
                                                 uint32_t tl, const u32x4 (&c)[5])
{
  const uint32_t addrs = sadw(c[1].z & 0xffff0000u, sadw(c[1].w, sadw(c[2].x & 0xffffu, 0u))); // src, dst
  const uint32_t ph = sadw(c[1].y & 0xff000000u, addrs);                                      // + proto
  const uint32_t ipsum = sadw(c[0].w & 0xffff0000u, sadw(c[1].x, sadw(c[1].y, addrs)));      // ip.chksum left out
  // L4 = frame bytes [34, 14 + tl): chunk 2 from byte 2, chunk 3 without
  // tcp.chksum (its bytes 2..3), chunk 4 up to the datagram's end
  const int end = 14 + (int) tl; // 52..80
  u32x4 c3 = mask_chunk(c[3], 0, min(end - 48, 16));
  c3.x &= 0x0000ffffu;
  uint32_t l4 = sad4(mask_chunk(c[2], 2, 16), 0u);
  l4 = sad4(c3, l4);
  l4 = sad4(mask_chunk(c[4], 0, max(end - 64, 0)), l4);
  const uint32_t ipc = inv_result(residue(fold32_to_16(ipsum)));
  const uint32_t r = fold32_to_16(l4) + fold32_to_16(ph) + bswap16(tl - 20u);
  const uint32_t tcpc = inv_result(residue(fold32_to_16(r)));
  if (p.out)
    stg((uint32_t *) p.out, i, ipc | (tcpc << 16));
  if (p.flags & TASX_F_INPLACE) {
    uint8_t *ip = (uint8_t *) fb + a0 + 14u;
    st8(ip + 10, ipc);
    st8(ip + 11, ipc >> 8);
    st8(ip + 36, tcpc);
    st8(ip + 37, tcpc >> 8);
  }
}

// tcp4_mix_kernel: TX batches that mix data segments and pure ACKs (what
// tx_flush sends: flow_tx_segment's ~1.5 KB frames and flow_tx_ack's 66 B
// frames, fastemu.c:544-566), TAS frames in stride mode, a room of >= 80 B.
// One wave takes 16 frames.  Phase 1: lane l < 16 loads chunks 0..4 of frame
// 16w + l (a whole ACK) and classifies the frame by its own total_length:
// short (38..66: finished by that lane alone, one memory latency), data
// (67..1522) or other (the general body, tcp4_tas_frame).  Phase 2: the data
// frames, compacted by a forward lane permute, go 4 per pass to the wave's
// 16-lane rows, and every pass's loads are in flight before the first is
// summed (tcp4_tas14_kernel's row body).  kTlFirst spends a 16-lane row and
// a second dependent latency on every ACK, and needs two generations of
// resident waves for 64K frames; here an ACK costs one lane and the 64K-frame
// batch fits one generation (4 waves per SIMD x 16 frames).
// A/B only (variant 19; TASX_MIX_F8=1: 8 frames per wave): bit-exact, but
// slower than kTlFirst wherever data frames are present (64K frames in 2048 B
// rooms, 0 / 50 / 100 % ACKs: 19.5-20.2 / 12.6-12.9 / 6.5-6.6 us with 16
// frames per wave, 18.7 / 12.2-12.3 / 6.1 us with 8, against 16.9-17.3 /
// 10.7-10.9 / 6.9 us; profiles/r02/r02m, r02n): a wave issues its data only
// after the slowest of its frames' phase-1 loads, a kTlFirst row as soon as
// its own total_length lands.
template <int U, int F = 16>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(F == 16 ? 4 : 6))) void tcp4_mix_kernel(tasx_tcp4_params p)
{
  static_assert(U == 6, "96 chunks cover the 1522-byte datagram bound");
  static_assert(F == 8 || F == 16, "frames per wave: 2 or 4 passes of 4 rows");
  constexpr int NP = F / 4;
  const int lane = (int) (threadIdx.x & 63u), gl = lane & 15, row = lane >> 4;
  const uint32_t w0 = (blockIdx.x * (kBlock / 64) + threadIdx.x / 64) * (uint32_t) F; // the wave's first frame
  if (w0 >= p.n)
    return; // the whole wave leaves together
  const uint8_t *fb = p.base; // loads at fb + 32-bit offsets (tas14_stride_ok)
  const uint32_t ipa = p.ip_off & ~15u, nf = min(p.n - w0, (uint32_t) F);
  const uint32_t st = (uint32_t) p.stride;

  // phase 1: frame w0 + lane on lanes 0..15
  const bool mine = lane < 16 && (uint32_t) lane < nf;
  const uint32_t a0 = (w0 + (uint32_t) gl) * st + ipa;
  u32x4 c[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)
    c[k] = u32x4{0u, 0u, 0u, 0u};
  if (mine) {
#pragma unroll
    for (int k = 0; k < 5; ++k)
      c[k] = ld16nt_off(fb, a0 + 16u * (uint32_t) k);
  }
  const uint32_t tl = bswap16(c[1].x & 0xffffu);
  const bool shortf = mine && tl >= 38u && tl <= 66u;
  const bool data = mine && tl > 66u && tl <= 1522u;
  const bool other = mine && !shortf && !data;
  const uint64_t dm = __builtin_amdgcn_ballot_w64(data), om = __builtin_amdgcn_ballot_w64(other);
  // compaction: data frame of rank r -> lane r, other frame of rank r -> lane
  // 32 + r (everything else lands in lanes 16..31 / 48..63, never read)
  const uint32_t below = (1u << (lane & 31)) - 1u; // lanes < 16 only matter
  const uint32_t rd = (uint32_t) __builtin_popcount((uint32_t) dm & below);
  const uint32_t ro = (uint32_t) __builtin_popcount((uint32_t) om & below);
  const int dst = data ? (int) rd : other ? 32 + (int) ro : lane < 16 ? 48 + lane : 16 + (lane & 15);
  const uint32_t pk = (uint32_t) __builtin_amdgcn_ds_permute(dst * 4, (int) ((uint32_t) gl | (tl << 8)));
  if (shortf)
    tas14_short_lane(p, w0 + (uint32_t) gl, fb, a0, tl, c);

  // phase 2: data frames 4 per pass, all passes' loads issued first.  The
  // loads are unconditional (an idle row reads the wave's first frame's
  // chunk 1, a line phase 1 just fetched) so that the waits before each pass
  // count exactly the loads ahead of it: under a branch the compiler must wait
  // for all of them before the first pass.
  const uint32_t nd = (uint32_t) __builtin_popcountll(dm);
  u32x4 v[NP][U];
  uint32_t q[NP];
#pragma unroll
  for (int ps = 0; ps < NP; ++ps) {
    q[ps] = (uint32_t) __shfl((int) pk, 4 * ps + row, 64);
    const bool act = 4u * ps + (uint32_t) row < nd;
    const uint32_t hend = act ? q[ps] >> 8 : 20u;
    const uint32_t r0 = (w0 + (act ? (q[ps] & 15u) : 0u)) * st + ipa;
    const uint32_t lastoff = r0 + 16u * ((14u + hend - 1u) >> 4), lo = r0 + 16u * (uint32_t) gl;
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[ps][u] = ld16nt_off(fb, min(lo + 256u * u, lastoff));
  }
#pragma unroll
  for (int ps = 0; ps < NP; ++ps) {
    if (nd > 4u * ps && 4u * ps + (uint32_t) row < nd) {
      const uint32_t r0 = (w0 + (q[ps] & 15u)) * st + ipa;
      tas14_finish<U, kTlFirst, false, false, false>(p, w0 + (q[ps] & 15u), gl, fb, r0, q[ps] >> 8, true, v[ps]);
    }
  }

  // other frames (total_length outside 38..1522): the general body, 4 per pass
  const uint32_t no = (uint32_t) __builtin_popcountll(om);
  for (uint32_t o = 0; o < no; o += 4u) {
    const uint32_t qo = (uint32_t) __shfl((int) pk, 32 + (int) o + row, 64);
    if (o + (uint32_t) row < no)
      tcp4_tas_frame<U, 0, 16, false>(p, w0 + (qo & 15u), gl, lane & ~15);
  }
}

template <typename K, typename P>
int launch(const char *name, K kern, const P &p, uint32_t groups_per_block, int max_blocks, hipStream_t s)
{
  uint64_t blocks = ((uint64_t) p.n + groups_per_block - 1) / groups_per_block;
  if (blocks > (uint64_t) max_blocks)
    blocks = (uint64_t) max_blocks;
  if (blocks == 0)
    return 0;
  tasx_note_kernel(name);
  hipLaunchKernelGGL(kern, dim3((uint32_t) blocks), dim3(kBlock), 0, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// residency knobs (KiB of reserved LDS) for A/B runs
uint32_t env_lds(const char *name, uint32_t dflt)
{
  const char *e = getenv(name);
  return e ? (uint32_t) atoi(e) * 1024u : dflt;
}

// persistent grids: blocks resident at once on the current device (8 waves of
// 64 VGPRs per SIMD = 8 blocks of 256 threads per CU)
uint32_t resident_blocks()
{
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return (uint32_t) cus * 8u;
}

template <typename K>
int launch_rows(const char *name, K kern, const tasx_tcp4_params &p, uint32_t frames_per_row, hipStream_t s)
{
  const uint64_t need = ((uint64_t) p.n + 16u * frames_per_row - 1) / (16u * frames_per_row);
  uint64_t blocks = frames_per_row ? need : resident_blocks();
  if (!frames_per_row && blocks > ((uint64_t) p.n + 15u) / 16u)
    blocks = ((uint64_t) p.n + 15u) / 16u;
  if (blocks == 0)
    return 0;
  tasx_note_kernel(name);
  hipLaunchKernelGGL(kern, dim3((uint32_t) blocks), dim3(kBlock), 0, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the row modes only A/B variants force (kHead5 goes through the product's
// launch_tas14_rows)
template <bool OFFS>
int launch_ab_rows(const tasx_tcp4_params &p, int mode, hipStream_t s)
{
  const uint32_t lds = env_lds("TASX_TAS14_NOHINT_LDS", 0u);
  switch (mode) {
  case kHintArrP:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<hints_pred,offs>" : "tcp4_tas14_kernel<hints_pred>",
                         tcp4_tas14_kernel<6, kHintArrP, false, 8, OFFS>, p, s, lds);
  case kHintArrS:
    return launch_groups(OFFS ? "tcp4_tas14_kernel<hints_sorted,offs>" : "tcp4_tas14_kernel<hints_sorted>",
                         tcp4_tas14_kernel<6, kHintArrS, false, 8, OFFS>, p, s, lds);
  case kMix:
    if (OFFS) // the mix kernel is a stride-mode form
      return launch_tas14_rows<OFFS>(p, kTlFirst, s);
    if (getenv("TASX_MIX_F8"))
      return launch_groups<8>("tcp4_mix_kernel<f8>", tcp4_mix_kernel<6, 8>, p, s);
    return launch_groups<4>("tcp4_mix_kernel", tcp4_mix_kernel<6>, p, s);
  default:
    return launch_tas14_rows<OFFS>(p, mode, s);
  }
}

} // namespace

// The headline kernel's access pattern with no checksum logic: the same rows,
// the same 6 clamped chunk loads per lane at 32-bit offsets from the SGPR
// base, the same 4-byte result store per frame and LDS reservation; the
// loaded words are only xor-folded.  bench.py times it beside the headline
// (its pattern_ceiling).
namespace {
__global__ __launch_bounds__(kBlock) void tcp4_pattern_kernel(tasx_tcp4_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return;
  const uint32_t a0 = i * (uint32_t) p.stride + (p.ip_off & ~15u), hend = p.flen0 - p.ip_off;
  const uint32_t lastoff = a0 + 16u * ((14u + hend - 1u) >> 4), lo = a0 + 16u * (uint32_t) gl;
  u32x4 v[6];
#pragma unroll
  for (int u = 0; u < 6; ++u)
    v[u] = ld16nt_off(p.base, min(lo + 256u * u, lastoff));
  uint32_t x = 0;
#pragma unroll
  for (int u = 0; u < 6; ++u)
    x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  x = row_sum16(x);
  if (gl == 15)
    stg((uint32_t *) p.out, i, x);
}

// The data/ACK mix's access pattern (tcp4_tas14_kernel<hints>, the flush_mix
// leg) with no checksum logic, for its latency roofline (bench.py
// mix_bounds): each row reads its hint, then (CHAIN = 0) the same clamped
// chunk loads as the product, xor-folded, or (CHAIN = 1) only the chunk
// holding the frame's end on lane 15 -- the row's dependent chain (hint ->
// frame -> result store) with almost no bytes behind it; 8 waves per SIMD as
// the product.
template <int CHAIN>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void tcp4_mix_pattern_kernel(tasx_tcp4_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if constexpr (CHAIN == 2) {
    // two frames per row, i and i + n / 2 (rounded up): both hints, then both
    // frames' chunk loads, one generation of resident rows for 64K frames
    const uint32_t half = (p.n + 1u) / 2u;
    if (i >= half)
      return;
    const uint32_t i2 = min(i + half, p.n - 1u);
    const uint32_t h1 = ldg(p.flen, i), h2 = ldg(p.flen, i2);
    uint32_t x1 = 0, x2 = 0;
    u32x4 v1[6], v2[6];
    {
      const uint32_t a1 = i * (uint32_t) p.stride + (p.ip_off & ~15u), a2 = i2 * (uint32_t) p.stride + (p.ip_off & ~15u);
      const uint32_t hl1 = h1 > p.ip_off + 20u ? min(h1 - p.ip_off, 1522u) : 20u;
      const uint32_t hl2 = h2 > p.ip_off + 20u ? min(h2 - p.ip_off, 1522u) : 20u;
      const uint32_t l1 = a1 + 16u * ((14u + hl1 - 1u) >> 4), l2 = a2 + 16u * ((14u + hl2 - 1u) >> 4);
#pragma unroll
      for (int u = 0; u < 6; ++u)
        v1[u] = ld16nt_off(p.base, min(a1 + 16u * (uint32_t) gl + 256u * u, l1));
#pragma unroll
      for (int u = 0; u < 6; ++u)
        v2[u] = ld16nt_off(p.base, min(a2 + 16u * (uint32_t) gl + 256u * u, l2));
    }
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      x1 ^= v1[u].x ^ v1[u].y ^ v1[u].z ^ v1[u].w;
      x2 ^= v2[u].x ^ v2[u].y ^ v2[u].z ^ v2[u].w;
    }
    x1 = row_sum16(x1);
    x2 = row_sum16(x2);
    if (gl == 15) {
      stg((uint32_t *) p.out, i, x1);
      if (i + half < p.n)
        stg((uint32_t *) p.out, i2, x2);
    }
    return;
  }
  if (i >= p.n)
    return;
  const uint32_t a0 = i * (uint32_t) p.stride + (p.ip_off & ~15u);
  const uint32_t h = ldg(p.flen, i);
  const uint32_t hl = h > p.ip_off + 20u ? min(h - p.ip_off, 1522u) : 20u;
  const uint32_t lastoff = a0 + 16u * ((14u + hl - 1u) >> 4), lo = a0 + 16u * (uint32_t) gl;
  uint32_t x = 0;
  if constexpr (CHAIN) {
    if (gl == 15) {
      const u32x4 t = ld16nt_off(p.base, lastoff);
      x = t.x ^ t.y ^ t.z ^ t.w;
    }
  } else {
    u32x4 v[6];
#pragma unroll
    for (int u = 0; u < 6; ++u)
      v[u] = ld16nt_off(p.base, min(lo + 256u * u, lastoff));
#pragma unroll
    for (int u = 0; u < 6; ++u)
      x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  x = row_sum16(x);
  if (gl == 15)
    stg((uint32_t *) p.out, i, x);
}
} // namespace

extern "C" int tasx_ab_tcp4_mix_pattern(const void *base, uint64_t stride, uint32_t n, const uint32_t *flen,
                                        uint32_t ip_off, int chain, uint32_t *out, void *stream)
{
  tasx_tcp4_params p;
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.stride = stride;
  p.n = n;
  p.flen = flen;
  p.ip_off = ip_off;
  p.l4_off = ip_off + 20u;
  p.out = (uint16_t *) out;
  // the product's own geometry checks: 16-byte aligned rooms of at least 1536 bytes, 32-bit offsets
  if (!out || !flen || !base || (ip_off & 15u) != 14u || (stride & 15u) || stride < 1536u ||
      (uint64_t) n * stride > 0xffffffffull || ((uintptr_t) base & 15u))
    return -EINVAL;
  if (chain == 2) { // two frames per row: half the rows
    tasx_tcp4_params q = p;
    q.n = (n + 1u) / 2u;
    const uint64_t blocks = ((uint64_t) q.n + kBlock / 16 - 1) / (kBlock / 16);
    if (blocks == 0)
      return 0;
    tasx_note_kernel("tcp4_mix_pattern_kernel<pair>");
    hipLaunchKernelGGL(tcp4_mix_pattern_kernel<2>, dim3((uint32_t) blocks), dim3(kBlock), 0, (hipStream_t) stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  return chain ? launch_groups("tcp4_mix_pattern_kernel<chain>", tcp4_mix_pattern_kernel<1>, p, (hipStream_t) stream, 0u)
               : launch_groups("tcp4_mix_pattern_kernel", tcp4_mix_pattern_kernel<0>, p, (hipStream_t) stream, 0u);
}

extern "C" int tasx_ab_tcp4_pattern(const void *base, uint64_t stride, uint32_t n, uint32_t flen0, uint32_t ip_off,
                                    uint32_t *out, void *stream)
{
  tasx_tcp4_params p;
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.stride = stride;
  p.n = n;
  p.flen0 = flen0;
  p.ip_off = ip_off;
  p.l4_off = ip_off + 20u;
  p.out = (uint16_t *) out;
  if (!out || !tas14_ok(p))
    return -EINVAL;
  return launch_groups("tcp4_pattern_kernel", tcp4_pattern_kernel, p, (hipStream_t) stream, kOccLds);
}

// ---------------------------------------------------------------------------
// the variants (TASX_EXT_PASS: not one of them, the product path runs)

static int g_xrun_ov = -2;
// the xrun of every grid (0 = grid order; -1 = the product's rule), from
// tasx_ab_set_xrun or TASX_XRUN
extern "C" int tasx_ab_set_xrun(int xrun)
{
  if (xrun < -1 || xrun > 20)
    return -22;
  g_xrun_ov = xrun;
  return 0;
}

extern "C" TASX_INTERNAL int ab_xrun(uint64_t blocks)
{
  (void) blocks;
  if (g_xrun_ov == -2) {
    const char *e = getenv("TASX_XRUN");
    g_xrun_ov = e ? atoi(e) : -1;
  }
  return g_xrun_ov;
}

extern "C" TASX_INTERNAL int ab_launch_raw(const tasx_raw_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  switch (variant) {
  case 1:
    return launch("raw_cksum_kernel", raw_cksum_kernel<16, 8>, *p, kBlock / 16, 256 * 64, s);
  case 2:
    return launch_groups("raw_group_kernel", raw_group_kernel<6>, *p, s);
  // round 4 (stride mode from a 16-byte aligned base, else automatic): 45 / 46
  // = 32 / 64 lanes per packet with 3 / 2 loads per lane, no residency cap; 47 =
  // the product's 16-lane rows without the cap; 48 = 32 lanes with the cap
  case 45: case 46: case 47: case 48:
    if (p->off == nullptr && ((uintptr_t) p->base & 15u) == 0 &&
        (uint64_t) (kBlock / 16) * p->stride + TASX_RAW_MAX_LEN + 16u < (1ull << 32)) {
      switch (variant) {
      case 45: return launch_groups<32>("raw_sad_kernel<s32,g32>", raw_sad_kernel<3, true, 32>, *p, s, 0u);
      case 46: return launch_groups<64>("raw_sad_kernel<s32,g64>", raw_sad_kernel<2, true, 64>, *p, s, 0u);
      case 47: return launch_groups("raw_sad_kernel<s32,nocap>", raw_sad_kernel<6, true>, *p, s, 0u);
      default: return launch_groups<32>("raw_sad_kernel<s32,g32,cap>", raw_sad_kernel<3, true, 32>, *p, s, kOccLds);
      }
    }
    return TASX_EXT_PASS;
  default:
    return TASX_EXT_PASS;
  }
}

extern "C" TASX_INTERNAL int ab_launch_tcp4(const tasx_tcp4_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  const bool rows = !tas14_ok(*p) && (tas14_nohint_ok(*p) || tas14_offs_ok(*p));
  // 9 / 10 / 11 / 19 / 20 / 21 / 28: force the total_length-first / head-5 /
  // whole-room / mix / per-frame-hint / predicated-hint / sorted-hint row mode
  // where its room requirement holds (else the product's choice)
  if ((variant >= 9 && variant <= 11) || (variant >= 19 && variant <= 21) || variant == 28) {
    const uint32_t from_a0 = p->room > (p->ip_off & ~15u) ? p->room - (p->ip_off & ~15u) : 0u;
    const int m = variant == 9 ? kTlFirst : variant == 10 ? kHead5 : variant == 11 ? kRoom : variant == 19 ? kMix
                : variant == 20 ? kHintArr : variant == 28 ? kHintArrS : kHintArrP;
    if (!rows || !((m == kTlFirst) || ((m == kHintArr || m == kHintArrP || m == kHintArrS) && p->flen) ||
                   ((m == kHead5 || m == kMix) && from_a0 >= 80u) || (m == kRoom && from_a0 >= 1536u)))
      return TASX_EXT_PASS;
    return p->off ? launch_ab_rows<true>(*p, m, s) : launch_ab_rows<false>(*p, m, s);
  }
  // 12 / 13 / 14: the persistent total_length-first rows (resident grid / 2 /
  // 4 frames per row) where tcp4_tas14_kernel's stride form applies
  // 15 / 16 / 17 / 18: tcp4_tas14_kernel<tl_first> (stride mode) in blocks of
  // 64 / 128 / 512 / 1024 threads instead of 256
  // 22 / 23 / 24 / 25: tcp4_tas14_kernel<hints> (stride mode, per-frame hints)
  // in blocks of 64 / 128 / 512 / 1024 threads
  // 43 / 44: the whole-room / total_length-first rows with the headline's
  // residency (no waves-per-EU floor, the 30 KiB LDS cap) instead of 8 waves per SIMD
  if ((variant == 43 || variant == 44) && !p->flen && !tas14_ok(*p) && tas14_nohint_ok(*p)) {
    const uint32_t from_a0 = p->room > (p->ip_off & ~15u) ? p->room - (p->ip_off & ~15u) : 0u;
    if (variant == 43 && from_a0 >= 1536u)
      return launch_groups("tcp4_tas14_kernel<room,occ>", tcp4_tas14_kernel<6, kRoom, false, 1>, *p, s, kOccLds);
    if (variant == 44)
      return launch_groups("tcp4_tas14_kernel<tl_first,occ>", tcp4_tas14_kernel<6, kTlFirst, false, 1>, *p, s, kOccLds);
  }
  const uint32_t nlds = env_lds("TASX_TAS14_NOHINT_LDS", 0u);
  if (variant == 42 && p->flen && !tas14_ok(*p) && (tas14_nohint_ok(*p) || tas14_offs_ok(*p))) // hints, line-paired generations
    return p->off ? launch_groups("tcp4_tas14_kernel<hints,offs,linepair>",
                                  tcp4_tas14_kernel<6, kHintArr, false, 8, true, kBlock, false, kFlowNone, kLinePair>, *p, s, nlds)
                  : launch_groups("tcp4_tas14_kernel<hints,linepair>",
                                  tcp4_tas14_kernel<6, kHintArr, false, 8, false, kBlock, false, kFlowNone, kLinePair>, *p, s, nlds);
  if (variant == 38 && p->flen && !p->off && !tas14_ok(*p) && tas14_nohint_ok(*p)) // hints, the row-body fallback
    return launch_groups("tcp4_tas14_kernel<hints,rowfb>",
                         tcp4_tas14_kernel<6, kHintArr, false, 8, false, kBlock, false, kFlowNone, kRowFallback>, *p, s, nlds);
  if (variant == 37 && p->flen && !p->off && !tas14_ok(*p) && tas14_nohint_ok(*p)) // hints, next generation's hint lines prefetched
    return launch_groups("tcp4_tas14_kernel<hints,prefetch>",
                         tcp4_tas14_kernel<6, kHintArr, false, 8, false, kBlock, false, kFlowNone, kHintPrefetch>, *p, s, nlds);
  if (variant >= 22 && variant <= 25 && p->flen && tas14_nohint_ok(*p)) {
    switch (variant) {
    case 22: return launch_groups<16, 64>("tcp4_tas14_kernel<hints,bs64>", tcp4_tas14_kernel<6, kHintArr, false, 8, false, 64>, *p, s);
    case 23: return launch_groups<16, 128>("tcp4_tas14_kernel<hints,bs128>", tcp4_tas14_kernel<6, kHintArr, false, 8, false, 128>, *p, s);
    case 24: return launch_groups<16, 512>("tcp4_tas14_kernel<hints,bs512>", tcp4_tas14_kernel<6, kHintArr, false, 8, false, 512>, *p, s);
    default: return launch_groups<16, 1024>("tcp4_tas14_kernel<hints,bs1024>", tcp4_tas14_kernel<6, kHintArr, false, 8, false, 1024>, *p, s);
    }
  }
  if (variant >= 15 && variant <= 18 && !tas14_ok(*p) && tas14_nohint_ok(*p)) {
    switch (variant) {
    case 15: return launch_groups<16, 64>("tcp4_tas14_kernel<tl_first,bs64>", tcp4_tas14_kernel<6, kTlFirst, false, 8, false, 64>, *p, s);
    case 16: return launch_groups<16, 128>("tcp4_tas14_kernel<tl_first,bs128>", tcp4_tas14_kernel<6, kTlFirst, false, 8, false, 128>, *p, s);
    case 17: return launch_groups<16, 512>("tcp4_tas14_kernel<tl_first,bs512>", tcp4_tas14_kernel<6, kTlFirst, false, 8, false, 512>, *p, s);
    default: return launch_groups<16, 1024>("tcp4_tas14_kernel<tl_first,bs1024>", tcp4_tas14_kernel<6, kTlFirst, false, 8, false, 1024>, *p, s);
    }
  }
  if (variant >= 12 && variant <= 14 && !tas14_ok(*p) && tas14_nohint_ok(*p))
    return launch_rows("tcp4_tas14_rows_kernel", tcp4_tas14_rows_kernel<6>, *p,
                       variant == 12 ? 0u : variant == 13 ? 2u : 4u, s);
  if (variant == 8 && p->l4_off == p->ip_off + 20u) {
    static const uint32_t lds = env_lds("TASX_WAVE_TCP4_LDS", 0u);
    return launch_groups("tcp4_wave_kernel", tcp4_wave_kernel<TASX_WAVE_U>, *p, s, lds);
  }
  switch (variant) {
  case 1:
    return launch("tcp4_cksum_kernel", tcp4_cksum_kernel<16, 8>, *p, kBlock / 16, 256 * 64, s);
  case 4:
    return p->diag && tas_kernel_ok(*p) ? launch_groups("tcp4_tas_kernel<diag>", tcp4_tas_kernel<6, 1>, *p, s) : -2;
  case 5: // 32-lane groups (slower than 16, profiles/r01_variant_sweeps.jsonl)
    if (tas_kernel_ok(*p))
      return launch_groups<32>("tcp4_tas_kernel<g32>", tcp4_tas_kernel<3, 0, 32>, *p, s);
    break;
  default:
    break;
  }
  return TASX_EXT_PASS;
}

extern "C" TASX_INTERNAL int ab_launch_verify(const tasx_tcp4_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  if (tas14_ok(*p) || !(tas14_nohint_ok(*p) || tas14_offs_ok(*p)))
    return TASX_EXT_PASS;
  const int mode = p->flen ? kHintArr : kTlFirst;
  const uint32_t lds = env_lds("TASX_TAS14_VERIFY_LDS", 0u);
  if (variant == 9) // total_length first whatever the call carries
    return p->off ? launch_tas14_verify<true>(*p, kTlFirst, s) : launch_tas14_verify<false>(*p, kTlFirst, s);
  if (variant == 42 && mode == kHintArr && !p->off) // line-paired generations
    return launch_groups("tcp4_tas14_kernel<hints,verify,linepair>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowNone, kLinePair>, *p, s, lds);
  if (variant == 38 && mode == kHintArr && !p->off) // the row-body fallback
    return launch_groups("tcp4_tas14_kernel<hints,verify,rowfb>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowNone, kRowFallback>, *p, s, lds);
  if (variant == 37 && mode == kHintArr && !p->off) // next generation's hint lines prefetched
    return launch_groups("tcp4_tas14_kernel<hints,verify,prefetch>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowNone, kHintPrefetch>, *p, s, lds);
  return TASX_EXT_PASS;
}

template <bool OFFS>
static int ab_rx_rows(const tasx_tcp4_params &p, int mode, hipStream_t s, int variant)
{
  const uint32_t lds = env_lds("TASX_TAS14_VERIFY_LDS", 0u);
  if (variant == 26) // the lookup inside the rows
    return mode == kHintArr ? launch_rx_rows<OFFS, kHintArr, kFlowRow>(p, s, lds)
                            : launch_rx_rows<OFFS, kTlFirst, kFlowRow>(p, s, lds);
  if (variant == 27) // two frames per lookup lane, lookup blocks over consecutive frames
    return mode == kHintArr ? launch_rx_rows<OFFS, kHintArr, kFlowSplit>(p, s, lds)
                            : launch_rx_rows<OFFS, kTlFirst, kFlowSplit>(p, s, lds);
  if (variant == 35) // XCD-matched lookup blocks with two frames per lane
    return mode == kHintArr ? launch_rx_rows<OFFS, kHintArr, kFlowSplitX2>(p, s, lds)
                            : launch_rx_rows<OFFS, kTlFirst, kFlowSplitX2>(p, s, lds);
  if (variant == 36) // the round-2 product (one frame per lane, lookup blocks over consecutive frames)
    return mode == kHintArr ? launch_rx_rows<OFFS, kHintArr, kFlowSplit1>(p, s, lds)
                            : launch_rx_rows<OFFS, kTlFirst, kFlowSplit1>(p, s, lds);
  if (mode != kHintArr || OFFS)
    return TASX_EXT_PASS;
  switch (variant) {
  case 43: // the product with non-temporal flow-state key loads
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,fsnt>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, 1024>, p, s, lds);
  case 42: // the product with line-paired generations
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,linepair>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, kLinePair>, p, s, lds);
  case 41: // the product with the lookup waves at issue priority 3
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,prio>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, kLookupPrio>, p, s, lds);
  case 40: // timing: the product's verify blocks alone (results wrong)
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,verify_only>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, kVerifyOnly>, p, s, lds);
  case 39: // timing: the product's lookup blocks alone (results wrong)
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,lookup_only>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, kLookupOnly>, p, s, lds);
  case 38: // the product with the row-body fallback
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,rowfb>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, kRowFallback>, p, s, lds);
  case 37: // the product with the next generation's hint lines prefetched
    return launch_splitx("tcp4_tas14_kernel<hints,verify,flow,prefetch>",
                         tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplitX, kHintPrefetch>, p, s, lds);
  case 28: // lookup blocks after their verify blocks, same XCD
    return launch_inter("tcp4_tas14_kernel<hints,verify,flow_inter>",
                        tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowInter>, p, s, lds);
  // timing-only ablations of the round-2 product's lookup blocks (results
  // wrong): 29 no frame key load, 30 no CRC, 31 no flow-state key load, 33 no
  // bucket loads, 34 the frame key only
  case 33:
    return launch_split<1>("tcp4_tas14_kernel<hints,verify,flow,nobucket>",
                           tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplit1, 8>, p, s, lds);
  case 34:
    return launch_split<1>("tcp4_tas14_kernel<hints,verify,flow,keyonly>",
                           tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplit1, 12>, p, s, lds);
  case 29:
    return launch_split<1>("tcp4_tas14_kernel<hints,verify,flow,nokey>",
                           tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplit1, 1>, p, s, lds);
  case 30:
    return launch_split<1>("tcp4_tas14_kernel<hints,verify,flow,nocrc>",
                           tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplit1, 2>, p, s, lds);
  case 31:
    return launch_split<1>("tcp4_tas14_kernel<hints,verify,flow,nofskey>",
                           tcp4_tas14_kernel<6, kHintArr, true, 8, false, kBlock, false, kFlowSplit1, 4>, p, s, lds);
  default:
    return TASX_EXT_PASS;
  }
}

extern "C" TASX_INTERNAL int ab_launch_rx(const tasx_tcp4_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  if (tas14_ok(*p)) {
    const uint32_t lds = env_lds("TASX_TAS14_VERIFY_HINT_LDS", kOccLds);
    switch (variant) {
    case 26:
      return launch_groups("tcp4_tas14_kernel<hint,verify,flow_row>",
                           tcp4_tas14_kernel<6, kHint, true, 1, false, kBlock, false, kFlowRow>, *p, s, lds);
    case 27:
      return launch_split<1>("tcp4_tas14_kernel<hint,verify,flow_f1>",
                             tcp4_tas14_kernel<6, kHint, true, 1, false, kBlock, false, kFlowSplit1>, *p, s, lds);
    case 32:
      return launch_splitx<1>("tcp4_tas14_kernel<hint,verify,flow_xcd>",
                              tcp4_tas14_kernel<6, kHint, true, 1, false, kBlock, false, kFlowSplitX>, *p, s, lds);
    case 36: // the round-2 product: lookup blocks over consecutive frames
      return launch_split<2>("tcp4_tas14_kernel<hint,verify,flow_split2>",
                             tcp4_tas14_kernel<6, kHint, true, 1, false, kBlock, false, kFlowSplit>, *p, s, lds);
    default:
      return TASX_EXT_PASS;
    }
  }
  if (tas14_nohint_ok(*p) || tas14_offs_ok(*p)) {
    const int mode = p->flen ? kHintArr : kTlFirst;
    return p->off ? ab_rx_rows<true>(*p, mode, s, variant) : ab_rx_rows<false>(*p, mode, s, variant);
  }
  return TASX_EXT_PASS;
}
