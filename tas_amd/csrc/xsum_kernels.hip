// xsum_kernels.hip -- CDNA4 (gfx950) kernels for TAS's software TCP/IP checksum
// path (the --fp-no-xsumoffload branch of tcp_checksums(),
// /root/reference/tas/fast/fast_flows.c:1058-1069).
//
// Bandwidth-bound integer fold, no MFMA.  Layout and arithmetic:
//   * A packet (RAW payload, or the L4 segment of a TCP4 frame) is covered by
//     the naturally aligned 16-byte chunks [start & ~15, end rounded up).  A
//     16-lane group (one DPP row) owns a packet; lane gl loads chunks gl,
//     gl+16, ... with non-temporal global_load_dwordx4, U per lane issued back
//     to back with no branches (lanes past the packet re-read its last chunk:
//     same line, no extra HBM traffic, dropped by a select).  Reading an
//     aligned chunk that contains a valid byte never crosses a page, so it
//     cannot fault.
//   * Sums are taken over ADDRESS-aligned LE 16-bit words.  DPDK sums words
//     counted from the buffer start; for an odd start the two frames differ by
//     a byte swap of the folded result (RFC 1071 section 2(B)), applied at the end.
//   * Each lane accumulates the 32-bit words of its chunks in 64 bits (exact:
//     never wraps for packets < 2^32 words).  Because 2^16 == 1 (mod 0xffff),
//     the dword sum is congruent to the 16-bit word sum, and every end-around
//     fold keeps both the residue mod 0xffff and "zero iff all words zero" --
//     which is exactly what rte_raw_cksum returns.
//     Bytes before / after the packet in its first / last chunk are removed by
//     exact subtraction on the lane that holds that chunk.
//   * Group reduction: 4 DPP row_shr adds; the total lands in lane 15.
//   * TCP4 (rte_ipv4_cksum + rte_ipv4_udptcp_cksum) depends only on the
//     residue mod 0xffff of (header sum) and of (L4 sum + pseudo-header), so the
//     zeroed checksum fields are handled by masking or by subtracting their
//     bytes modulo 0xffff.
//
// Kernels in the product library (tasx_set_kernel_variant):
//   2 = raw_sad_kernel (general) / tcp4_frame_kernel (any layout),
//   3 = tcp4_tas_kernel (TAS frame layout, stride mode),
//   6 = tcp4_tas14_kernel (TAS frames in 16-byte aligned rooms: the headline with
//       a uniform frame-length hint; per-row total_length modes otherwise),
//   7 = raw_wave_kernel (RAW with per-packet lengths: a wave's 4 packets as one
//       chunk sequence).
// The device code lives in xsum_rows.h.
#include "xsum_rows.h"

// ---------------------------------------------------------------------------
// launchers (C ABI, internal to libtasx)

// the launched kernel's name, per calling thread (tasx_last_kernel)
static thread_local const char *t_last_kernel = "";

extern "C" const char *tasx_last_kernel(void)
{
  return t_last_kernel;
}

extern "C" void tasx_note_kernel(const char *name)
{
  t_last_kernel = name;
}

// completion word: stream-ordered after the work before it, one lane stores
// seq into pinned host memory with system-scope release, so a host spinning on
// the word sees every earlier result (tasx_flush's wait, tasx_host.c)
namespace {
__global__ __launch_bounds__(64) void post_done_kernel(uint32_t *word, uint32_t seq)
{
  if (threadIdx.x == 0)
    __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
} // namespace

extern "C" int tasx_launch_post_done(uint32_t *word, uint32_t seq, void *stream)
{
  hipLaunchKernelGGL(post_done_kernel, dim3(1), dim3(64), 0, (hipStream_t) stream, word, seq);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The offload branch of tcp_checksums() (fast_flows.c:1060-1064): ip.chksum
// = 0 and tcp.chksum = tx_xsum_enable() = network_ip_phdr_xsum(ip.src,
// ip.dest, IP_PROTO_TCP, l3_paylen) (fastemu.h:97-102, network.h:157-173):
// the pseudo-header words (the address fields' bytes as native little-endian
// 16-bit words, proto << 8, the L3 payload length in network order), folded
// twice, NOT inverted -- the NIC finishes the checksum.  l3_paylen =
// ip.total_length - 20 as a 16-bit value (what every caller passes,
// fast_flows.c:936,1012,1074).  One lane per frame; 12 header bytes read.
namespace {
__global__ __launch_bounds__(kBlock) void tcp4_offload_kernel(tasx_tcp4_params p)
{
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= p.n)
    return;
  uint8_t *f = p.base + pkt_offset(p.off, p.stride, i);
  uint8_t *ip = f + p.ip_off;
  const uint32_t tl = (ld8(ip + 2) << 8) | ld8(ip + 3);
  uint32_t sum = (6u << 8) + bswap16((tl - 20u) & 0xffffu);
#pragma unroll
  for (int k = 12; k < 20; k += 2)
    sum += ld8(ip + k) | (ld8(ip + k + 1) << 8);
  sum = (sum >> 16) + (sum & 0xffffu);
  sum = (sum >> 16) + (sum & 0xffffu);
  if (p.out)
    stg(p.out, i, (uint16_t) sum);
  if (p.flags & TASX_F_INPLACE) {
    uint8_t *tcp = f + p.l4_off;
    st8(ip + 10, 0u);
    st8(ip + 11, 0u);
    st8(tcp + 16, sum);
    st8(tcp + 17, sum >> 8);
  }
}
} // namespace

extern "C" int tasx_launch_tcp4_offload(const tasx_tcp4_params *p, void *stream)
{
  const uint64_t blocks = ((uint64_t) p->n + kBlock - 1) / kBlock;
  if (blocks == 0)
    return 0;
  if (blocks > 0x7fffffffull)
    return -2;
  t_last_kernel = "tcp4_offload_kernel";
  hipLaunchKernelGGL(tcp4_offload_kernel, dim3((uint32_t) blocks), dim3(kBlock), 0, (hipStream_t) stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int tasx_launch_raw(const tasx_raw_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  switch (variant) {
  case 2: // the general form
    return launch_groups("raw_sad_kernel", raw_sad_kernel<6>, *p, s, kOccLds);
  case 7:
    return launch_groups("raw_wave_kernel", raw_wave_kernel<TASX_WAVE_U>, *p, s, TASX_WAVE_LDS);
  case 3:
  case 6: // the 16-lane rows whatever the lengths
    break;
  default: // 0 automatic (TCP4-only variants run it too): per-packet lengths -> 7
    if (p->len)
      return launch_groups("raw_wave_kernel", raw_wave_kernel<TASX_WAVE_U>, *p, s, TASX_WAVE_LDS);
    break;
  }
  if (p->off == nullptr && ((uintptr_t) p->base & 15u) == 0 &&
      (uint64_t) (kBlock / 16) * p->stride + TASX_RAW_MAX_LEN + 16u < (1ull << 32))
    return launch_groups("raw_sad_kernel<s32>", raw_sad_kernel<6, true>, *p, s, kOccLds);
  return launch_groups("raw_sad_kernel", raw_sad_kernel<6>, *p, s, kOccLds);
}

template <bool OFFS>
static int launch_tas14_rx(const tasx_tcp4_params &p, int mode, hipStream_t s)
{
  // RX bursts without a uniform length are data/ACK mixes: one frame per
  // lookup lane, each lookup block over the frames of the 16 verify blocks on
  // its own XCD, so that the verify rows find the frames' first lines in L2
  // (64K frames, 0 / 50 / 100 % ACKs: 17.4 / 12.1 / 7.7-7.9 us against 18.3-18.6
  // / 12.8-12.9 / 8.8-9.0 for lookup blocks over consecutive frames, and 16.9 /
  // 13.0 / 7.1-7.3 with two frames per lane; profiles/r03/INDEX.md r03b)
  return mode == kHintArr ? launch_rx_rows<OFFS, kHintArr>(p, s) : launch_rx_rows<OFFS, kTlFirst>(p, s);
}

// RX verification + flow lookup: the row kernels' selection (as
// tasx_launch_tcp4_verify) with the lookup blocks first in the same grid
// (kFlowSplitX*); batches no row kernel takes run the general verify kernel
// and then flow_lookup_kernel
extern "C" int tasx_launch_tcp4_rx(const tasx_tcp4_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  const bool auto6 = variant == 0 || variant == 6 || variant >= 7;
  if (auto6 && tas14_ok(*p)) {
    // a uniform received length is a data burst: two frames per lookup lane,
    // each lookup block over the frames of the 32 verify blocks on its own XCD
    // (64K frames: 16.8 against 17.1 us with one frame per lane and 17.6-17.9
    // with lookup blocks over consecutive frames; profiles/r03/INDEX.md r03b)
    return launch_splitx<2>("tcp4_tas14_kernel<hint,verify,flow>",
                            tcp4_tas14_kernel<6, kHint, true, 1, false, kFlowSplitX2>, *p, s, kOccLds);
  }
  if (auto6 && (tas14_nohint_ok(*p) || tas14_offs_ok(*p))) {
    const int mode = p->flen ? kHintArr : kTlFirst;
    return p->off ? launch_tas14_rx<true>(*p, mode, s) : launch_tas14_rx<false>(*p, mode, s);
  }
  int r = tasx_launch_tcp4_verify(p, variant, stream);
  if (r != 0)
    return r;
  tasx_flow_params fp = {};
  fp.base = p->base;
  fp.off = p->off;
  fp.stride = p->stride;
  fp.flowht = p->flowht;
  fp.flowst = p->flowst;
  fp.hash_out = p->hash_out;
  fp.fid_out = p->fid_out;
  fp.n = p->n;
  fp.ip_off = p->ip_off;
  fp.l4_off = p->l4_off;
  fp.ht_entries = p->ht_entries;
  fp.fs_num = p->fs_num;
  fp.fs_stride = p->fs_stride;
  fp.fs_key_off = p->fs_key_off;
  r = tasx_launch_flow_lookup(&fp, 0, stream);
  tasx_note_kernel("tcp4 verify + flow_lookup_kernel");
  return r;
}

extern "C" int tasx_launch_tcp4_verify(const tasx_tcp4_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  const bool auto6 = variant == 0 || variant == 6 || variant >= 7;
  if (auto6 && tas14_ok(*p))
    return launch_groups("tcp4_tas14_kernel<hint,verify>", tcp4_tas14_kernel<6, kHint, true>, *p, s, kOccLds);
  // RX batches mix data and ACKs too: as the TX form, 8 waves per SIMD and no
  // LDS cap (64K frames, per-frame hints, 0 / 25 / 50 / 75 % ACKs: 17.0 / 14.2
  // / 11.9 / 10.2 -> 17.1 / 13.8 / 10.9 / 8.7 us; profiles/r01_ackmix_verify_ab.txt),
  // and the TX form's row modes: the received lengths as per-frame hints ->
  // each row reads exactly its received bytes at once (a total_length that
  // disagrees -- padding, truncation, a forged length -- is redone by the
  // bounded general body; profiles/r02/r02ac), else total_length first: RX
  // bursts are mixes, where whole-room rows lose (64K frames, room 2048, 0 /
  // 50 % ACKs: 16.3 / 16.3 us against 16.9 / 10.8-11.1; profiles/r02/r02ad).
  if (auto6 && (tas14_nohint_ok(*p) || tas14_offs_ok(*p))) {
    const int mode = p->flen ? kHintArr : kTlFirst;
    return p->off ? launch_tas14_verify<true>(*p, mode, s) : launch_tas14_verify<false>(*p, mode, s);
  }
  return launch_groups("tcp4_frame_kernel<verify>", tcp4_frame_kernel<6, true>, *p, s);
}

extern "C" int tasx_launch_tcp4(const tasx_tcp4_params *p, int variant, void *stream)
{
  hipStream_t s = (hipStream_t) stream;
  if (variant != 2 && variant != 3)
    variant = 0; // 6 = the automatic choice; the RAW-only number runs it too
  if (variant == 0) {
    // TAS frames in 16-byte rooms: a uniform hint, per-frame hints or none ->
    // tcp4_tas14_kernel; frames by offsets -> its OFFS form
    if (tas14_ok(*p))
      return launch_groups("tcp4_tas14_kernel<hint>", tcp4_tas14_kernel<6, kHint>, *p, s, kOccLds);
    if (tas14_nohint_ok(*p))
      return launch_tas14_rows<false>(*p, tas14_mode(*p), s);
    if (tas14_offs_ok(*p))
      return launch_tas14_rows<true>(*p, tas14_mode(*p), s);
    // other TAS-layout batches with a hint -> 3, the rest -> 2
    variant = tas_kernel_ok(*p) && (p->flen || p->flen0) ? 3 : 2;
  }
  if (variant == 3 && tas_kernel_ok(*p))
    return launch_groups("tcp4_tas_kernel", tcp4_tas_kernel<6>, *p, s);
  return launch_groups("tcp4_frame_kernel", tcp4_frame_kernel<6>, *p, s);
}
