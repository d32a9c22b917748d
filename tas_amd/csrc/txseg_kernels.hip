// txseg_kernels.hip -- fused TX segment build for gfx950 (SURVEY.md section 8f
// row 1): the payload copy of flow_tx_segment() (flow_tx_read() from the
// flow's circular TX buffer, /root/reference/tas/fast/fast_flows.c:833-846 and
// :930-933, dma_read tas/fast/dma.h:39-53) fused with the tcp_checksums() that
// follows it (:936 -> :1058-1069).  TAS reads the payload twice (rte_memcpy,
// then the checksum loop); here each payload byte is read once from the TX
// buffer, written once into the frame, and summed from registers.
//
// Kernels (tasx_launch_txseg): tx_segment_lds_kernel for TAS's layout (aligned
// source loads realigned through a per-row LDS slice), tx_segment_u_kernel
// (any layout: one unaligned window load per frame chunk, txseg_row), and the
// aligned-gather kernel below for checksum fields past the frame's first 256
// bytes.
//
// Aligned-gather kernel layout: one 16-lane group (a DPP row) per segment, as in the checksum
// kernels.  The group walks the frame's address-aligned 16-byte chunks
// covering [l4_off, hdrs_len + payload).  For a chunk that holds payload bytes
// the lane loads the two aligned source chunks spanning the payload bytes'
// window in the TX buffer (clamped so both hold valid bytes: they cannot
// fault), funnel-shifts them into frame alignment (v_alignbyte_b32), writes
// them (one dwordx4 store, byte stores at the two partial ends) and sums the
// chunk value the frame will hold.  Header chunks (before hdrs_len) are read
// from the frame.  A chunk whose payload window straddles the end of the
// circular buffer (at most one per segment) is gathered byte by byte.  Bytes
// the IPv4 total_length covers beyond hdrs_len + payload (never produced by
// flow_tx_segment, :897) are summed from the frame in a second pass.  The
// arithmetic (exact 64-bit dword sums, end-around folds, residues) is the
// checksum kernels' (xsum_kernels.hip header comment).
#include "txseg_rows.h"

extern "C" int tasx_launch_txseg(const tasx_txseg_params *p, void *stream)
{
  constexpr uint64_t spb = kBlock / 16;
  const uint64_t blocks = ((uint64_t) p->n + spb - 1) / spb;
  if (blocks == 0)
    return 0;
  const dim3 grid((uint32_t) blocks), block(kBlock);
  hipStream_t s = (hipStream_t) stream;
  // the unaligned-load kernel needs both checksum fields within the frame's first
  // 16 chunks (any frame alignment) and shm_len >= 16
  const bool u_ok = p->l4_off + 18u + 15u <= 256u && p->ip_off + 12u + 15u <= 256u && p->shm_len >= 16u;
  // the TAS kernel: IPv4 at 14, TCP at 34 (its other segments go to the general body)
  const bool tas = p->ip_off == 14u && p->l4_off == 34u;
  if (!u_ok) {
    // checksum fields beyond the frame's first 256 bytes: the aligned-gather build
    tasx_note_kernel("tx_segment_kernel");
    hipLaunchKernelGGL((tx_segment_kernel<6>), grid, block, 0, s, *p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (tas) {
    // aligned L2-allocating loads realigned through LDS (34-35 us against 43 us
    // for the round-2 form's unaligned windows on the bench's pattern;
    // tools/txseg_lds_probe.hip)
    tasx_note_kernel("tx_segment_lds_kernel");
    hipLaunchKernelGGL((tx_segment_lds_kernel<true>), grid, block, 0, s, *p);
  } else {
    tasx_note_kernel("tx_segment_u_kernel");
    hipLaunchKernelGGL((tx_segment_u_kernel<6, true>), grid, block, 0, s, *p);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
