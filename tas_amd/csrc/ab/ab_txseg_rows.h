// ab/ab_txseg_rows.h -- comparison build only (libtasx_ab.so): the TX
// segment build forms kept beside the product's (txseg_rows.h) for the tests
// and the bench's access-pattern ceiling:
//   tx_segment_tas_kernel -- the round-2 product (one unaligned non-temporal
//     window load per frame chunk, header-first stores, DPP tail); tests run
//     it beside the product on every TX case (TASX_TXSEG_DEBUG=30, "r2")
//   tx_segment_lds_ab_kernel<..., OPT> -- the product's row with its round-3
//     options: OPT 8 = the access pattern alone (bench.py's tx_segment
//     pattern_ceiling, TASX_TXSEG_DEBUG=40)
// The round-1 diagnostics forms, the one-segment-per-wave kernel and the
// other ablations were null results (profiles/r02-r04) and are gone (round 6).
#ifndef TASX_AB_TXSEG_ROWS_H_
#define TASX_AB_TXSEG_ROWS_H_

#include "../txseg_rows.h"

namespace {

// ---------------------------------------------------------------------------
// tx_segment_tas_kernel: TAS data segments as flow_tx_segment() builds them
// (fast_flows.c:877-955): IPv4 at frame + 14, TCP at + 34 (host-checked for
// the batch), hdrs_len 66 (TCP header + 12-byte timestamp option, :887-888),
// frames 16-byte aligned (the mbuf data room).  The header geometry is then
// fixed and the per-chunk work is the copy itself: frame chunk k >= 5 holds
// payload [16k - 66, 16k - 50), one unaligned window load, one store, four
// v_sad_u16.  Chunks 0..4 (ethernet + IPv4 + TCP + option, and chunk 4's
// first 14 payload bytes) are read from the frame and written back whole at
// the end with both checksums inserted; the IPv4 / pseudo-header channels
// come from chunks 0..2 as in tcp4_tas14_kernel (xsum_kernels.hip).  A
// segment with another hdrs_len or frame alignment, or whose ip.total_length
// is not 52 + payload (:897), is done by the general body (txseg_row), which
// rewrites the same payload bytes and then the checksums.  When the
// descriptor's room (the mbuf data room) covers the frame's last 16-byte
// chunk, that chunk is written whole, its bytes past the frame with their own
// values, instead of by dword and byte stores.
// OPT: how the frame's first block is written, and A/B ablations.
//   kTxHeaderFirst (the product): chunks 0..4 (headers with stale checksum
//     fields, chunk 4's payload) are stored right after the first round's loads
//     are issued, every payload chunk as soon as it lands, and at the end only
//     the two 16-bit checksum fields -- into lines the kernel has just written,
//     merged in L2 (44.9-45.0 against 46.0 us, traffic 1.126 against 1.143 x
//     algorithmic; profiles/r02/r02ar).
//   kTxDppTail (the product, with kTxHeaderFirst): the row total reaches every
//     lane by row rotations and the lane holding chunk 1 finishes and writes
//     both fields, instead of four ds_bpermute round trips to and from lane 15
//     (0.1-0.3 us better in 4 of 4 same-box pairs; profiles/r02/r02ax, r02ay).
//     Occupancy: the kernel holds 105 VGPRs (4 waves per SIMD); 5 waves
//     (WPE 5: 96 VGPRs, a small spill) costs 48 us and residency capped at 3
//     or 2 blocks per CU 46 / 50 us.
//   0: the round-1 form -- the first 256-byte block (headers with both
//     checksums + the payload chunks kept in vfb) written by one instruction
//     at the end; kTxLineKeep: keep only chunk 4's 128-byte line; kTxFieldsOnly:
//     keep nothing, write back chunks 1, 3, 4; kTxSimple: branch-free loop for
//     the common case (profiles/r02/r02v, r02x).
//   Ablations (timing only, results wrong; profiles/r02/r02u): kTxNoScratch,
//     kTxNoWriteBack, kTxNoWindows (chunk-4 / piece-2 window loads),
//     kTxNoFallback (general body not compiled in), kTxNoPayloadStores.
enum : int {
  kTxNoScratch = 1, kTxNoWriteBack = 2, kTxNoWindows = 4, kTxNoFallback = 8, kTxNoPayloadStores = 16,
  kTxLineKeep = 32, kTxFieldsOnly = 64, kTxSimple = 128, kTxHeaderFirst = 256, kTxDppTail = 512,
  kTxNoHeaderStore = 1024, kTxNoFields = 2048, kTxNoSums = 4096 // timing-only ablations (profiles/r02/r02az)
};
template <int U, bool NTS, int WPE = 1, int OPT = kTxHeaderFirst | kTxDppTail>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void tx_segment_tas_kernel(tasx_txseg_params p)
{
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group leaves together
  const u32x4 d0 = ld16((const u32x4 *) p.segs, 2 * i), d1 = ld16((const u32x4 *) p.segs, 2 * i + 1);
  const uint64_t frame_off = d0.x | ((uint64_t) d0.y << 32);
  const uint64_t tx_base = d0.z | ((uint64_t) d0.w << 32);
  const uint32_t tx_len = d1.x, pos = d1.y, pay_ = d1.z & 0xffffu, hl_ = d1.z >> 16;
  const bool ok = (pay_ == 0 || pos < tx_len) && pay_ <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl_ >= p.l4_off + 20;
  uint8_t *const f = p.frames + frame_off;
  bool fast = ok && hl_ == 66u && ((uintptr_t) f & 15u) == 0;
  if (fast) {
    const int pay = (int) pay_, fend = 66 + pay;
    const int K = (fend + 15) >> 4;
    // the descriptor's room covers the last chunk: write it whole, the bytes
    // past the frame with their own values (sub-dword stores cost ~10% here).
    // A scratch room (TASX_TXSEG_SCRATCH) also lets the build write the frame's
    // last 128-byte block whole, with zeros past the frame: no read of the last
    // chunk and no partial-line write for the memory side to merge.
    const uint32_t room = d1.w & ~TASX_TXSEG_SCRATCH;
    const bool scratch = (d1.w & TASX_TXSEG_SCRATCH) != 0u && room >= 16u * (uint32_t) K;
    const bool whole = room >= 16u * (uint32_t) K;
    int kend = K; // chunks [K, kend): scratch zeros up to the block's end
    if (scratch) {
      const uint64_t be = (frame_off + (uint64_t) fend + 127u) & ~127ull;
      kend = max(K, min((int) ((be - frame_off + 15u) >> 4), (int) (room >> 4)));
    }
    const int aoff = (int) (((uintptr_t) f >> 4) & 15u);
    const int kh = (gl - aoff) & 15; // this lane's chunk in the frame's first 256-byte block
    const uint8_t *const shm = p.shm;
    const uint32_t s1 = (uint32_t) (tx_base + pos);
    const int wrap = (int) tx_len - (int) pos;
    const int wrapc = (pay > 0 && wrap < pay) ? wrap : 0x7fffffff; // payload index where piece 2 starts
    const uint32_t smax = (uint32_t) (p.shm_len - 16u);
    auto woff = [&](int j0) -> uint32_t { return s1 + (uint32_t) j0 - (j0 >= wrapc ? tx_len : 0u); };
    const bool straddle = wrapc < pay && ((66 + wrap) & 15);
    const int ks = straddle ? (66 + wrap) >> 4 : -1;
    const uint32_t xoff = straddle ? s1 - tx_len + (uint32_t) (16 * ks - 66) : s1;
    // up front: the header chunk, chunk 4's window (payload [-2, 14)), the piece-2 window
    const u32x4 hv = ld16((const u32x4 *) f, (uint32_t) min(kh, 4));
    const uint32_t o4 = s1 - 2u;
    const u32x4 w4 = (OPT & kTxNoWindows) ? hv : ld16u(shm, min(o4, smax));
    const u32x4 xw = (OPT & kTxNoWindows) ? hv : ld16u(shm, min(xoff, smax));
    u32x4 tv = {0u, 0u, 0u, 0u};
    if (!scratch)
      tv = ld16((const u32x4 *) f, (uint32_t) (K - 1)); // the frame's last chunk as it is

    // whole payload chunks 5..K-1; each store instruction covers whole 256-byte
    // blocks.  The payload chunks of the frame's first block (k < fbe) are kept
    // in vfb and stored at the end together with the header chunks, so the
    // block's lines are written whole by one instruction (a line written in two
    // parts at different times costs an HBM read-modify-write).
    int fbe = aoff <= 10 ? 16 - aoff : 0;
    if (OPT & kTxLineKeep) { // A/B: keep only the payload chunks of chunk 4's 128-byte line
      const int lo8 = aoff & 7;
      fbe = min(fbe, 8 * ((lo8 + 4) / 8 + 1) - lo8);
    }
    if (OPT & (kTxFieldsOnly | kTxHeaderFirst)) // A/B: keep nothing (64: the write-back stores chunks 1, 3, 4 only;
      fbe = 0;          // 256: chunks 0..4 stored early, the two checksum fields at the end)
    // chunks 0..4 (tcp4_tas14_kernel's map for 0..3; chunk 4 = option pad + payload [0, 14))
    auto header_chunk = [&]() -> u32x4 {
      u32x4 h = hv;
      if (kh == 4) {
        u32x4 win = o4 <= smax ? w4 : gather16(shm, o4, p.shm_len);
        if (ks == 4)
          win = splice(win, xoff <= smax ? xw : gather16(shm, xoff, p.shm_len), wrap + 2, 16);
        h = splice(hv, win, 2, fend - 64);
      }
      return h;
    };
    auto store_header = [&](const u32x4 &h) {
      uint8_t *const cp = f + 16 * kh;
      const int hi = fend - 16 * kh;
      if (kh < 5 && hi >= 16)
        *(__attribute__((address_space(1))) u32x4 *) cp = h;
      else if (kh < 5 && whole && kh < K) // h holds the frame's own bytes past its end
        *(__attribute__((address_space(1))) u32x4 *) cp = h;
      else if (kh < 5)
        store_range(cp, h, 0, hi, false);
    };
    u32x4 vfb = hv;
    uint32_t acc = 0;
    const int base0 = 5 - ((5 + aoff) & 15);
    // the common case, wave-wide: every row a fast one with no wrap inside its
    // payload, every window inside the region, one round of chunks.  Its loop
    // has no per-chunk branches but the store's predicate (sums by select)
    const bool simple_row = fast && wrapc == 0x7fffffff && o4 <= smax && base0 + 16 * U >= K &&
                            s1 + (uint32_t) (16 * (K - 1) - 66) <= smax;
    const bool simple = (OPT & kTxSimple) && __builtin_amdgcn_ballot_w64(!simple_row) == 0ull;
    if (simple) {
      u32x4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(max(base0 + gl + 16 * u, 5), K - 1);
        a[u] = ld16u(shm, s1 + (uint32_t) (16 * k - 66));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = base0 + gl + 16 * u, hi = fend - 16 * k;
        const u32x4 v = a[u];
        const bool in = k >= 5 && k < K, full = in && hi >= 16;
        const bool keep = u == 0 && k < fbe;
        if (full && !keep)
          __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
        if (u == 0)
          vfb = full && keep ? v : vfb;
        const uint32_t sv = sad4(v, 0u);
        acc += full ? sv : 0u;
        if (in && hi < 16) { // the frame's last chunk (one lane per row)
          acc += sad_below(v, (uint32_t) hi);
          uint8_t *const cp = f + 16 * k;
          if (whole)
            *(__attribute__((address_space(1))) u32x4 *) cp = splice(tv, v, 0, hi);
          else
            store_range(cp, v, 0, hi, false);
        }
      }
    }
    for (int base = base0; !simple && base < K; base += 16 * U) {
      u32x4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(max(base + gl + 16 * u, 5), K - 1);
        a[u] = ld16u(shm, min(woff(16 * k - 66), smax));
      }
      if ((OPT & kTxHeaderFirst) && !(OPT & kTxNoHeaderStore) && base == base0) // the header chunks (stale checksum fields) go out first
        store_header(header_chunk());
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = base + gl + 16 * u, j0 = 16 * k - 66;
        if (k < 5 || k >= K)
          continue;
        u32x4 v = a[u];
        const uint32_t off = woff(j0);
        if (off > smax) // a window reaching past the region's end: byte by byte
          v = gather16(shm, off, p.shm_len);
        if (k == ks)
          v = splice(v, xoff <= smax ? xw : gather16(shm, xoff, p.shm_len), wrap - j0, 16);
        uint8_t *const cp = f + 16 * k;
        const int hi = fend - 16 * k;
        if (u == 0 && k < fbe && hi >= 16) {
          vfb = v;
          acc = sad4(v, acc);
        } else if (hi >= 16) {
          if (OPT & kTxNoPayloadStores)
            ;
          else if (NTS)
            __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
          else
            *(__attribute__((address_space(1))) u32x4 *) cp = v;
          if (!(OPT & kTxNoSums))
            acc = sad4(v, acc);
        } else {
          acc += sad_below(v, (uint32_t) hi);
          if (whole)
            *(__attribute__((address_space(1))) u32x4 *) cp = splice(tv, v, 0, hi);
          else
            store_range(cp, v, 0, hi, false);
        }
      }
    }

    if (scratch && !(OPT & kTxNoScratch)) { // the scratch chunks past the frame outside its first block
      const int k = K + gl;
      if (k < kend && k >= fbe)
        __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
    }

    u32x4 h = header_chunk();
    const uint32_t m0 = kh == 2 ? 0xffff0000u : (kh == 3 ? 0x0000ffffu : 0xffffffffu);
    uint32_t l4 = sad4(u32x4{h.x & m0, h.y, h.z, h.w}, 0u);
    if (kh == 4 && fend < 80)
      l4 = sad_below(h, (uint32_t) (fend - 64));
    acc += (kh >= 2 && kh <= 4) ? l4 : 0u;
    const uint32_t c0d3 = row_ror<1>(h.w), c2d0 = row_ror<15>(h.x);
    const uint32_t addrs = sadw(h.z & 0xffff0000u, sadw(h.w, sadw(c2d0 & 0xffffu, 0u)));
    const uint32_t ph = sadw(h.y & 0xff000000u, addrs);
    const uint32_t ipsum = sadw(c0d3 & 0xffff0000u, sadw(h.x, sadw(h.y, addrs)));
    const int l1 = (int) ((threadIdx.x & 63u) & ~15u) + ((1 + aoff) & 15); // lane holding chunk 1
    if ((OPT & kTxDppTail) && (OPT & kTxHeaderFirst)) {
      // no LDS round trips: every lane gets the row total by row rotations,
      // and the lane holding chunk 1 (ip.len, the IP header and pseudo-header
      // sums) finishes both checksums and writes both fields itself
      acc += row_ror<8>(acc);
      acc += row_ror<4>(acc);
      acc += row_ror<2>(acc);
      acc += row_ror<1>(acc);
      const bool ok1 = kh == 1 && bswap16(h.x & 0xffffu) == 52u + (uint32_t) pay;
      fast = (__builtin_amdgcn_ballot_w64(ok1) >> l1) & 1ull; // otherwise the general body redoes the segment
      if (ok1) {
        const uint32_t ipc = inv_result(residue(fold32_to_16(ipsum)));
        const uint32_t tcpc = inv_result(
            residue(fold32_to_16(fold32_to_16(acc) + fold32_to_16(ph) + bswap16(32u + (uint32_t) pay))));
        if (p.out)
          stg(p.out, i, ipc | (tcpc << 16));
        if (!(OPT & kTxNoFields)) {
          *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) ipc;
          *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) tcpc;
        }
      }
    } else {
    acc = row_sum16(acc);
    const uint32_t ip1 = (uint32_t) __shfl((int) ipsum, l1, 64), ph1 = (uint32_t) __shfl((int) ph, l1, 64);
    const uint32_t tl = bswap16((uint32_t) __shfl((int) (h.x & 0xffffu), l1, 64));
    fast = tl == 52u + (uint32_t) pay; // otherwise the general body redoes the segment
    const uint32_t ipc = inv_result(residue(fold32_to_16(ip1)));
    const uint32_t len = 32u + (uint32_t) pay;
    const uint32_t tcpc = inv_result(residue(fold32_to_16(fold32_to_16(acc) + fold32_to_16(ph1) + bswap16(len))));
    const uint32_t res = (uint32_t) __shfl((int) (ipc | (tcpc << 16)), (int) ((threadIdx.x & 63u) | 15u), 64);
    if ((OPT & kTxHeaderFirst) && fast) { // only the two fields are left to write
      if (gl == 15 && p.out)
        stg(p.out, i, res);
      if (kh == 1)
        *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) res;
      if (kh == 3)
        *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) (res >> 16);
    } else if (fast && !(OPT & kTxNoWriteBack)) {
      if (gl == 15 && p.out)
        stg(p.out, i, res);
      // the first block: header chunks with the checksums inserted (ip.chksum:
      // chunk 1 bytes 8-9, tcp.chksum: chunk 3 bytes 2-3) and the kept payload chunks
      if (kh == 1)
        h.z = (h.z & 0xffff0000u) | (res & 0xffffu);
      if (kh == 3)
        h.x = (h.x & 0x0000ffffu) | (res & 0xffff0000u);
      uint8_t *const cp = f + 16 * kh;
      const int hi = fend - 16 * kh;
      if ((OPT & kTxFieldsOnly) && (kh == 0 || kh == 2))
        ; // unchanged header chunks
      else if ((kh < 5 || kh < fbe) && hi >= 16)
        *(__attribute__((address_space(1))) u32x4 *) cp = kh < 5 ? h : vfb;
      else if (kh < 5 && whole && kh < K) // h holds the frame's own bytes past its end
        *(__attribute__((address_space(1))) u32x4 *) cp = h;
      else if (kh < 5)
        store_range(cp, h, 0, hi, false);
      else if (!(OPT & kTxNoScratch) && kh >= K && kh < kend && kh < fbe) // scratch chunks inside the first block
        *(__attribute__((address_space(1))) u32x4 *) cp = u32x4{0u, 0u, 0u, 0u};
    }
    }
  }
  if (!(OPT & kTxNoFallback) && !fast) // (3 chunks per lane and round: keeps the fallback's registers below the fast path's)
    txseg_row<3, NTS>(p, i, gl);
}

// ---------------------------------------------------------------------------
// tx_segment_lds_kernel (round 3, the product for TAS's layout): the same
// segment build, one 16-lane row per segment, with the payload read by
// ALIGNED, L2-allocating 16-byte loads and realigned through a per-row LDS
// slice instead of one unaligned non-temporal window load per frame chunk.
//   For the frame's (at most 96) chunks the row loads the aligned source chunks that
//   cover the payload windows: piece A (before the circular buffer
//   wraps) from its 128-byte line on, so that lanes own whole lines, then piece
//   B (after the wrap).  Lane gl, slot u loads virtual chunk gl + 16u (7 slots:
//   112 chunks, enough for 96 frame chunks at any shift) and writes it to slot
//   1 + gl + 16u of the slice.  Each lane then reads its frame chunk's 16-byte
//   window back at its byte offset as five dwords and funnel-shifts them
//   (v_alignbyte_b32); the chunk that straddles the wrap splices a piece-B
//   window in.  Header chunks 0..3 (read from the frame) and chunk 4 (header
//   bytes 64-65 + payload [0, 14)) go out in round 0's store instructions with
//   stale checksum fields, every store non-temporal and covering whole 256-byte
//   blocks (lanes own frame chunks by address); the two 16-bit fields are
//   stored at the end by the lane holding chunk 1, after the row total has
//   reached it by DPP row rotations.
//   Why: an unaligned window shares its first and last 128-byte lines with the
//   neighbouring windows, and with non-temporal loads those lines were fetched
//   again; aligned temporal loads let L2 merge them.  On the bench's pattern
//   (tools/txseg_lds_probe.hip, profiles/r03/r03c-r03d): 43.3 us for the
//   unaligned non-temporal windows, 39.4 us for the same windows temporal,
//   34.2-34.9 us for this scheme.
//   Aligned loads never leave the pages of the bytes they hold, and each load
//   address is clamped to the aligned chunks that touch the shm region, so no
//   load faults; bytes outside what a window needs are masked away.
//   Rows that are not TAS data segments (hdrs_len != 66, a frame off 16-byte
//   alignment, total_length != 52 + payload, a rejected descriptor) go to the
//   general body (txseg_row), as before.
// SLOTS load slots per lane: 6 (96 aligned chunks: piece A from its 16-byte
// chunk on, 25.3 KiB of LDS per block, 6 blocks per CU) or 7 (112: piece A from
// its 128-byte line on, so lanes own whole lines; 29.4 KiB, 5 blocks per CU).
// A window's bytes [o, o + 16) lie in the loaded chunks; its fifth dword, read
// past them, lies in the same aligned chunk as byte o + 15.
template <bool NTS, int SLOTS = 6, int WPE = 1, int OPT = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void tx_segment_lds_ab_kernel(tasx_txseg_params p)
{
  constexpr int kLdsSlots = SLOTS, kLdsSlice = lds_slice<SLOTS>();
  constexpr uintptr_t kAlignA = SLOTS >= 7 ? 127u : 15u;
  __shared__ __attribute__((aligned(16))) uint8_t lds[(kBlock / 16) * kLdsSlice];
  const int gl = threadIdx.x & 15;
  const uint32_t i = blockIdx.x * (kBlock / 16) + threadIdx.x / 16;
  if (i >= p.n)
    return; // whole 16-lane group leaves together
  uint8_t *const sl = lds + (threadIdx.x / 16) * kLdsSlice;
  const u32x4 d0 = ld16((const u32x4 *) p.segs, 2 * i), d1 = ld16((const u32x4 *) p.segs, 2 * i + 1);
  const uint64_t frame_off = d0.x | ((uint64_t) d0.y << 32);
  const uint64_t tx_base = d0.z | ((uint64_t) d0.w << 32);
  const uint32_t tx_len = d1.x, pos = d1.y, pay_ = d1.z & 0xffffu, hl_ = d1.z >> 16;
  const bool ok = (pay_ == 0 || pos < tx_len) && pay_ <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl_ >= p.l4_off + 20;
  uint8_t *const f = p.frames + frame_off;
  // one round of 96 frame chunks: frames up to 1536 bytes (TAS's data
  // segments are at most 66 + TCP_MSS = 1514, fast_flows.c:37, :887-888);
  // larger ones go to the general body
  bool fast = ok && hl_ == 66u && ((uintptr_t) f & 15u) == 0 && pay_ <= 1536u - 66u;
  if (fast) {
    const int pay = (int) pay_, fend = 66 + pay;
    const int K = (fend + 15) >> 4;
    // the room: the last chunk written whole (its bytes past the frame with
    // their own values), or -- scratch -- the frame's last 128-byte block
    // written whole with zeros past the frame (no read, no partial line; within
    // the round's 96 chunks)
    const uint32_t room = d1.w & ~TASX_TXSEG_SCRATCH;
    const bool scratch = (d1.w & TASX_TXSEG_SCRATCH) != 0u && room >= 16u * (uint32_t) K;
    const bool whole = room >= 16u * (uint32_t) K;
    int kend = K; // chunks [K, kend): scratch zeros up to the block's end
    if (scratch) {
      const uint32_t fo7 = (uint32_t) frame_off & 127u;
      kend = max(K, min(min((int) ((((fo7 + (uint32_t) fend + 127u) & ~127u) - fo7 + 15u) >> 4), (int) (room >> 4)), 96));
    }
    const int aoff = (int) (((uintptr_t) f >> 4) & 15u);
    const int kh = (gl - aoff) & 15; // this lane's chunk in every 16-chunk group of the frame
    // Shm positions as 32-bit offsets from the region's first aligned chunk
    // sbase (an SGPR base; shm_len < 4 GiB, checked by the host), modulo 2^32:
    // loads are clamped to the aligned chunks that touch the region, so an
    // offset that wrapped below the region (payload index -2 of a buffer at its
    // start: chunk 4's don't-care bytes) reads some chunk of the region.
    const uintptr_t sb = (uintptr_t) p.shm;
    const uint8_t *const sbase = (const uint8_t *) (sb & ~(uintptr_t) 15);
    const uint32_t sh0 = (uint32_t) (sb & 15u);
    const uint32_t hi_ok = (uint32_t) ((sb + p.shm_len - 1u) & ~(uintptr_t) 15) - (uint32_t) (sb & ~(uintptr_t) 15);
    const uint32_t t0 = sh0 + (uint32_t) tx_base, s1 = t0 + pos; // ring start, payload index 0
    const int wrap = (int) tx_len - (int) pos;
    const int wrapc = (pay > 0 && wrap < pay && !(OPT & 2)) ? wrap : 0x7fffffff; // payload index where piece B starts
    const u32x4 hv = ld16((const u32x4 *) f, (uint32_t) min(kh, 4)); // header chunks 0..4
    uint32_t acc = 0;
    u32x4 vlast = hv; // the frame's last chunk when it is partial (its lane: kh == (K - 1) & 15)
    const int hlast = fend - 16 * (K - 1); // bytes of the frame in its last chunk, 1..16
    {
      // payload windows of chunks [4, K): payload [jlo, jhi)
      const int jlo = -2, jhi = 16 * K - 66;
      const int aend = min(jhi, wrapc);
      // piece A: payload [jlo, aend) at s1 + j, from its 16-byte chunk (7 slots:
      // its 128-byte line) on
      const uint32_t bA = s1 + (uint32_t) jlo, cA = bA & ~(uint32_t) kAlignA;
      const int nA = aend > jlo ? (int) ((((bA + (uint32_t) (aend - jlo) + 15u) & ~15u) - cA) >> 4) : 0;
      // piece B: payload [max(jlo, wrapc), jhi) at the ring start + j - wrapc
      const int jb = max(jlo, wrapc);
      const uint32_t bB = t0 + (uint32_t) (jb > wrapc ? jb - wrapc : 0), cB = bB & ~15u;
      const int nB = jhi > wrapc ? (int) ((((bB + (uint32_t) (jhi - jb) + 15u) & ~15u) - cB) >> 4) : 0;
      // virtual chunk v is piece A's chunk v, else piece B's chunk v - nA; past
      // the end the last one again (an L2 hit)
      const int nAB = max(nA + nB, 1);
      const uint32_t dB = nB > 0 ? cB - cA - 16u * (uint32_t) nA : 0u;
      u32x4 a[kLdsSlots];
#pragma unroll
      for (int u = 0; u < kLdsSlots; ++u) {
        const int v = min(gl + 16 * u, nAB - 1);
        const uint32_t ro = cA + 16u * (uint32_t) v + (v >= nA ? dB : 0u);
        a[u] = ld16_off(sbase, min(ro, hi_ok));
      }
      if constexpr (!(OPT & 8)) {
#pragma unroll
        for (int u = 0; u < kLdsSlots; ++u)
          *(u32x4 *) (sl + kLdsLead + 16 * (gl + 16 * u)) = a[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      // LDS byte offsets: payload index 0 in piece A, piece B's first byte;
      // window u at o0 + 256u (+ dW for a window in piece B)
      const int oA = kLdsLead + (int) (s1 - cA);
      const int oB = kLdsLead + 16 * nA + (int) (t0 - cB);
      const int o0 = oA + 16 * kh - 66; // >= 0: the lead covers chunk 0's window
      const int dW = wrapc < pay ? oB - oA - wrapc : 0;
      u32x4 w[6]; // the windows of frame chunks 16u + kh
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        const int j0 = 16 * (16 * u + kh) - 66;
        const int o = min(o0 + 256 * u + (j0 >= wrapc ? dW : 0), kLdsSlice - 20);
        w[u] = (OPT & 8) ? a[u] : lds_window(sl, (uint32_t) o);
      }
      // the chunk holding the wrap (a row whose payload wraps off a chunk
      // boundary): its bytes from wrapc - j0 on are piece B's
      const int ks = wrapc < pay ? (66 + wrapc) >> 4 : -1;
      const bool strad = !(OPT & 8) && ks >= 0 && ((66 + wrapc) & 15) != 0 && kh == (ks & 15);
      if (__builtin_amdgcn_ballot_w64(strad) != 0ull) {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int j0 = 16 * (16 * u + kh) - 66;
          if (strad && u == (ks >> 4))
            w[u] = splice(w[u], lds_window(sl, (uint32_t) min(max(oB + j0 - wrapc, 0), kLdsSlice - 20)),
                          wrapc - j0, 16);
        }
      }
      // slot 0: header chunks 0..3 as read, chunk 4 = header bytes 64-65 +
      // payload [0, 14); L4 sums from chunk 2's byte 2 on (TCP starts at 34),
      // chunk 3 without tcp.chksum (bytes 2-3).  Slot 0 (the frame's first two
      // lines, both checksum fields) is stored L2-allocating so that the fields
      // stored at the end merge there; the rest non-temporal.
      if (kh < 4)
        w[0] = hv;
      else if (kh == 4)
        w[0] = splice(hv, w[0], 2, 16);
      const uint32_t mx = kh == 2 ? 0xffff0000u : (kh == 3 ? 0x0000ffffu : kh < 2 ? 0u : 0xffffffffu);
      const uint32_t mr = kh < 2 ? 0u : 0xffffffffu;
      if (__builtin_amdgcn_ballot_w64(K < 81) == 0ull) {
        // every row of the wave holds at least 81 chunks: slots 0..4 are whole
        // frame chunks, only slot 5 holds the frame's end
        acc = sad4(u32x4{w[0].x & mx, w[0].y & mr, w[0].z & mr, w[0].w & mr}, acc);
        if (OPT & 4)
          __builtin_nontemporal_store(w[0], (__attribute__((address_space(1))) u32x4 *) (f + 16 * kh));
        else
          *(__attribute__((address_space(1))) u32x4 *) (f + 16 * kh) = w[0];
#pragma unroll
        for (int u = 1; u < 5; ++u) {
          acc = sad4(w[u], acc);
          __builtin_nontemporal_store(w[u], (__attribute__((address_space(1))) u32x4 *) (f + 16 * (16 * u + kh)));
        }
        const int k = 80 + kh;
        const bool full = k < K - 1 || (k == K - 1 && hlast == 16);
        const uint32_t t = sad4(w[5], acc);
        acc = full ? t : acc;
        vlast = k == K - 1 ? w[5] : vlast;
        if (full || (k >= K && k < kend))
          __builtin_nontemporal_store(k < K ? w[5] : u32x4{0u, 0u, 0u, 0u}, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
      } else {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int k = 16 * u + kh;
          const u32x4 v = w[u];
          // whole chunks here, the partial last one after the loop
          const bool full = k < K - 1 || (k == K - 1 && hlast == 16);
          const uint32_t t = u == 0 ? sad4(u32x4{v.x & mx, v.y & mr, v.z & mr, v.w & mr}, acc) : sad4(v, acc);
          acc = full ? t : acc;
          vlast = k == K - 1 ? v : vlast;
          // whole chunks, and scratch zeros past the frame to its block's end
          if (full || (k >= K && k < kend)) {
            const u32x4 sv = k < K ? v : u32x4{0u, 0u, 0u, 0u};
            if (u == 0 && !(OPT & 4))
              *(__attribute__((address_space(1))) u32x4 *) (f + 16 * k) = sv;
            else
              __builtin_nontemporal_store(sv, (__attribute__((address_space(1))) u32x4 *) (f + 16 * k));
          }
        }
      }
    }
    if (hlast < 16 && kh == ((K - 1) & 15)) { // the frame's partial last chunk (one lane)
      acc += sad_below(vlast, (uint32_t) hlast);
      uint8_t *const cp = f + 16 * (K - 1);
      if (whole) // its bytes past the frame with their own values (scratch: zeros)
        __builtin_nontemporal_store(splice(scratch ? u32x4{0u, 0u, 0u, 0u} : ld16((const u32x4 *) cp, 0u), vlast, 0, hlast),
                                    (__attribute__((address_space(1))) u32x4 *) cp);
      else
        store_range(cp, vlast, 0, hlast, false);
    }
    // IPv4 and pseudo-header channels from header chunks 0..2 (tcp4_tas14_kernel's map)
    const uint32_t c0d3 = row_ror<1>(hv.w), c2d0 = row_ror<15>(hv.x);
    const uint32_t addrs = sadw(hv.z & 0xffff0000u, sadw(hv.w, sadw(c2d0 & 0xffffu, 0u)));
    const uint32_t ph = sadw(hv.y & 0xff000000u, addrs);
    const uint32_t ipsum = sadw(c0d3 & 0xffff0000u, sadw(hv.x, sadw(hv.y, addrs)));
    const int l1 = (int) ((threadIdx.x & 63u) & ~15u) + ((1 + aoff) & 15); // lane holding chunk 1
    acc += row_ror<8>(acc);
    acc += row_ror<4>(acc);
    acc += row_ror<2>(acc);
    acc += row_ror<1>(acc);
    const bool ok1 = kh == 1 && bswap16(hv.x & 0xffffu) == 52u + (uint32_t) pay;
    fast = (__builtin_amdgcn_ballot_w64(ok1) >> l1) & 1ull; // otherwise the general body redoes the segment
    if (ok1) {
      const uint32_t ipc = inv_result(residue(fold32_to_16(ipsum)));
      const uint32_t tcpc = inv_result(
          residue(fold32_to_16(fold32_to_16(acc) + fold32_to_16(ph) + bswap16(32u + (uint32_t) pay))));
      if (p.out)
        stg(p.out, i, ipc | (tcpc << 16));
      *(__attribute__((address_space(1))) uint16_t *) (f + 24) = (uint16_t) ipc;
      *(__attribute__((address_space(1))) uint16_t *) (f + 50) = (uint16_t) tcpc;
    }
  }
  if (!(OPT & 1) && !fast)
    txseg_row<3, NTS>(p, i, gl);
}

} // namespace
#endif
