// server_device.h -- the persistent flush server's kernel (round 4; see
// server_kernels.hip for the protocol, and the epochs of round 6).
#ifndef TASX_SERVER_DEVICE_H_
#define TASX_SERVER_DEVICE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tasx_kernels.h"

#include "xsum_device.h"
#include "txseg_device.h"

namespace {

constexpr int kSrvBlock = 1024;           // 64 rows of 16 lanes: one frame per row
constexpr int kSys = 1 | 16;              // cache policy sc0 sc1: system scope
constexpr int kNt = 2;                    // non-temporal (the frame loads, after an acquire)
constexpr uint32_t kRsrcWord3 = 0x00020000u; // gfx9 buffer resource dword 3

__device__ __forceinline__ uint64_t ld_sys64(const uint64_t *p)
{
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys32(uint32_t *p, uint32_t v)
{
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys64(uint64_t *p, uint64_t v)
{
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t rlane64(uint64_t x, int l)
{
  const uint32_t lo = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) x, l);
  const uint32_t hi = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) (x >> 32), l);
  return ((uint64_t) hi << 32) | lo;
}

// One TAS TX frame per 16-lane row: frame start at byte fo of the region
// (16-byte aligned; IPv4 at +14, TCP at +34), datagram length tl in
// [38, 1522] (the host checks both).  The arithmetic of tcp4_tas14_kernel's
// rows (xsum_kernels.hip tas14_finish, TX): lane gl holds chunks gl + 16u;
// chunk 2's first two bytes and tcp.chksum (chunk 3, bytes 2-3) masked, lane 1
// forms the IPv4 and pseudo-header channels with chunk 0's and chunk 2's
// dwords moved in by DPP, bytes past the datagram come off on lane 15 (its
// last load is the last chunk).  Returns false (no store) when the frame's own
// total_length is not tl: the frame changed after it was submitted.
template <int POL = kNt>
__device__ __forceinline__ bool srv_row(__amdgpu_buffer_rsrc_t rs, uint32_t fo, uint32_t tl, int gl)
{
  constexpr int U = 6;
  const uint32_t last = (14u + tl - 1u) >> 4, lastoff = fo + 16u * last;
  const uint32_t lo = fo + 16u * (uint32_t) gl;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, min(lo + 256u * u, lastoff), 0, POL);
  const uint32_t tail = 14u + tl - 16u * last; // bytes of the last chunk inside, 1..16
  const u32x4 h = v[0];
  const uint32_t m0 = gl == 2 ? 0xffff0000u : (gl == 3 ? 0x0000ffffu : 0xffffffffu);
  uint32_t acc = sad4(u32x4{h.x & m0, h.y, h.z, h.w}, 0u);
  acc = (gl < 2 || (uint32_t) gl > last) ? 0u : acc;
  const uint32_t c0d3 = row_shr<1>(h.w), c2d0 = row_shl<1>(h.x);
  const uint32_t addrs = sadw(h.z & 0xffff0000u, sadw(h.w, sadw(c2d0 & 0xffffu, 0u))); // src, dst
  const uint32_t ph = sadw(h.y & 0xff000000u, addrs);                                    // + proto
  const uint32_t ipsum = sadw(c0d3 & 0xffff0000u, sadw(h.x, sadw(h.y, addrs)));         // ip.chksum left out
  const uint32_t tlw = h.x & 0xffffu;
#pragma unroll
  for (int u = 1; u < U; ++u) {
    const uint32_t s = sad4(v[u], acc);
    acc = ((uint32_t) gl + 16u * u <= last) ? s : acc;
  }
  {
    uint32_t gm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = tail > 4u * j ? min(tail - 4u * j, 4u) : 0u;
      gm[j] = (uint32_t) (~0ull << (8u * k));
    }
    const u32x4 t = v[U - 1];
    const uint32_t g = sad4(u32x4{t.x & gm[0], t.y & gm[1], t.z & gm[2], t.w & gm[3]}, 0u);
    acc -= gl == 15 ? g : 0u;
  }
  acc = row_sum16(acc);
  const uint32_t ip15 = row_shr<14>(ipsum), ph15 = row_shr<14>(ph), tl15 = bswap16(row_shr<14>(tlw));
  const bool ok = tl15 == tl;
  if (gl == 15 && ok) {
    const uint32_t ipc = inv_result(residue(fold32_to_16(ip15)));
    const uint32_t r = fold32_to_16(acc) + fold32_to_16(ph15) + bswap16(tl - 20u);
    const uint32_t tcpc = inv_result(residue(fold32_to_16(r)));
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short) ipc, rs, fo + 24u, 0, kSys);  // ip.chksum
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short) tcpc, rs, fo + 50u, 0, kSys); // tcp.chksum
  }
  return ok;
}

// K = P.k workgroups serve ring r (context r): workgroup k takes the ring's
// positions p = k, k + K, k + 2K, ..., so one takes the ring's next batch
// while another sums the current one (one workgroup per ring summed its
// batches one after the other: 14-15 M frames/s at 8 threads x 7 in flight,
// profiles/r04/r04d), reading frames in turn (the read token, below), and
// each posts its own slot's done word.  Wave 0 polls the workgroup's next
// position: lanes read the 64 entry words, lanes 0-1 the two header words,
// lane 2 the control word, all system scope, in one round trip; a slot is
// taken when the header and every entry carry the position's tag.  After
// P.cold_ticks without a batch only the header and control words are read
// (16 + 8 bytes a poll instead of 528, about every 3 us): idle rings cost the
// PCIe link almost nothing, and the first batch after the lull pays one more
// round trip.  The other 15 waves wait at the barrier meanwhile (no issue
// slots).  Then row j sums frame j, and thread 0 posts done[p mod RING] =
// p + 1 after every wave's stores completed.
// Payload windows per lane in a TX segment row: 6 x 16 lanes x 16 B covers a
// 1448-byte payload's chunks in one PCIe round trip (3 took two: 15.5-15.8
// against 16.5-16.6 M segments/s at 8 x 3, 18.6-19.6 against 16.8-17.8 us at
// 1 x 1, profiles/r04/r04z); 128 VGPRs, no scratch.
constexpr int kSrvTxU = 6;

// The frame-load cache policies measured in round 4 (no acquire, system-scope
// loads, write-through TX stores, no release, ...; profiles/r04/INDEX.md
// r04g-r04v), the per-batch timing form (profiles/r05 r05h), the acquire at
// agent scope or left out for pricing (profiles/r05 r05l) and a workgroup
// taking its next queued slot under the same acquire (round 6, r06b: no
// effect on what a busy server costs other work) were measured against this
// form and are gone from the source.
__global__ __launch_bounds__(kSrvBlock) void flush_server_kernel(tasx_srv_params P)
{
  __shared__ uint32_t s_off[TASX_SRV_FB], s_tl[TASX_SRV_FB];
  __shared__ uint64_t s_w[TASX_SRV_WORDS]; // a TX segment slot's entry words
  __shared__ uint32_t s_cmd, s_n, s_bytes, s_bad, s_seg;
  __shared__ uint64_t s_base;
  const uint32_t K = P.k, r = blockIdx.x / K;
  const int lane = threadIdx.x & 63, gl = threadIdx.x & 15;
  uint8_t *const mem = P.mem;
  const uint8_t *const ring = P.ring;
  uint32_t *const dline = (uint32_t *) (mem + TASX_SRV_DONE(r));
  uint32_t *const tokw = P.tok + r * TASX_SRV_TOKW;
  if (threadIdx.x == 0)
    s_bad = 0u;
  __syncthreads();
  // a first launch starts on a zeroed block (every ring at position 0); a
  // resumed one (tasx_server_resume) where this workgroup left off
  uint32_t *const posw = (uint32_t *) (mem + TASX_SRV_POSW(blockIdx.x));
  uint32_t p = P.resume ? __hip_atomic_load(posw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : blockIdx.x % K;
  uint64_t *const tactw = (uint64_t *) (mem + TASX_SRV_TACT(blockIdx.x));
  const uint64_t t_launch = wall_clock64();
  // the last batch's time carries over from the previous epoch: an idle ring
  // stays on header-only polls across epochs (the wall clock is the device's)
  uint64_t t_act = P.resume ? __hip_atomic_load(tactw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : t_launch;
  // The poller's reads of ring r's slot at position p: the entry words (every
  // lane; skipped when only the header is polled), the two header words
  // (lanes 0-1) and the control word (lane 2), all in one round trip.
  struct SlotRead {
    uint64_t e, hw;
  };
  auto read_slot = [&](bool entries) {
    const uint8_t *slot = ring + TASX_SRV_SLOTP(r, p);
    SlotRead v;
    v.e = entries ? ld_sys64((const uint64_t *) (slot + TASX_SRV_HDR) + lane) : 0ull;
    v.hw = lane < 2    ? ld_sys64((const uint64_t *) slot + lane)
           : lane == 2 ? ld_sys64((const uint64_t *) (ring + TASX_SRV_CTL))
                       : 0ull;
    return v;
  };
  // A read of position p: 1 = the batch is complete (taken: its descriptors
  // into LDS), 0 = nothing yet, 2 = the header without all its entries (the
  // host still writing them, or a header-only poll: read the whole slot at
  // once), 3 = stop, 4 = the epoch is over
  auto judge = [&](const SlotRead &v, bool entries, uint64_t now) -> int {
    const uint64_t tag = (uint64_t) ((p + 1u) & 0xffffu);
    const uint64_t h0 = rlane64(v.hw, 0), h1 = rlane64(v.hw, 1), c = rlane64(v.hw, 2);
    const bool seg = (h0 & TASX_SRV_SEG) != 0u;
    const uint32_t n = (uint32_t) (h0 & 0x7fffu), words = seg ? TASX_SRV_SEGW0 + 3u * n : n;
    const bool hdr = (h0 >> 48) == tag && (h1 >> 48) == tag && n >= 1u && n <= (seg ? TASX_SRV_SEGS : TASX_SRV_FB);
    // the stop word first (a pause, a stop, an abort): a slot ready in this
    // very read is left in the ring, and posw records it for a resumed launch
    // (taking it first, a workgroup whose ring never runs empty would never
    // see the stop word: ADVICE r05)
    if ((uint32_t) c != 0u)
      return 3;
    // the epoch's end, checked before a slot is taken as well: the next
    // epoch, queued behind this launch, takes it (an epoch bounds how long a
    // device-wide synchronize or a free elsewhere in the process waits for
    // this kernel; server_epochs in tasx_host.c)
    if (now - t_launch >= P.period_ticks)
      return 4;
    // a header-only read never takes the slot: unread entries (0) would match
    // the tag of every position p with p + 1 = 0 mod 2^16
    if (hdr && entries && __builtin_amdgcn_ballot_w64((uint32_t) lane < words && (v.e >> 48) != tag) == 0ull) {
      if ((uint32_t) lane < words) {
        s_off[lane] = (uint32_t) v.e;
        s_tl[lane] = (uint32_t) (v.e >> 32) & 0xffffu;
        s_w[lane] = v.e;
      }
      // a TX slot's entries past the first 64: the host wrote them before
      // the header this read saw, so one more round trip has them all
      // (tagged all the same; a mismatch is read again)
      bool torn = false;
      if (words > TASX_SRV_FB) {
        const uint64_t *e2 = (const uint64_t *) (ring + TASX_SRV_SLOTP(r, p) + TASX_SRV_HDR) + TASX_SRV_FB;
        const bool mine = (uint32_t) lane < words - TASX_SRV_FB;
        uint64_t w2 = 0ull;
        torn = true;
        for (int t = 0; t < 64 && torn; ++t) { // bounded: a host that broke the protocol ends up flagged
          w2 = mine ? ld_sys64(e2 + lane) : 0ull;
          torn = __builtin_amdgcn_ballot_w64(mine && (w2 >> 48) != tag) != 0ull;
        }
        if (mine)
          s_w[TASX_SRV_FB + lane] = w2;
      }
      if (lane == 0) {
        s_seg = seg ? 1u : 0u;
        s_n = torn ? 0u : n; // a slot still torn is not built, and flags the ring
        if (torn)
          s_bad = 1u;
        s_bytes = (uint32_t) (h0 >> 16);
        s_base = h1 & 0xffffffffffffull;
      }
      t_act = wall_clock64();
      return 1;
    }
    return hdr ? 2 : 0;
  };
  for (;;) {
    if (threadIdx.x < 64) {
      bool entries = true;
      int st;
      // the wall clock is read every 8th empty poll (s_memrealtime is a
      // memory-path message, not a register read)
      uint64_t now = wall_clock64();
      for (uint32_t np = 1;; ++np) {
        st = judge(read_slot(entries), entries, now);
        if (st == 1 || st >= 3)
          break;
        entries = true;
        if (st == 2)
          continue; // the header is in: read the whole slot again at once
        if ((np & 7u) == 0u)
          now = wall_clock64();
        const uint64_t idle = now - t_act;
        if (idle >= P.cold_ticks) {
          entries = false;
          __builtin_amdgcn_s_sleep(127);
        } else if (idle >= P.hot_ticks) {
          __builtin_amdgcn_s_sleep(32);
        } else {
          __builtin_amdgcn_s_sleep(1);
        }
      }
      // The ring's read token (K > 1): the workgroups of a ring poll and take
      // their positions independently, but read frames one position at a
      // time, in ring order -- a busy server's frame reads in flight through
      // the XCDs' L2s are what it costs device-resident work on the same GPU
      // (profiles/r06/INDEX.md r06d).  The slot has only been read (nothing
      // is posted before its rows ran), so a stop or the epoch's end while
      // waiting leaves it in the ring for the next launch, as in judge().
      if (st == 1 && K > 1u) {
        for (uint32_t sp = 1;; ++sp) {
          if (__hip_atomic_load(tokw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p)
            break;
          if ((sp & 7u) == 0u) {
            if ((uint32_t) ld_sys64((const uint64_t *) (ring + TASX_SRV_CTL)) != 0u) {
              st = 3;
              break;
            }
            if (wall_clock64() - t_launch >= P.period_ticks) {
              st = 4;
              break;
            }
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (lane == 0)
        s_cmd = st == 1 ? 0u : st == 3 ? 1u : 2u;
      // a batch taken: this CU's L1 and the XCD's L2 drop
      // their non-coherent lines before any frame load
      if (st == 1)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    if (s_cmd != 0u) {
      if (threadIdx.x == 0) { // the position polled and not taken: where the next launch starts
        st_sys32(posw, p);
        st_sys64(tactw, t_act);
      }
      break;
    }
    const uint32_t row = threadIdx.x >> 4;
    if (s_seg) {
      // TX segment slot: row r builds segment r (payload gathered from the
      // app's TX buffer into the frame, both checksums stored): the general
      // row of the TX segment build (txseg_device.h), over PCIe both ways
      if (row < s_n) {
        const uint64_t wa = s_w[TASX_SRV_SEGW0 + 3 * row], wb = s_w[TASX_SRV_SEGW0 + 1 + 3 * row],
                       wc = s_w[TASX_SRV_SEGW0 + 2 + 3 * row];
        const uint32_t hl = (uint32_t) s_w[2] & 0xffffu, room16 = (uint32_t) (s_w[2] >> 16) & 0xffffu;
        const uint32_t tx_len = ((uint32_t) (wb >> 32) & 0xffffu) | (((uint32_t) (wc >> 32) & 0xffffu) << 16);
        const u32x4 d0 = u32x4{(uint32_t) wa, 0u, (uint32_t) wc, 0u};
        const u32x4 d1 = u32x4{tx_len, (uint32_t) wb, ((uint32_t) (wa >> 32) & 0xffffu) | (hl << 16),
                               (room16 & 0x7fffu) | ((room16 & 0x8000u) ? 0x80000000u : 0u)};
        tasx_txseg_params tp;
        tp.shm = (const uint8_t *) (uintptr_t) (s_w[0] & 0xffffffffffffull);
        tp.shm_len = (uint32_t) s_w[1];
        tp.frames = (uint8_t *) (uintptr_t) s_base;
        tp.segs = nullptr;
        tp.out = nullptr;
        tp.n = s_n;
        tp.ip_off = (uint32_t) (s_w[1] >> 32) & 0xffu;
        tp.l4_off = (uint32_t) (s_w[1] >> 40) & 0xffu;
        // reads stay inside the region the host validated the frame against
        // (s_bytes from the frame region's start, the frame 16-byte aligned in it)
        const uint32_t rb = s_bytes > (uint32_t) wa ? s_bytes - (uint32_t) wa : 0u;
        const bool good = txseg_row_d<kSrvTxU, false>(tp, row, d0, d1, gl, rb);
        if (gl == 15 && !good) // total_length changed since submission: frame left alone, ring flagged
          atomicOr(&s_bad, 1u);
      }
    } else if (row < s_n) {
      const uint64_t base = s_base;
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *) (uintptr_t) base, 0, (int) s_bytes,
                                                                    (int) kRsrcWord3);
      const uint32_t fo = s_off[row], tl = s_tl[row];
      bool ok = (fo & 15u) == 0u && tl >= 38u && tl <= 1522u;
      ok = ok && srv_row(rs, fo, tl, gl);
      if (gl == 15 && !ok)
        atomicOr(&s_bad, 1u);
    }
    if (K > 1u) {
      // every row has issued its stores, and a store is issued only once the
      // loads it is made of have landed: the ring's next position may read
      // while these stores are still on their way (a barrier without a
      // memory fence: nothing here waits for them)
      __builtin_amdgcn_s_barrier();
      // (by the last wave: its rows are past every batch TAS flushes, 32
      // frames or 41 segments, so the wait for its own memory operations the
      // compiler puts before the store has nothing to wait for)
      if (threadIdx.x == kSrvBlock - 1)
        __hip_atomic_store(tokw, p + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this wave's field stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
      if (s_seg) // the TX build's plain stores: every dirty line out of the L2 before the done word
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if (s_bad) { // sticky in the ring's line: a frame changed after submission (or a malformed slot)
        st_sys32(dline + TASX_SRV_ERRW, 1u);
        s_bad = 0u; // (the rows of the next batch set it only after the next barrier)
      }
      st_sys32(dline + p % TASX_SRV_RING, p + 1u);
    }
    p += K;
  }
}

} // namespace

#endif
