// txseg_device.h -- the general TX segment row (SURVEY.md section 8f row 1:
// flow_tx_read + tcp_checksums of flow_tx_segment,
// /root/reference/tas/fast/fast_flows.c:833-846, :930-936) and the byte
// helpers it needs, shared by txseg_kernels.hip (tx_segment_u_kernel and the
// fallback rows of the TAS-layout kernels) and server_kernels.hip (the flush
// server's TX segment slots).  Include after tasx_kernels.h and
// xsum_device.h.
#pragma once

namespace {

// byte b of v set to x (no-op unless 0 <= b < 16)
__device__ __forceinline__ u32x4 put_byte(u32x4 v, int b, uint32_t x)
{
  const uint32_t sh = 8u * (uint32_t) (b & 3), m = ~(0xffu << sh), y = (x & 0xffu) << sh;
  const int j = b >> 2;
  return u32x4{j == 0 ? (v.x & m) | y : v.x, j == 1 ? (v.y & m) | y : v.y, j == 2 ? (v.z & m) | y : v.z,
               j == 3 ? (v.w & m) | y : v.w};
}

// store bytes [lo, hi) of v into the 16-byte aligned chunk at cp: whole
// dwords as dword stores, the rest as byte stores (constant offsets from one
// address)
// write-through (sc0 sc1) vector stores: they reach host memory without an
// L2 write-back (the flush server's TX segment slots)
__device__ __forceinline__ void wt_store16(uint8_t *p, u32x4 v)
{
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void wt_store4(uint8_t *p, uint32_t v)
{
  asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void wt_store1(uint8_t *p, uint32_t v)
{
  asm volatile("global_store_byte %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// store_range with write-through stores
__device__ __forceinline__ void store_range_wt(uint8_t *cp, u32x4 v, int lo, int hi)
{
  if (lo >= hi)
    return;
  if (lo == 0 && hi == 16) {
    wt_store16(cp, v);
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (lo <= 4 * j && 4 * j + 4 <= hi) {
      wt_store4(cp + 4 * j, w[j]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * j + q >= lo && 4 * j + q < hi)
          wt_store1(cp + 4 * j + q, w[j] >> (8 * q));
    }
  }
}

__device__ __forceinline__ void store_range(uint8_t *cp, u32x4 v, int lo, int hi, bool nt = true)
{
  if (lo >= hi)
    return;
  if (lo == 0 && hi == 16) {
    if (nt)
      __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *) cp);
    else
      *(__attribute__((address_space(1))) u32x4 *) cp = v;
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (lo <= 4 * j && 4 * j + 4 <= hi) {
      stg((uint32_t *) cp, (uint32_t) j, w[j]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * j + q >= lo && 4 * j + q < hi)
          st8(cp + 4 * j + q, w[j] >> (8 * q));
    }
  }
}


// bytes [lo, hi) of ins, the rest of base (lo, hi in [0, 16])
__device__ __forceinline__ u32x4 splice(u32x4 base, u32x4 ins, int lo, int hi)
{
  uint64_t l0, l1, h0, h1;
  below_mask((uint32_t) min(max(lo, 0), 16), l0, l1);
  below_mask((uint32_t) min(max(hi, 0), 16), h0, h1);
  const uint64_t m0 = h0 & ~l0, m1 = h1 & ~l1;
  const uint32_t m[4] = {(uint32_t) m0, (uint32_t) (m0 >> 32), (uint32_t) m1, (uint32_t) (m1 >> 32)};
  return u32x4{(ins.x & m[0]) | (base.x & ~m[0]), (ins.y & m[1]) | (base.y & ~m[1]),
               (ins.z & m[2]) | (base.z & ~m[2]), (ins.w & m[3]) | (base.w & ~m[3])};
}

// word sum of bytes [lo, hi) of v (lo, hi in [0, 16])
__device__ __forceinline__ uint32_t sad_range(u32x4 v, int lo, int hi)
{
  uint64_t l0, l1, h0, h1;
  below_mask((uint32_t) min(max(lo, 0), 16), l0, l1);
  below_mask((uint32_t) min(max(hi, 0), 16), h0, h1);
  const uint64_t m0 = h0 & ~l0, m1 = h1 & ~l1;
  return sad4(u32x4{v.x & (uint32_t) m0, v.y & (uint32_t) (m0 >> 32), v.z & (uint32_t) m1,
                    v.w & (uint32_t) (m1 >> 32)}, 0u);
}

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4u gcu4u;

// 16 bytes at any byte offset (global_load_dwordx4 at an unaligned address),
// non-temporal: payload windows are read once (-2% on the TX build)
__device__ __forceinline__ u32x4 ld16u(const uint8_t *base, uint32_t off)
{
  const u32x4u v = __builtin_nontemporal_load((gcu4u *) (base + off)); // read once
  return u32x4{v.x, v.y, v.z, v.w};
}

// the window at shm offset `off` byte by byte; bytes outside [0, shm_len) as 0
__device__ __noinline__ u32x4 gather16(const uint8_t *shm, uint32_t off, uint64_t shm_len)
{
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  for (int b = 0; b < 16; ++b) {
    const uint32_t a = off + (uint32_t) b;
    if (a < shm_len)
      w[b >> 2] |= ld8(shm + a) << (8 * (b & 3));
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

// segment i on the 16 lanes of one DPP row (lane gl); any frame layout
// The descriptor (tasx_tx_seg, two 16-byte words) is passed in: txseg_row
// below loads it from p.segs; the flush server (server_kernels.hip) decodes it
// from its ring slot.  rbound: the bytes from the frame start the row may read
// (whole chunks); a frame whose ip.total_length reaches past its written bytes
// and past rbound is left untouched and the row returns false (the server's
// frames were validated against their region when submitted: a total_length
// changed since then must not make the row read beyond the region).  Every
// other row returns true, those dma_read() rejects (frame untouched) included.
template <int U, bool NTS, bool WT = false>
__device__ __forceinline__ bool txseg_row_d(const tasx_txseg_params &p, uint32_t i, u32x4 d0, u32x4 d1, int gl,
                                            uint32_t rbound = 0xffffffffu)
{
  const uint64_t frame_off = d0.x | ((uint64_t) d0.y << 32);
  const uint64_t tx_base = d0.z | ((uint64_t) d0.w << 32);
  const uint32_t tx_len = d1.x, pos = d1.y, pay_ = d1.z & 0xffffu, hl_ = d1.z >> 16;
  const bool ok = (pay_ == 0 || pos < tx_len) && pay_ <= tx_len && tx_base <= p.shm_len &&
                  tx_len <= p.shm_len - tx_base && hl_ >= p.l4_off + 20;
  if (!ok) {
    if (gl == 15 && p.out)
      stg(p.out, i, 0u);
    return true;
  }
  uint8_t *const f = p.frames + frame_off;
  uint8_t *const ip = f + p.ip_off;
  const int fh = (int) ((uintptr_t) f & 15);
  uint8_t *const c0 = f - fh;
  const int hl = (int) hl_, pay = (int) pay_, fend = hl + pay;
  // chunks: [0, nhc) hold header bytes, [nhc, kpay) are whole payload chunks,
  // [kpay, K) the partial last one
  const int K = (fh + fend + 15) >> 4, nhc = (fh + hl + 15) >> 4, kpay = max((fh + fend) >> 4, nhc);
  // TX buffer pieces (32-bit shm offsets, modular)
  const uint8_t *const shm = p.shm;
  const uint32_t s1 = (uint32_t) (tx_base + pos), s2 = s1 - tx_len;
  const int wrap = (int) tx_len - (int) pos;
  const bool wraps = pay > 0 && wrap < pay;
  const uint32_t smax = (uint32_t) (p.shm_len - 16u);
  auto woff = [&](int j0) -> uint32_t { return (wraps && j0 >= wrap ? s2 : s1) + (uint32_t) j0; };
  // the chunk holding payload index `wrap` (not on a chunk boundary) and its piece-2 window
  const bool straddle = wraps && ((fh + hl + wrap) & 15);
  const int ks = straddle ? (fh + hl + wrap) >> 4 : -1;
  const uint32_t xoff = straddle ? s2 + (uint32_t) (16 * ks - fh - hl) : woff(16 * nhc - fh - hl);

  // ---- up-front loads: IPv4 header words, total_length, this lane's header
  // chunk, its boundary chunk's window, the straddle chunk's piece-2 window
  const uint32_t tl = (ld8(ip + 2) << 8) | ld8(ip + 3);
  // (the row's lanes agree: one uniform load)
  const bool tl_ok = p.ip_off + tl <= (uint32_t) fend || ((p.ip_off + tl + 15u) & ~15u) <= rbound;
  const int wl = min(gl, 9);
  const uint32_t w_ = ld8(ip + 2 * wl) | (ld8(ip + 2 * wl + 1) << 8);
  const uint32_t w = gl < 10 ? w_ : 0u;
  const u32x4 hv = ld16((const u32x4 *) c0, (uint32_t) min(gl, nhc - 1));
  // boundary entries: b < nhc header chunk b, b == nhc the straddle chunk,
  // b == nhc + 1 the partial last chunk
  const int bk0 = gl < nhc ? gl : gl == nhc ? ks : kpay;
  // (nothing below uses total_length before the whole-chunk loads are issued:
  // the loads above and the loop's loads share one memory latency)
  const int bkc = min(max(bk0, 0), K - 1);
  const uint32_t boff = woff(16 * bkc - fh - hl);
  const u32x4 bw = ld16u(shm, min(boff, smax));
  const u32x4 xw = ld16u(shm, min(xoff, smax));

  // ---- whole payload chunks [nhc, kpay) but the straddle chunk: U unaligned
  // window loads per lane, then stores and sums from the registers.  Lanes own
  // chunks by address, so each store instruction covers whole 256-byte blocks.
  uint32_t acc = 0;
  const int aoff = (int) (((uintptr_t) c0 >> 4) & 15u);
  for (int base = nhc - ((nhc + aoff) & 15); base < kpay; base += 16 * U) {
    u32x4 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(max(base + gl + 16 * u, nhc), kpay - 1);
      a[u] = ld16u(shm, min(woff(16 * k - fh - hl), smax));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + gl + 16 * u;
      const bool in = k >= nhc && k < kpay && k != ks;
      if (in && tl_ok) {
        uint8_t *const cp = c0 + 16 * k;
        if (WT)
          wt_store16(cp, a[u]);
        else if (NTS)
          __builtin_nontemporal_store(a[u], (__attribute__((address_space(1))) u32x4 *) cp);
        else
          *(__attribute__((address_space(1))) u32x4 *) cp = a[u];
      }
      const uint32_t t = sad4(a[u], acc);
      acc = in ? t : acc;
    }
  }
  if (!tl_ok) {
    if (gl == 15 && p.out)
      stg(p.out, i, 0u);
    return false;
  }
  const uint32_t len = tl >= 20 ? tl - 20 : 0;
  const int sum_lo = (int) p.l4_off, sum_end = sum_lo + (int) len, sum_hi = min(sum_end, fend);
  const int ck = (int) p.l4_off + 16 + fh; // tcp.chksum's chunk-grid position
  // total_length ends inside the whole payload chunks (never for flow_tx_segment's
  // frames, :897): take their bytes from sum_hi on back off
  for (int k = max((fh + sum_hi) >> 4, nhc) + gl; k < kpay; k += 16) {
    if (k == ks)
      continue;
    const int o = 16 * k - fh;
    acc -= sad_range(ld16u(shm, woff(o - hl)), sum_hi - o, 16);
  }

  // ---- boundary chunks (generic; one entry per lane in the common case)
  u32x4 vh = hv;
  for (int b = gl; b < nhc + 2; b += 16) {
    int k;
    if (b < nhc)
      k = b;
    else if (b == nhc)
      k = (straddle && ks >= nhc && ks < kpay) ? ks : -1;
    else
      k = kpay < K ? kpay : -1;
    if (k < 0)
      continue;
    const int o = 16 * k - fh, j0 = o - hl;
    u32x4 v;
    if (pay > 0 && o + 16 > hl && o < fend) { // payload bytes [hl - o, fend - o) of this chunk
      const uint32_t off = woff(j0);
      u32x4 win = (b == gl && k == bk0 && off <= smax) ? bw : (off <= smax ? ld16u(shm, off) : gather16(shm, off, p.shm_len));
      if (k == ks)
        win = splice(win, xoff <= smax ? xw : gather16(shm, xoff, p.shm_len), wrap - j0, 16);
      v = win;
      if (k < nhc)
        v = splice(b < 16 ? hv : ld16((const u32x4 *) c0, (uint32_t) k), win, hl - o, fend - o);
    } else {
      v = b < 16 ? hv : ld16((const u32x4 *) c0, (uint32_t) k);
    }
    u32x4 sv = v;
    if (k < nhc) { // tcp.chksum taken as zero
      sv = put_byte(sv, ck - 16 * k, 0u);
      sv = put_byte(sv, ck + 1 - 16 * k, 0u);
    }
    acc += sad_range(sv, sum_lo - o, sum_hi - o);
    if (b < 16 && k < nhc)
      vh = v; // written back with the checksums at the end
    else
      if (WT)
        store_range_wt(c0 + 16 * k, v, max(-o, 0), min(fend - o, 16));
      else
        store_range(c0 + 16 * k, v, max(-o, 0), min(fend - o, 16), false);
  }
  uint32_t part = acc;
  if (sum_end > fend) { // total_length reaches past the frame's written bytes
    const Chunks<U> t = chunk_range<U>(f + fend, (uint32_t) (sum_end - fend));
    part += group_lane_sum<U>(t, gl);
  }
  const uint32_t c_ip = (gl < 10 && gl != 5) ? w : 0u;
  const uint32_t c_ph = (gl >= 6 && gl < 10) ? w : (gl == 4 ? (w & 0xff00u) : 0u);
  part = row_sum16(part);
  const uint32_t s_ip = row_sum16(c_ip), s_ph = row_sum16(c_ph);
  const uint32_t ipc = inv_result(residue(fold32_to_16(s_ip)));
  uint32_t tcpc = 0;
  if (tl >= 20) {
    uint32_t r4 = fold32_to_16(part);
    if ((fh + (int) p.l4_off) & 1)
      r4 = bswap16(r4);
    tcpc = inv_result(residue(fold32_to_16(r4 + s_ph + bswap16(len))));
  }
  const uint32_t res = (uint32_t) __shfl((int) (ipc | (tcpc << 16)), (int) ((threadIdx.x & 63u) | 15u), 64);
  if (gl == 15 && p.out)
    stg(p.out, i, res);
  // header write-back: frame bytes [0, min(hdrs_len, frame end)) of chunk gl, checksums inserted
  if (gl < nhc) {
    const int b0 = 16 * gl, fi = (int) p.ip_off + 10 + fh;
    u32x4 v = put_byte(vh, fi - b0, res);
    v = put_byte(v, fi + 1 - b0, res >> 8);
    v = put_byte(v, ck - b0, res >> 16);
    v = put_byte(v, ck + 1 - b0, res >> 24);
    if (WT)
      store_range_wt(c0 + b0, v, max(fh - b0, 0), min(fh + fend - b0, 16));
    else
      store_range(c0 + b0, v, max(fh - b0, 0), min(fh + fend - b0, 16), false);
  }
  return true;
}

template <int U, bool NTS>
__device__ __forceinline__ void txseg_row(const tasx_txseg_params &p, uint32_t i, int gl)
{
  (void) txseg_row_d<U, NTS>(p, i, ld16((const u32x4 *) p.segs, 2 * i), ld16((const u32x4 *) p.segs, 2 * i + 1), gl);
}


} // namespace
