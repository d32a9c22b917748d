"""GPU parity of the round-3 host surfaces, bit-exact against the C oracle:

* tasx_tcp4_cksum_batch_host_offs / tasx_raw_cksum_batch_host_offs -- host
  packets scattered over a buffer the way TAS's mbufs lie in their per-core
  mempool (tas/fast/network.c:320-330): shuffled offsets, odd starts, mixed and
  TSO lengths, staged (CPU gather -> H2D -> kernel -> D2H) and zero-copy
  (the GPU reads the packets in place), slots small enough that every batch
  runs as many pipelined chunks;
* the feeder ordering rule: a batch the context flushes
  itself, then a feeder batch, with no poll in between;
* flush tickets across the 2^32 wrap (A/B test hook);
* RX received lengths beyond the stride slot;
* (round 4) errors found before any chunk is launched leave the
  context usable; forged total_length and zero-copy extents refused; other
  header layouts through all three forms.
"""
import numpy as np
import pytest
import torch

from tas_amd import pktgen, xsum

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    xsum.lib()
    yield
    torch.cuda.synchronize()


def _scatter(packets: list, seed: int, shifted: bool, pinned: bool):
    """Place packets (uint8 arrays) in one buffer in shuffled order, each at a
    64-byte aligned start (from the page-aligned or numpy base) or, shifted, at
    a random byte shift past it, with 16 bytes of slack after each (zero-copy
    kernels read whole 16-byte chunks).  Returns (buffer array, base address,
    offsets u64, pinned handle or None)."""
    rng = np.random.default_rng(seed)
    order = rng.permutation(len(packets))
    offs = np.zeros(len(packets), np.uint64)
    pos = 0
    for k in order:
        pos = (pos + 63) // 64 * 64 + (int(rng.integers(0, 64)) if shifted else 0)
        offs[k] = pos
        pos += len(packets[k]) + 16
    size = pos + 64
    pin = None
    if pinned:
        pin = xsum.PinnedBuffer(size)
        buf, base = pin.array, pin.addr
        buf[:] = rng.integers(0, 256, size, dtype=np.uint8)
    else:
        buf = rng.integers(0, 256, size, dtype=np.uint8)
        base = buf.ctypes.data
    for k, p in enumerate(packets):
        buf[int(offs[k]):int(offs[k]) + len(p)] = p
    return buf, base, offs, pin


@pytest.mark.parametrize("zerocopy", [False, True])
@pytest.mark.parametrize("form", ["lengths", "len0"])
def test_raw_host_offs(oracle, zerocopy, form):
    """rte_raw_cksum over scattered host packets: lengths 0..9001 (odd ones,
    the mixed-MTU sizes), odd starts; a 256 KiB slot makes many chunks."""
    n = 3000
    rng = np.random.default_rng(7 + zerocopy)
    if form == "lengths":
        lens = pktgen.mixed_lengths(n, seed=11).astype(np.int64)
        lens[::7] += 1                                   # odd tails
        lens[:40] = np.arange(40)                       # empty and short packets
        lens[40] = 9001
    else:
        lens = np.full(n, 1500, np.int64)
    pk = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in lens]
    buf, base, offs, pin = _scatter(pk, 13 + zerocopy, True, zerocopy)
    exp = oracle.raw_batch(buf, n, offsets=offs, lengths=lens.astype(np.uint32))
    ctx = 4
    xsum.ctx_init(ctx, 0, (16 << 10) if zerocopy else (256 << 10))  # many chunks either way
    try:
        if form == "lengths":
            got = xsum.raw_cksum_batch_host_offs(ctx, base, offs, n, lengths=lens.astype(np.uint32),
                                                 zerocopy=zerocopy)
        else:
            got = xsum.raw_cksum_batch_host_offs(ctx, base, offs, n, len0=1500, zerocopy=zerocopy)
        np.testing.assert_array_equal(got, exp)
        if not zerocopy:  # absolute addresses (base NULL)
            got = xsum.raw_cksum_batch_host_offs(ctx, None, offs + np.uint64(base), n,
                                                 lengths=lens.astype(np.uint32))
            np.testing.assert_array_equal(got, exp)
    finally:
        xsum.ctx_destroy(ctx)
        if pin is not None:
            pin.free()


def _tcp4_packets(n: int, seed: int, tso: bool):
    rng = np.random.default_rng(seed)
    if tso:
        frames = pktgen.tcp4_frames(n, payload=0, stride=65552, seed=seed, ip_total_len=65535)
        flen = np.full(n, 14 + 65535, np.uint32)
        return [frames[i * 65552:i * 65552 + 14 + 65535] for i in range(n)], flen
    pay = np.where(rng.random(n) < 0.4, 0, rng.integers(1, pktgen.TCP_MSS + 1, n)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=seed)
    f = frames.reshape(n, 2048)
    short = np.arange(3, n, 101)
    tl = (np.arange(len(short)) * 7) % 61                     # total_length 0..60: general bodies
    f[short, 16], f[short, 17] = tl >> 8, tl & 0xFF
    flen = (14 + (f[:, 16].astype(np.int64) << 8 | f[:, 17])).clip(14 + 38, 2048).astype(np.uint32)
    return [f[i, :max(int(flen[i]), 14 + 38)].copy() for i in range(n)], flen


@pytest.mark.parametrize("zerocopy", [False, True])
@pytest.mark.parametrize("kind", ["mix", "tso", "uniform"])
@pytest.mark.parametrize("shifted", [False, True])
def test_tcp4_host_offs(oracle, zerocopy, kind, shifted):
    """tcp_checksums() over scattered host frames: data/ACK mixes with short
    total_length, TSO segments (ip.len 65535), a uniform MTU batch (stride-mode
    records); frame starts 64-byte aligned (TAS rows) or at random byte shifts
    (general rows when zero-copy); out of place and in place; with and without
    frame-length hints; slots small enough for several chunks."""
    n = {"mix": 2500, "tso": 24, "uniform": 2000}[kind]
    if kind == "uniform":
        frames = pktgen.tcp4_frames(n, payload=1448, stride=2048, seed=23)
        pk = [frames[i * 2048:i * 2048 + 1514] for i in range(n)]
        flen = np.full(n, 1514, np.uint32)
    else:
        pk, flen = _tcp4_packets(n, 29 + (kind == "tso"), kind == "tso")
    buf, base, offs, pin = _scatter(pk, 31 + zerocopy, shifted, zerocopy)
    if not shifted:
        assert np.all((offs + np.uint64(base)) % np.uint64(16) == 0)
    ref = buf.copy()
    exp = oracle.tcp4_batch(ref, n, offsets=offs, inplace=True)
    ctx = 5
    # several chunks even for the TSO batch (staged: 7 records of 65552 B per
    # 512 KiB slot; zero-copy: 1025 descriptors per 64 KiB slot)
    xsum.ctx_init(ctx, 0, (64 << 10) if zerocopy else (512 << 10))
    try:
        got = xsum.tcp4_cksum_batch_host_offs(ctx, base, offs, n, zerocopy=zerocopy)
        np.testing.assert_array_equal(got, exp)
        got = xsum.tcp4_cksum_batch_host_offs(ctx, base, offs, n, frame_len=flen, zerocopy=zerocopy)
        np.testing.assert_array_equal(got, exp)
        xsum.tcp4_cksum_batch_host_offs(ctx, base, offs, n, out=False, inplace=True, zerocopy=zerocopy)
        np.testing.assert_array_equal(buf, ref)
    finally:
        xsum.ctx_destroy(ctx)
        if pin is not None:
            pin.free()


def test_host_offs_errors():
    ctx = 7
    xsum.ctx_init(ctx, 0, 1 << 16)
    try:
        offs = np.zeros(4, np.uint64)
        pk = np.zeros(4096, np.uint8)
        with pytest.raises(xsum.TasxError):   # zero-copy of pageable memory
            xsum.raw_cksum_batch_host_offs(ctx, pk.ctypes.data, offs, 4, len0=64, zerocopy=True)
        with pytest.raises(xsum.TasxError):   # zero-copy needs a base
            xsum.raw_cksum_batch_host_offs(ctx, None, offs, 4, len0=64, zerocopy=True)
        with pytest.raises(xsum.TasxError):   # a packet larger than the slot
            xsum.raw_cksum_batch_host_offs(ctx, pk.ctypes.data, offs, 1, lengths=np.array([70000], np.uint32))
        with pytest.raises(xsum.TasxError):   # beyond TASX_RAW_MAX_LEN
            xsum.raw_cksum_batch_host_offs(ctx, pk.ctypes.data, offs, 1, lengths=np.array([200000], np.uint32))
        with pytest.raises(xsum.TasxError):   # a TSO frame does not fit a 64 KiB slot
            big = pktgen.tcp4_frames(1, payload=0, stride=65552, ip_total_len=65535)
            xsum.tcp4_cksum_batch_host_offs(ctx, big.ctypes.data, offs, 1)
    finally:
        xsum.ctx_destroy(ctx)


def test_host_offs_error_leaves_context_usable(oracle):
    """a batch whose LAST frame does not fit a slot is
    refused before anything is launched (staged TCP4 and RAW), and the same
    context then runs a normal multi-chunk batch and a flush bit-exact."""
    ctx = 6
    xsum.ctx_init(ctx, 0, 1 << 16)                      # 43 MTU records per 64 KiB slot
    try:
        n = 200
        frames = pktgen.tcp4_frames(n, payload=(np.arange(n) * 31) % 1449, stride=2048, seed=61)
        big = pktgen.tcp4_frames(1, payload=0, stride=65552, ip_total_len=65535)
        buf = np.concatenate([frames, big])
        offs = np.arange(n, dtype=np.uint64) * np.uint64(2048)
        offs[-1] = frames.size                           # frame n - 1 is the TSO frame: 65,552 B records
        with pytest.raises(xsum.TasxError):
            xsum.tcp4_cksum_batch_host_offs(ctx, buf.ctypes.data, offs, n)
        lens = np.full(n, 1500, np.uint32)
        lens[-1] = 70000
        with pytest.raises(xsum.TasxError):
            xsum.raw_cksum_batch_host_offs(ctx, buf.ctypes.data, offs, n, lengths=lens)
        good = np.arange(n, dtype=np.uint64) * np.uint64(2048)
        ref = frames.copy()
        exp = oracle.tcp4_batch(ref, n, offsets=good, inplace=True)
        got = xsum.tcp4_cksum_batch_host_offs(ctx, frames.ctypes.data, good, n)
        np.testing.assert_array_equal(got, exp)
        exp_raw = oracle.raw_batch(frames, n, offsets=good, lengths=np.full(n, 1500, np.uint32))
        np.testing.assert_array_equal(
            xsum.raw_cksum_batch_host_offs(ctx, frames.ctypes.data, good, n, len0=1500), exp_raw)
        for i in range(32):
            xsum.tcp_checksums(ctx, frames.ctypes.data + i * 2048)
        xsum.tx_flush(ctx)
        np.testing.assert_array_equal(frames[:32 * 2048], ref[:32 * 2048])
    finally:
        xsum.ctx_destroy(ctx)


def test_host_offs_forged_total_length_and_extents():
    """with frame lengths given, a staged frame whose
    ip_off + total_length exceeds its length is refused (the gather would read
    past the mbuf); a zero-copy batch whose packets reach past the pinned
    allocation (or the registered region) is refused instead of faulting."""
    ctx = 8
    xsum.ctx_init(ctx, 0, 1 << 20)
    pin = xsum.PinnedBuffer(64 * 2048)
    try:
        frames = pktgen.tcp4_frames(64, payload=100, stride=2048, seed=71)
        pin.array[:] = frames
        offs = np.arange(64, dtype=np.uint64) * np.uint64(2048)
        flen = np.full(64, 14 + 52 + 100, np.uint32)
        xsum.tcp4_cksum_batch_host_offs(ctx, pin.addr, offs, 64, frame_len=flen)
        forged = frames.copy()
        forged[9 * 2048 + 16], forged[9 * 2048 + 17] = 0xFF, 0xF0          # total_length 65,520
        with pytest.raises(xsum.TasxError):
            xsum.tcp4_cksum_batch_host_offs(ctx, forged.ctypes.data, offs, 64, frame_len=flen)
        xsum.register_frames(ctx, pin.addr, pin.nbytes)
        far = offs.copy()
        far[-1] = np.uint64(pin.nbytes + (1 << 20))
        with pytest.raises(xsum.TasxError):
            xsum.tcp4_cksum_batch_host_offs(ctx, pin.addr, far, 64, frame_len=flen, zerocopy=True)
        with pytest.raises(xsum.TasxError):
            xsum.raw_cksum_batch_host_offs(ctx, pin.addr, far, 64, len0=1500, zerocopy=True)
        # the context still works
        xsum.tcp4_cksum_batch_host_offs(ctx, pin.addr, offs, 64, frame_len=flen, zerocopy=True)
    finally:
        xsum.ctx_destroy(ctx)
        pin.free()


@pytest.mark.parametrize("ip_off,l4_off", [(18, 42), (0, 24), (22, 46)])
def test_host_offs_other_layouts(oracle, ip_off, l4_off):
    """staged, zero-copy and the device-resident batch agree
    with the oracle for ip_off != 14 and l4_off = ip_off + 24 (IP options),
    data and short segments, out of place and in place."""
    n, stride = 700, 2048
    rng = np.random.default_rng(ip_off * 7 + l4_off)
    buf0 = rng.integers(0, 256, n * stride, dtype=np.uint8)
    f = buf0.reshape(n, stride)
    tl = rng.integers(20, 1500, n)
    tl[::9] = rng.integers(0, 20, len(tl[::9]))               # total_length < 20: tcp.chksum 0
    f[:, ip_off + 2], f[:, ip_off + 3] = tl >> 8, tl & 0xFF
    offs = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    ref = buf0.copy()
    exp = oracle.tcp4_batch(ref, n, offsets=offs, ip_off=ip_off, l4_off=l4_off, inplace=True)
    ctx = 10
    xsum.ctx_init(ctx, 0, 256 << 10)
    pin = xsum.PinnedBuffer(buf0.size)
    try:
        for zc in (False, True):
            b = buf0.copy() if not zc else None
            if zc:
                pin.array[:] = buf0
            base = pin.addr if zc else b.ctypes.data
            got = xsum.tcp4_cksum_batch_host_offs(ctx, base, offs, n, ip_off=ip_off, l4_off=l4_off, zerocopy=zc)
            np.testing.assert_array_equal(got, exp)
            xsum.tcp4_cksum_batch_host_offs(ctx, base, offs, n, out=False, inplace=True, ip_off=ip_off,
                                            l4_off=l4_off, zerocopy=zc)
            np.testing.assert_array_equal(pin.array if zc else b, ref)
        d = torch.from_numpy(buf0.copy()).to(DEV)
        got = xsum.tcp4_cksum_batch(d, n, offsets=torch.from_numpy(offs.astype(np.int64)).to(DEV), ip_off=ip_off,
                                    l4_off=l4_off)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint16), exp)
    finally:
        xsum.ctx_destroy(ctx)
        pin.free()


# ---------------------------------------------------------------------------
# flush ordering and tickets

def test_feeder_after_local_flush_no_poll(oracle):
    """A batch outside the registered region is flushed by the context itself
    (ticket t, staged), then a feeder batch (t + 1) is submitted with no poll
    in between, and only t + 1 is waited for: the staged results of t must be
    in its frames when the wait returns, and its slot must not be reused early."""
    ctx = 15
    n = 32
    xsum.feeder_start(0)
    pin = None
    try:
        xsum.ctx_init(ctx, 0, 1 << 20)
        frames = pktgen.tcp4_frames(4 * n, payload=(np.arange(4 * n) * 29) % 1449, stride=2048, seed=901)
        ref = frames.copy()
        oracle.tcp4_batch(ref, 4 * n, stride=2048, inplace=True)
        pin = xsum.PinnedBuffer(frames.size + 4096)
        pin.array[:] = 0
        pin.array[:frames.size] = frames
        xsum.register_frames(ctx, pin.addr, pin.nbytes)
        xsum.use_feeder(ctx)
        for rnd in range(6):
            outside = pktgen.tcp4_frames(n, payload=(np.arange(n) * 41 + rnd) % 1449, stride=2048, seed=910 + rnd)
            ref_out = outside.copy()
            oracle.tcp4_batch(ref_out, n, stride=2048, inplace=True)
            for i in range(n):                                  # local (staged) flush t
                xsum.tcp_checksums(ctx, outside.ctypes.data + i * 2048)
            t = xsum.flush_submit(ctx)
            b = rnd % 4
            pin.array[b * n * 2048:(b + 1) * n * 2048] = frames[b * n * 2048:(b + 1) * n * 2048]
            for i in range(n):                                  # feeder flush t + 1
                xsum.tcp_checksums(ctx, pin.addr + (b * n + i) * 2048)
            t2 = xsum.flush_submit(ctx)
            assert t2 == t + 1
            xsum.flush_wait(ctx, t2)
            np.testing.assert_array_equal(outside, ref_out)
            np.testing.assert_array_equal(pin.array[b * n * 2048:(b + 1) * n * 2048],
                                          ref[b * n * 2048:(b + 1) * n * 2048])
        assert xsum.ctx_stats(ctx) == (0, 6) and xsum.feeder_flushes(ctx) == 6
        xsum.use_feeder(ctx, False)
        xsum.feeder_stop(0)
    finally:
        try:
            xsum.ctx_destroy(ctx)
        except xsum.TasxError:
            pass
        try:
            xsum.feeder_stop(0)
        except xsum.TasxError:
            pass
        if pin is not None:
            pin.free()


@pytest.mark.parametrize("zero_copy", [False, True])
def test_flush_tickets_across_wrap(oracle, zero_copy):
    """Tickets restarted at 2^32 - 6 (A/B hook): 12 pipelined flushes of
    varying size, up to 4 in flight, run across the wrap (ticket 0 included);
    every frame is exact and tickets stay consecutive mod 2^32."""
    ctx = 2
    with xsum.using_library(xsum.AB_LIB_PATH) as L:
        xsum.ctx_init(ctx, 0, 1 << 20)
        pin = None
        try:
            assert L.tasx_ab_ctx_set_tickets(ctx, 0xFFFFFFFA) == 0
            nb, n = 12, 48
            frames = pktgen.tcp4_frames(nb * n, payload=(np.arange(nb * n) * 37) % 1449, stride=2048, seed=77)
            orig = frames.copy()
            ref = frames.copy()
            oracle.tcp4_batch(ref, nb * n, stride=2048, inplace=True)
            if zero_copy:
                pin = xsum.PinnedBuffer(frames.size + 4096)
                pin.array[:] = 0
                pin.array[:frames.size] = frames
                xsum.register_frames(ctx, pin.addr, pin.nbytes)
                base, view = pin.addr, pin.array[:frames.size]
            else:
                base, view = frames.ctypes.data, frames
            tickets, inflight = [], []
            for b in range(nb):
                k = n - 5 * (b % 3)
                for i in range(b * n, b * n + k):
                    xsum.tcp_checksums(ctx, base + i * 2048)
                t = xsum.flush_submit(ctx)
                tickets.append(t)
                inflight.append(t)
                if len(inflight) >= 4:
                    xsum.flush_wait(ctx, inflight.pop(0))
            xsum.flush_wait(ctx, tickets[-1])
            assert tickets == [(0xFFFFFFFB + j) & 0xFFFFFFFF for j in range(nb)]
            assert 0 in tickets
            for b in range(nb):
                k = n - 5 * (b % 3)
                lo, hi = b * n * 2048, (b * n + k) * 2048
                np.testing.assert_array_equal(view[lo:hi], ref[lo:hi])
                np.testing.assert_array_equal(view[hi:(b + 1) * n * 2048], orig[hi:(b + 1) * n * 2048])
            assert xsum.flush_poll(ctx, tickets[-1])
        finally:
            xsum.ctx_destroy(ctx)
            if pin is not None:
                pin.free()


# ---------------------------------------------------------------------------
# RX: received lengths beyond the frame's slot

@pytest.mark.parametrize("form", ["flen", "flen0", "flen_room"])
def test_verify_hint_beyond_slot(oracle, form):
    """Received lengths larger than the stride slot (or the room) are capped
    at it: reads stay in the frame's slot, results as the oracle bounded by
    min(hint, slot).  Frames packed at the end of their allocation."""
    n, stride = 4096, 128
    rng = np.random.default_rng(5)
    frames = pktgen.tcp4_frames(n, payload=rng.integers(0, 60, n), stride=stride, seed=93)
    oracle.tcp4_batch(frames, n, stride=stride, inplace=True)
    f = frames.reshape(n, stride)
    forged = np.arange(n) % 4 == 1
    forged[-1] = True
    f[forged, 16], f[forged, 17] = 0x05, 0xDC                            # total_length 1500
    d = torch.empty(frames.size, dtype=torch.uint8, device=DEV)
    d.copy_(torch.from_numpy(frames))
    hint = np.where(np.arange(n) % 2 == 0, 1514, 66 + (np.arange(n) % 40)).astype(np.int32)
    hint[-1] = 1514
    if form == "flen":
        got = xsum.tcp4_verify_batch(d, n, stride=stride, frame_len=torch.from_numpy(hint).to(DEV))
        bound = np.minimum(hint, stride).astype(np.uint32)
    elif form == "flen0":
        got = xsum.tcp4_verify_batch(d, n, stride=stride, frame_len=1514)
        bound = stride
    else:
        got = xsum.tcp4_verify_batch(d, n, stride=stride, frame_len=torch.from_numpy(hint).to(DEV), room=112)
        bound = np.minimum(hint, 112).astype(np.uint32)
    exp = oracle.tcp4_verify_batch_bounded(frames, n, bound, stride=stride)
    np.testing.assert_array_equal(got.cpu().numpy(), exp)
    assert np.all(got.cpu().numpy()[forged] & xsum.RX_L4_OK == 0)
