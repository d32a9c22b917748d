"""The persistent flush server (ABI 6; tas_amd/csrc/server_kernels.hip): TAS's
tx_flush batches (tas/fast/fastemu.c:544-566, at most TXBUF_SIZE = 32 frames,
tas/include/fastpath.h:38) handed to one long-running kernel per GPU through
descriptor rings in pinned memory -- no HIP call on the submitting thread.
Every test checks the frames bit for bit against the C oracle's
tcp_checksums (fast_flows.c:1058-1069) over the same frames.

Run on the MI355X box:  python -m pytest tests/test_server.py -m gpu -x -q
"""
import ctypes
import errno
import threading
import time

import numpy as np
import pytest
import torch

from tas_amd import pktgen, xsum

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    xsum.lib()
    yield
    _stop_quietly_or_fail()  # never leave a server running past the module


@pytest.fixture(autouse=True)
def _stop_server_after_each_test():
    """A test that fails between its server_start and its server_stop must not
    fail every later test with "already running": after each test (its own
    finally blocks have destroyed its contexts, which detaches them) stop the
    server if one is still running."""
    yield
    _stop_quietly_or_fail()


def _stop_quietly_or_fail():
    """Stop the server if one runs; "not running" (-EINVAL) is the normal case.
    Anything else is reported, never swallowed: -EBUSY (contexts a failed test
    left attached) aborts the server first so that later tests start clean,
    and -EIO (its kernel did not leave within the bound: its memory stays
    mapped, leaked) fails the teardown, as a kernel still running could fault
    on regions later tests free."""
    try:
        xsum.server_stop(0)
        return
    except xsum.TasxError as e:
        if e.code == -errno.EINVAL:
            return
        first = e
    if first.code == -errno.EBUSY:
        try:
            xsum.server_abort(0)
            xsum.server_stop(0)
        except xsum.TasxError as e2:
            pytest.fail(f"server left attached and not stoppable after abort: {first}; {e2}")
        pytest.fail(f"server left with contexts attached (aborted and stopped): {first}")
    pytest.fail(f"server stop after the test failed: {first}")


def _stop_if_running():
    """A test's own finally: stop the server if it still runs.  "Not running"
    (-EINVAL) and "contexts still attached" (-EBUSY: the autouse fixture
    aborts and reports it) pass; a kernel that did not leave (-EIO) raises."""
    try:
        xsum.server_stop(0)
    except xsum.TasxError as e:
        if e.code not in (-errno.EINVAL, -errno.EBUSY):
            raise


def _frames(nframes: int, seed: int, short: bool = True):
    """tx_flush-shaped frames (data segments of 0..1448 B, pure ACKs) at a
    2048 B mbuf stride in a pinned region, checksum fields stale."""
    pay = np.where(np.arange(nframes) % 3 == 0, 0, (np.arange(nframes) * 53 + seed) % 1449)
    frames = pktgen.tcp4_frames(nframes, payload=pay, stride=2048, seed=seed)
    if short:  # total_length < 38: a batch holding one goes through the context itself
        f = frames.reshape(nframes, 2048)
        bad = np.arange(5, nframes, 97)
        f[bad, 16], f[bad, 17] = 0, (np.arange(len(bad)) * 7) % 38
    pin = xsum.PinnedBuffer(frames.size + 4096)
    pin.array[:] = 0
    pin.array[:frames.size] = frames
    return pin, frames


def _ref(oracle, frames, n):
    ref = frames.copy()
    oracle.tcp4_batch(ref, n, stride=2048, inplace=True)
    return ref


class _Ctxs:
    def __init__(self, ids, per_ctx_bytes=1 << 20):
        self.ids, self.pins = list(ids), []
        for c in self.ids:
            xsum.ctx_init(c, 0, per_ctx_bytes)

    def close(self):
        for c in self.ids:
            try:
                xsum.ctx_destroy(c)
            except xsum.TasxError:
                pass
        for p in self.pins:
            p.free()


def test_server_interleaved_contexts(oracle):
    """Three contexts on one server, batches submitted interleaved, 32 frames
    each, completions in each context's ticket order; the batches holding a
    frame the server does not take (total_length < 38) are flushed by their
    context after its server tickets; stop refuses while contexts are attached."""
    ids, nb, n = (2, 7, 15), 12, 32
    xsum.server_start(0)
    cx = _Ctxs(ids)
    try:
        with pytest.raises(xsum.TasxError):
            xsum.server_start(0)                     # one server per GPU
        refs = []
        for k, c in enumerate(ids):
            pin, frames = _frames(nb * n, 300 + k)
            cx.pins.append(pin)
            refs.append(_ref(oracle, frames, nb * n))
            with pytest.raises(xsum.TasxError):
                xsum.use_server(c)                   # no frame region yet
            xsum.register_frames(c, pin.addr, pin.nbytes)
            xsum.use_server(c)
        tickets = {c: [] for c in ids}
        for b in range(nb):
            for k, c in enumerate(ids):
                for i in range(n):
                    xsum.tcp_checksums(c, cx.pins[k].addr + (b * n + i) * 2048)
                tickets[c].append(xsum.flush_submit(c))
        for k, c in enumerate(ids):
            assert tickets[c] == list(range(1, nb + 1))
            xsum.flush_wait(c, tickets[c][-1])
            assert all(xsum.flush_poll(c, t) for t in tickets[c])
            np.testing.assert_array_equal(cx.pins[k].array[:refs[k].size], refs[k])
            local = sum(1 for b in range(nb) if any((b * n + i) % 97 == 5 and b * n + i >= 5 for i in range(n)))
            assert xsum.server_flushes(c) == nb - local
            assert xsum.ctx_stats(c)[0] == local     # those went zero-copy through the context
        batches, frames_done = xsum.server_stats(0)
        assert batches == sum(xsum.server_flushes(c) for c in ids)
        with pytest.raises(xsum.TasxError):
            xsum.server_stop(0)                      # contexts attached
        for c in ids:
            xsum.use_server(c, False)
        xsum.server_stop(0)
        with pytest.raises(xsum.TasxError):
            xsum.server_stop(0)                      # not running
    finally:
        cx.close()
        _stop_if_running()


def test_server_reused_mbufs_and_large_flush(oracle):
    """The same mbufs refilled with new frames between flushes (a line read by
    an earlier batch must never be served again), one flush of 200 frames
    (split over four ring slots: 64 per slot), and back-to-back synchronous
    tasx_flush calls."""
    xsum.server_start(0)
    cx = _Ctxs([4])
    try:
        n = 200
        pin = xsum.PinnedBuffer(n * 2048 + 4096)
        cx.pins.append(pin)
        xsum.register_frames(4, pin.addr, pin.nbytes)
        xsum.use_server(4)
        for rnd in range(6):
            pay = (np.arange(n) * (37 + rnd) + 11 * rnd) % 1449
            pay[rnd::5] = 0
            frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=700 + rnd)
            pin.array[:frames.size] = frames
            ref = _ref(oracle, frames, n)
            m = n if rnd % 2 == 0 else 32
            for i in range(m):
                xsum.tcp_checksums(4, pin.addr + i * 2048)
            xsum.tx_flush(4)
            np.testing.assert_array_equal(pin.array[:m * 2048], ref[:m * 2048])
        assert xsum.server_flushes(4) == 3 * 4 + 3 * 1 and xsum.ctx_stats(4) == (0, 0)
        xsum.use_server(4, False)
        xsum.server_stop(0)
    finally:
        cx.close()


@pytest.mark.parametrize("mem", ["host_alloc", "registered", "registered_huge"])
def test_server_refilled_mbufs_every_flush(oracle, mem):
    """TAS reuses an mbuf as soon as its frame has left: 300 flushes of 32
    frames through the SAME 32 mbufs, new headers and payload every time, in
    pinned memory from tasx_host_alloc and in plain pages pinned by
    tasx_ctx_register_frames (hipHostRegister, as a DPDK mempool would be;
    `registered_huge`: a 2 MiB transparent huge page, as DPDK's hugepage
    mempool).  The ring's workgroups come back to the same mbufs every few
    flushes: a frame line cached in an XCD's L2 by an earlier batch must never
    be summed."""
    import mmap
    xsum.server_start(0)
    cx = _Ctxs([6])
    raw = mm = None
    try:
        n, rounds, nbytes = 32, 300, 32 * 2048 + 4096
        if mem == "host_alloc":
            pin = xsum.PinnedBuffer(nbytes)
            cx.pins.append(pin)
            arr, addr = pin.array, pin.addr
        elif mem == "registered_huge":
            huge = 2 << 20
            mm = mmap.mmap(-1, 2 * huge, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
            off = (-base) % huge
            mm.madvise(mmap.MADV_HUGEPAGE, off, huge)
            raw = np.frombuffer(mm, dtype=np.uint8, count=huge, offset=off)
            raw[:] = 0
            arr, addr = raw[:nbytes], base + off
        else:
            raw = np.zeros(nbytes + 4096, np.uint8)
            off = (-raw.ctypes.data) % 4096
            arr, addr = raw[off:off + nbytes], raw.ctypes.data + off
        xsum.register_frames(6, addr, nbytes)
        xsum.use_server(6)
        for rnd in range(rounds):
            pay = (np.arange(n) * (31 + rnd) + 7 * rnd) % 1449
            pay[rnd % 4::4] = 0
            frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=9000 + rnd)
            arr[:frames.size] = frames
            ref = _ref(oracle, frames, n)
            for i in range(n):
                xsum.tcp_checksums(6, addr + i * 2048)
            xsum.tx_flush(6)
            np.testing.assert_array_equal(arr[:frames.size], ref, err_msg=f"round {rnd}")
        assert xsum.server_flushes(6) == rounds
        xsum.use_server(6, False)
        xsum.server_stop(0)
    finally:
        cx.close()
        _stop_if_running()
        del raw  # unregistered by the context's release (at the server's stop at the latest)
        arr = None
        if mm is not None:
            try:
                mm.close()
            except BufferError:  # a view still held (by a failure's traceback): the process frees it
                pass


def test_server_ring_wrap_and_tag_wrap(oracle):
    """70,000 one-frame flushes with up to 8 in flight: the 8-slot ring wraps
    8,750 times and the 16-bit slot tags wrap (position 65,535 -> 0) with the
    server reading every slot fresh, once right after an idle spell that put
    the ring on header-only polls; every frame right."""
    xsum.server_start(0)
    cx = _Ctxs([9])
    try:
        nf = 64
        pin, frames = _frames(nf, 901, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nf)
        xsum.register_frames(9, pin.addr, pin.nbytes)
        xsum.use_server(9)
        total, inflight = 70000, []
        for k in range(total):
            if k in (65535, 65536 + 7):
                # the ring idle past the header-only threshold (2 ms) just
                # before the positions whose tag is 0 (p + 1 = 2^16): the
                # header-only poll must not take a slot whose entries it did
                # not read
                for t in inflight:
                    xsum.flush_wait(9, t)
                inflight = []
                time.sleep(0.005)
            xsum.tcp_checksums(9, pin.addr + (k % nf) * 2048)
            inflight.append(xsum.flush_submit(9))
            if len(inflight) >= 8:
                xsum.flush_wait(9, inflight.pop(0))
        xsum.flush_wait(9, inflight[-1])
        np.testing.assert_array_equal(pin.array[:frames.size], ref)
        assert xsum.server_flushes(9) == total
        xsum.use_server(9, False)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_server_reattach_keeps_ring_position(oracle):
    """The ring's workgroups take positions k mod K and wait at the ring's next
    one: a context detached after a number of flushes that is no multiple of K
    (nor of the ring's 8 slots), then attached again -- also after the context
    was destroyed and created anew under the same id while the server ran (its
    memory released at the server's stop: HIP frees wait for the server's
    kernel) -- continues at that position, and every frame comes back right."""
    xsum.server_start(0)
    cx = _Ctxs([5])
    try:
        nf = 40
        pin, frames = _frames(nf, 333, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nf)
        xsum.register_frames(5, pin.addr, pin.nbytes)
        k, done = 0, 0
        for rnd, m in enumerate((3, 5, 1, 7, 11, 13)):
            if rnd == 3:  # destroy and create the context anew under the same id
                xsum.ctx_destroy(5)
                xsum.ctx_init(5, 0, 1 << 20)
                xsum.register_frames(5, pin.addr, pin.nbytes)
            xsum.use_server(5)
            before = xsum.server_flushes(5)
            inflight = []
            for _ in range(m):
                xsum.tcp_checksums(5, pin.addr + (k % nf) * 2048)
                k += 1
                inflight.append(xsum.flush_submit(5))
            xsum.flush_wait(5, inflight[-1])
            assert xsum.server_flushes(5) - before == m
            done += m
            xsum.use_server(5, False)
        assert k == done
        np.testing.assert_array_equal(pin.array[:frames.size], ref)
        assert xsum.server_stats(0)[0] == done
        # HIP frees wait for every stream of the device: refused while the
        # server runs instead of hanging; the buffer is released after the stop
        tmp = xsum.PinnedBuffer(4096)
        assert xsum.lib().tasx_host_free(tmp.addr) == -errno.EBUSY
        assert xsum.lib().tasx_feeder_stop(0) == -errno.EINVAL  # none running: checked first
        xsum.server_stop(0)
        tmp.free()
        assert tmp.addr == 0
    finally:
        cx.close()
        _stop_if_running()


def test_server_frames_it_does_not_take(oracle):
    """The server takes a batch only if every frame starts 16-byte aligned
    inside the registered region and all the chunks it reads lie inside it
    (tasx_host.c server_ok).  A frame moved 8 bytes off its mbuf start, and a
    last frame whose final chunk would cross the region's end (the region cut
    at the frame's last byte), send their batches through the context itself;
    every frame right, and only the clean batch counted as a server flush."""
    xsum.server_start(0)
    cx = _Ctxs([11])
    try:
        n = 64
        pin, frames = _frames(n, 555, short=False)
        cx.pins.append(pin)
        buf = pin.array
        offs = np.arange(n, dtype=np.uint64) * 2048
        # frame 10 moved 8 bytes into its room
        buf[10 * 2048 + 8:10 * 2048 + 8 + 1600] = frames[10 * 2048:10 * 2048 + 1600]
        offs[10] += 8
        tl63 = (int(buf[63 * 2048 + 16]) << 8) | int(buf[63 * 2048 + 17])
        region = 63 * 2048 + 14 + tl63                 # ends at frame 63's last byte
        assert region % 16 != 0
        ref = buf.copy()
        oracle.tcp4_batch(ref, n, offsets=offs, inplace=True)
        xsum.register_frames(11, pin.addr, region)
        xsum.use_server(11)
        batches = [[i for i in range(32) if i != 10], [10] + list(range(32, 41)), list(range(41, 64))]
        for b in batches:
            for i in b:
                xsum.tcp_checksums(11, pin.addr + int(offs[i]))
            xsum.tx_flush(11)
        assert xsum.server_flushes(11) == 1
        assert sum(xsum.ctx_stats(11)) == 2                # the other two went through the context
        for i in range(n):
            o = int(offs[i])
            np.testing.assert_array_equal(buf[o:o + 1514], ref[o:o + 1514], err_msg=f"frame {i}")
        xsum.use_server(11, False)
        xsum.server_stop(0)
    finally:
        cx.close()
        _stop_if_running()


def test_server_changed_frame_is_reported(oracle):
    """A frame whose total_length changes after tasx_flush_submit (TAS must
    not touch a frame before its ticket completes) is left alone by the
    server, and the context's poll and wait report -EIO from then on; the
    detach still completes (reporting -EIO once), and re-attached the context
    flushes correctly again."""
    xsum.server_start(0)
    cx = _Ctxs([13])
    try:
        nf = 8
        pin, frames = _frames(nf, 121, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nf)
        xsum.register_frames(13, pin.addr, pin.nbytes)
        xsum.use_server(13)
        seen, t = False, 0
        for _ in range(50):
            time.sleep(0.003)  # the ring idle: header-only polls, a few microseconds apart
            xsum.tcp_checksums(13, pin.addr)
            t = xsum.flush_submit(13)
            pin.array[17] ^= 0x04  # total_length 52 -> 48 under the server
            try:
                xsum.flush_wait(13, t)
            except xsum.TasxError as e:
                assert e.code == -errno.EIO
                seen = True
            pin.array[17] ^= 0x04
            if seen:
                break
        assert seen, "the frame was never changed before the server read it"
        with pytest.raises(xsum.TasxError):
            xsum.flush_poll(13, t)  # sticky until detached
        with pytest.raises(xsum.TasxError) as ei:
            xsum.use_server(13, False)  # detaches, and reports it once more
        assert ei.value.code == -errno.EIO
        xsum.use_server(13)
        pin.array[:frames.size] = frames
        for i in range(nf):
            xsum.tcp_checksums(13, pin.addr + i * 2048)
        xsum.tx_flush(13)
        np.testing.assert_array_equal(pin.array[:frames.size], ref)
        xsum.use_server(13, False)
        xsum.server_stop(0)
    finally:
        cx.close()
        _stop_if_running()


def test_server_threads(oracle):
    """Eight fast-path threads, each with its own context bound
    (tasx_set_thread_ctx) and attached to the server, 60 tx_flush batches
    each with up to 7 in flight (poll, then wait for the oldest): every frame
    of every thread checksummed exactly."""
    ids, nb, n = tuple(range(1, 9)), 60, 32
    xsum.server_start(0)
    cx = _Ctxs(ids)
    errs, refs = [], []
    try:
        for k, c in enumerate(ids):
            pin, frames = _frames(nb * n, 500 + k, short=False)
            cx.pins.append(pin)
            refs.append(_ref(oracle, frames, nb * n))
            xsum.register_frames(c, pin.addr, pin.nbytes)
            xsum.use_server(c)

        def core(k, c):
            try:
                xsum.set_thread_ctx(c)
                inflight = []
                for b in range(nb):
                    for i in range(n):
                        xsum.tcp_checksums(xsum.CTX_SELF, cx.pins[k].addr + (b * n + i) * 2048)
                    inflight.append(xsum.flush_submit(xsum.CTX_SELF))
                    while inflight and xsum.flush_poll(xsum.CTX_SELF, inflight[0]):
                        inflight.pop(0)
                    if len(inflight) >= 7:
                        xsum.flush_wait(xsum.CTX_SELF, inflight.pop(0))
                if inflight:
                    xsum.flush_wait(xsum.CTX_SELF, inflight[-1])
                xsum.set_thread_ctx(xsum.CTX_SELF)
            except Exception as e:  # reported below
                errs.append(e)
        th = [threading.Thread(target=core, args=(k, c)) for k, c in enumerate(ids)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert not errs, errs
        for k, c in enumerate(ids):
            np.testing.assert_array_equal(cx.pins[k].array[:refs[k].size], refs[k])
            assert xsum.server_flushes(c) == nb
        for c in ids:
            xsum.use_server(c, False)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_server_stop_is_bounded_and_restarts(oracle):
    """Stop returns promptly (the kernel polls the stop word between batches),
    a new server starts in its place, a context re-attaches and its flushes
    are right; the feeder and the server are exclusive per context."""
    cx = _Ctxs([12])
    try:
        pin, frames = _frames(64, 77, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, 64)
        xsum.register_frames(12, pin.addr, pin.nbytes)
        for rnd in range(3):
            xsum.server_start(0)
            xsum.use_server(12)
            pin.array[:frames.size] = frames
            for i in range(64):
                xsum.tcp_checksums(12, pin.addr + i * 2048)
            xsum.tx_flush(12)
            np.testing.assert_array_equal(pin.array[:frames.size], ref)
            xsum.use_server(12, False)
            t0 = time.perf_counter()
            xsum.server_stop(0)
            assert time.perf_counter() - t0 < 0.5
        xsum.feeder_start(0)
        try:
            xsum.use_feeder(12)
            xsum.server_start(0)
            with pytest.raises(xsum.TasxError):
                xsum.use_server(12)                  # attached to the feeder
            xsum.use_feeder(12, False)
            xsum.server_stop(0)
        finally:
            xsum.feeder_stop(0)
    finally:
        cx.close()
        _stop_if_running()


@pytest.mark.parametrize("odd,shm_mem", [(False, "host_alloc"), (True, "host_alloc"), (True, "registered"),
                                         (True, "registered_huge")])
def test_server_tx_segments(oracle, odd, shm_mem):
    """The fused TX segment build through the server (tasx_server_tx_segments,
    SURVEY 8f rows 1 + 2 at TAS's batch size): payloads gathered from the
    app's TX buffers in pinned host memory (tasx_host_alloc, or plain pages
    pinned by tasx_ctx_register_shm; wraps of the circular buffers, odd buffer
    bases and lengths), written into the mbufs and both checksums
    stored, 32 segments per flush (two ring slots each), against the oracle's
    flow_tx_read + tcp_checksums; interleaved with checksum-only flushes of
    the same context (ticket order); a descriptor the host refuses (frame not
    16-byte aligned) submits nothing; dma_read-invalid ones (payload beyond
    the buffer) leave their frame as it is, as the oracle does."""
    n = 96
    pay = np.where(np.arange(n) % 5 == 0, (np.arange(n) * 37) % 1449, pktgen.TCP_MSS)
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=4096, nflows=12, odd=odd, seed=0x5E6 + odd,
                                           room=pktgen.MBUF_ROOM)
    segs = segs.copy()
    segs["payload"][17] = 4097                     # > tx_len: dma_read would assert; left alone
    exp_fr = fr.copy()
    oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    import mmap
    xsum.server_start(0)
    cx = _Ctxs([14])
    mm = raw_shm = shm_arr = None
    try:
        hf = xsum.PinnedBuffer(fr.size + 4096)
        cx.pins.append(hf)
        if shm_mem == "host_alloc":
            hs = xsum.PinnedBuffer(sl + 64)
            cx.pins.append(hs)
            shm_arr, shm_addr = hs.array, hs.addr
        elif shm_mem == "registered_huge":  # a 2 MiB transparent huge page: TAS's default hugepage tas_shm
            huge = 2 << 20
            assert sl + 64 <= huge
            mm = mmap.mmap(-1, 2 * huge, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
            o = (-base) % huge
            mm.madvise(mmap.MADV_HUGEPAGE, o, huge)
            raw_shm = np.frombuffer(mm, dtype=np.uint8, count=huge, offset=o)
            raw_shm[:] = 0
            shm_arr, shm_addr = raw_shm[:sl + 64], base + o
        else:  # plain pages, pinned by tasx_ctx_register_shm (hipHostRegister), as TAS's tas_shm would be
            raw_shm = np.zeros(sl + 8192, np.uint8)
            o = (-raw_shm.ctypes.data) % 4096
            shm_arr, shm_addr = raw_shm[o:o + sl + 64], raw_shm.ctypes.data + o
        shm_arr[:sl] = shm[:sl]
        hf.array[:] = 0
        hf.array[:fr.size] = fr
        # a checksum-only batch in the same frame region, after the segments' frames
        tail = pktgen.tcp4_frames(2, payload=100, stride=2048, seed=99)
        hf.array[fr.size:fr.size + tail.size] = tail[:4096]
        tail_ref = tail.copy()
        oracle.tcp4_batch(tail_ref, 2, stride=2048, inplace=True)
        xsum.register_frames(14, hf.addr, hf.nbytes)
        xsum.register_shm(14, shm_addr, sl)
        xsum.use_server(14)
        bad = segs[:1].copy()
        bad["frame_off"] += 8
        with pytest.raises(xsum.TasxError):
            xsum.server_tx_segments(14, bad)
        tickets = []
        for b in range(0, n, 32):
            tickets.append(xsum.server_tx_segments(14, segs[b:b + 32]))
            if b == 32:
                for i in range(2):
                    xsum.tcp_checksums(14, hf.addr + fr.size + i * 2048)
                tickets.append(xsum.flush_submit(14))
        assert tickets == sorted(tickets) and len(set(tickets)) == len(tickets)
        xsum.flush_wait(14, tickets[-1])
        np.testing.assert_array_equal(hf.array[:fr.size], exp_fr)
        np.testing.assert_array_equal(hf.array[fr.size:fr.size + 4096], tail_ref[:4096])
        assert xsum.server_flushes(14) == 3 * 1 + 1     # 32 segments: one slot (up to 41)
        xsum.use_server(14, False)
        xsum.server_stop(0)
    finally:
        cx.close()
        _stop_if_running()
        raw_shm = shm_arr = None  # unregistered by the context's release
        if mm is not None:
            try:
                mm.close()
            except BufferError:  # a view still held (by a failure's traceback): the process frees it
                pass


def test_server_beside_feeder_and_device_batches(oracle):
    """The server shares its GPU: one context on the server, one on the shared
    feeder, and 64K-frame device-resident batches on a torch stream, all
    running together; every result right.  (The server's per-batch acquire
    only drops the XCDs' non-coherent L2 lines; the feeder's and the batch
    kernels' own launch boundaries keep them correct.)"""
    n = 32
    dev_n = 65536
    dframes = torch.from_numpy(pktgen.tcp4_frames(dev_n, stride=2048, seed=4242)).cuda()
    dref = xsum.tcp4_cksum_batch(dframes, dev_n, stride=2048).cpu().numpy()
    xsum.server_start(0)
    xsum.feeder_start(0)
    cx = _Ctxs([3, 10])
    try:
        pins, refs = [], []
        for k, c in enumerate((3, 10)):
            pin, frames = _frames(8 * n, 610 + k, short=False)
            cx.pins.append(pin)
            pins.append(pin)
            refs.append(_ref(oracle, frames, 8 * n))
            xsum.register_frames(c, pin.addr, pin.nbytes)
        xsum.use_server(3)
        xsum.use_feeder(10)
        s = torch.cuda.Stream()
        outs = []
        tickets = {3: [], 10: []}
        for b in range(8):
            with torch.cuda.stream(s):
                outs.append(xsum.tcp4_cksum_batch(dframes, dev_n, stride=2048, stream=s))
            for k, c in enumerate((3, 10)):
                for i in range(n):
                    xsum.tcp_checksums(c, pins[k].addr + (b * n + i) * 2048)
                tickets[c].append(xsum.flush_submit(c))
        for c in (3, 10):
            xsum.flush_wait(c, tickets[c][-1])
        s.synchronize()
        for k in range(2):
            np.testing.assert_array_equal(pins[k].array[:refs[k].size], refs[k])
        assert xsum.server_flushes(3) == 8
        xsum.use_server(3, False)
        xsum.use_feeder(10, False)
        xsum.server_stop(0)   # before any copy back: HIP's synchronous copies may wait for every stream
        xsum.feeder_stop(0)
        for o in outs:
            np.testing.assert_array_equal(o.cpu().numpy(), dref)
    finally:
        cx.close()
        for stop in (xsum.server_stop, xsum.feeder_stop):
            try:
                stop(0)
            except xsum.TasxError:
                pass


def _finish_on_cpu(oracle, pin, refs):
    """The glue's recovery step: the frames handed
    back by tasx_take_unfinished take TAS's CPU path (here the oracle's
    tcp_checksums, in place)."""
    offs = np.array([ip - 14 - pin.addr for ip, l4 in refs], np.uint64)
    assert all(l4 == ip + 20 for ip, l4 in refs)
    if len(offs):
        oracle.tcp4_batch(pin.array, len(offs), offsets=offs, inplace=True)
    return offs


def test_server_abort_hands_back_unfinished(oracle):
    """ABI 8 error contract: batches queued to a server whose
    kernel is aborted come back through tasx_take_unfinished; finished on the
    CPU, every frame equals the oracle's.  Batches the server completed before
    the abort are not handed back; the context works again afterwards (zero-copy
    flush of its own), the server stops once it is detached, and restarts."""
    n, nb = 32, 6
    xsum.server_start(0)
    cx = _Ctxs([5])
    try:
        pin, frames = _frames(nb * n, 900, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nb * n)
        xsum.register_frames(5, pin.addr, pin.nbytes)
        xsum.use_server(5)
        for i in range(n):                               # one batch the server finishes
            xsum.tcp_checksums(5, pin.addr + i * 2048)
        xsum.tx_flush(5)
        xsum.server_abort(0)
        for b in range(1, nb):                           # queued to the gone kernel
            for i in range(n):
                xsum.tcp_checksums(5, pin.addr + (b * n + i) * 2048)
            xsum.flush_submit(5)
        with pytest.raises(xsum.TasxError):
            xsum.flush_wait(5, nb)
        back = xsum.take_unfinished(5)
        offs = _finish_on_cpu(oracle, pin, back)
        assert sorted(offs.tolist()) == [k * 2048 for k in range(n, nb * n)]
        np.testing.assert_array_equal(pin.array[:ref.size], ref)
        assert xsum.pending(5) == 0 and xsum.take_unfinished(5) == []
        assert xsum.flush_poll(5, nb) is True            # every ticket settled
        with pytest.raises(xsum.TasxError):
            xsum.use_server(5)                           # the aborted server takes no context
        xsum.server_stop(0)                              # detached by the settle
        pin.array[:frames.size] = frames                 # the context's own (zero-copy) flush
        for i in range(n):
            xsum.tcp_checksums(5, pin.addr + i * 2048)
        xsum.tx_flush(5)
        np.testing.assert_array_equal(pin.array[:n * 2048], ref[:n * 2048])
        xsum.server_start(0)                             # and a new server serves it again
        xsum.use_server(5)
        for i in range(n):
            xsum.tcp_checksums(5, pin.addr + (n + i) * 2048)
        pin.array[n * 2048:2 * n * 2048] = frames[n * 2048:2 * n * 2048]
        xsum.tx_flush(5)
        np.testing.assert_array_equal(pin.array[:2 * n * 2048], ref[:2 * n * 2048])
        xsum.use_server(5, False)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_server_detach_from_gone_kernel(oracle):
    """a context attached to a server whose kernel has gone, with
    batches outstanding, detaches (-EIO once, its frames in the unfinished
    store), so the server stops and a new one starts; destroying such a context
    needs no detach of its own."""
    n = 32
    xsum.server_start(0)
    cx = _Ctxs([6, 7])
    try:
        pins = []
        for k, c in enumerate((6, 7)):
            pin, frames = _frames(3 * n, 950 + k, short=False)
            cx.pins.append(pin)
            pins.append((pin, _ref(oracle, frames, 3 * n)))
            xsum.register_frames(c, pin.addr, pin.nbytes)
            xsum.use_server(c)
        xsum.server_abort(0)
        for k, c in enumerate((6, 7)):
            for b in range(3):
                for i in range(n):
                    xsum.tcp_checksums(c, pins[k][0].addr + (b * n + i) * 2048)
                xsum.flush_submit(c)
        with pytest.raises(xsum.TasxError):
            xsum.use_server(6, False)                    # -EIO: detached from the gone kernel
        xsum.use_server(6, False)                        # already detached
        back = xsum.take_unfinished(6)
        assert len(back) == 3 * n
        _finish_on_cpu(oracle, pins[0][0], back)
        np.testing.assert_array_equal(pins[0][0].array[:pins[0][1].size], pins[0][1])
        xsum.ctx_destroy(7)                              # still attached: destroy detaches it
        cx.ids.remove(7)
        xsum.server_stop(0)
        xsum.server_start(0)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_server_tx_segments_abort_and_bad_offsets(oracle):
    """TX segments queued to an aborted server come back through
    tasx_take_unfinished_segs as submitted; built on the CPU (the oracle's
    flow_tx_read + tcp_checksums) every frame equals the oracle's.  A
    descriptor whose frame_off would wrap the bounds check is refused."""
    n = 40
    shm, fr, segs, sl = pktgen.tx_segments(n, tx_len=4096, nflows=8, seed=0x7A7, room=pktgen.MBUF_ROOM)
    exp_fr = fr.copy()
    oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    xsum.server_start(0)
    cx = _Ctxs([9])
    try:
        hf = xsum.PinnedBuffer(fr.size + 4096)
        hs = xsum.PinnedBuffer(sl + 64)
        cx.pins += [hf, hs]
        hs.array[:sl] = shm[:sl]
        hf.array[:] = 0
        hf.array[:fr.size] = fr
        xsum.register_frames(9, hf.addr, hf.nbytes)
        xsum.register_shm(9, hs.addr, sl)
        xsum.use_server(9)
        for off in (0xFFFFFFFFFFFFFFF0, hf.nbytes, hf.nbytes - 16):
            bad = segs[:1].copy()
            bad["frame_off"] = off
            with pytest.raises(xsum.TasxError):
                xsum.server_tx_segments(9, bad)
        xsum.server_abort(0)
        t = xsum.server_tx_segments(9, segs)             # 40 segments: two slots of 20
        with pytest.raises(xsum.TasxError):
            xsum.flush_wait(9, t)
        assert xsum.take_unfinished(9) == []
        back = xsum.take_unfinished_segs(9)
        assert len(back) == n
        np.testing.assert_array_equal(np.sort(back, order="frame_off"), np.sort(segs, order="frame_off"))
        frames_now = hf.array[:fr.size].copy()
        oracle.tx_segment_batch(shm, sl, frames_now, back)
        np.testing.assert_array_equal(frames_now, exp_fr)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_shm_registered_by_two_contexts(oracle):
    """every core registers the same tas_shm; the pin is counted,
    so destroying the first context to register it leaves it mapped for the
    others -- TX segments through the second context still build right."""
    n = 32
    shm, fr, segs, sl = pktgen.tx_segments(n, tx_len=4096, nflows=4, seed=0x5A5, room=pktgen.MBUF_ROOM)
    exp_fr = fr.copy()
    oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    raw_shm = np.zeros(sl + 8192, np.uint8)              # plain pages: pinned by the library
    o = (-raw_shm.ctypes.data) % 4096
    shm_arr, shm_addr = raw_shm[o:o + sl + 64], raw_shm.ctypes.data + o
    shm_arr[:sl] = shm[:sl]
    cx = _Ctxs([11, 12])
    try:
        hf = xsum.PinnedBuffer(fr.size + 4096)
        cx.pins.append(hf)
        hf.array[:] = 0
        hf.array[:fr.size] = fr
        for c in (11, 12):
            xsum.register_shm(c, shm_addr, sl)
        xsum.register_frames(12, hf.addr, hf.nbytes)
        xsum.ctx_destroy(11)                             # the first registrant goes
        cx.ids.remove(11)
        xsum.server_start(0)
        xsum.use_server(12)
        xsum.flush_wait(12, xsum.server_tx_segments(12, segs))
        np.testing.assert_array_equal(hf.array[:fr.size], exp_fr)
        xsum.use_server(12, False)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_server_left_running_by_a_failed_test_a():
    """(With _b.) A test that fails with its server started: the per-test
    fixture stops it, so the next test's server_start succeeds."""
    xsum.server_start(0)
    xsum.ctx_init(13, 0, 1 << 20)
    xsum.ctx_destroy(13)                                 # no server_stop: as a failed test leaves it


def test_server_left_running_by_a_failed_test_b():
    xsum.server_start(0)
    xsum.server_stop(0)


def test_take_unfinished_without_a_failure(oracle):
    """ABI 8 on a healthy context, no server: tasx_take_unfinished waits for
    the flushes in flight (they finish on the GPU: nothing comes back for
    them) and hands back the frames recorded but never submitted -- the glue
    finishes those on the CPU; the context flushes on the GPU afterwards."""
    n = 32
    cx = _Ctxs([12])
    try:
        pin, frames = _frames(4 * n, 977, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, 4 * n)
        xsum.register_frames(12, pin.addr, pin.nbytes)
        for b in range(2):                               # two zero-copy flushes in flight
            for i in range(n):
                xsum.tcp_checksums(12, pin.addr + (b * n + i) * 2048)
            xsum.flush_submit(12)
        for i in range(n):                               # recorded, never submitted
            xsum.tcp_checksums(12, pin.addr + (2 * n + i) * 2048)
        back = xsum.take_unfinished(12)
        offs = _finish_on_cpu(oracle, pin, back)
        assert sorted(offs.tolist()) == [k * 2048 for k in range(2 * n, 3 * n)]
        np.testing.assert_array_equal(pin.array[:3 * n * 2048], ref[:3 * n * 2048])
        assert xsum.pending(12) == 0 and xsum.take_unfinished(12) == []
        assert xsum.flush_poll(12, 2) is True
        for i in range(n):                               # and the GPU path again
            xsum.tcp_checksums(12, pin.addr + (3 * n + i) * 2048)
        xsum.tx_flush(12)
        np.testing.assert_array_equal(pin.array[:4 * n * 2048], ref[:4 * n * 2048])
    finally:
        cx.close()


# seeds of the random-walk tests: one by default; TASX_STRESS_SEEDS=N runs N
# (a stress run on the GPU box, profiles/r05 r05zd)
STRESS_SEEDS = list(range(int(__import__("os").environ.get("TASX_STRESS_SEEDS", "1"))))


def _pause_now(rng, drained: bool, submit):
    """ABI 9 in a random walk: pause the server (with batches in flight unless
    `drained`), and when drained hand it 1-3 batches while paused (their
    tickets stay open until the resume), then resume."""
    xsum.server_pause(0)
    if drained:
        for _ in range(int(rng.integers(1, 4))):
            submit()
    xsum.server_resume(0)


@pytest.mark.parametrize("pauses", [False, True])
@pytest.mark.parametrize("seed", STRESS_SEEDS)
def test_server_random_flushes(oracle, seed, pauses):
    """A seeded random walk over the server's contract: 1,500 flushes of 1 to
    130 frames (batches over 64 frames take several slots), up to 1-8 in
    flight (the depth changing as it goes), mbufs refilled with new frames as
    soon as their flush completed (the lines an earlier batch read must never
    be served again), a few frames the server does not take (their batches go
    through the context itself), submit or synchronous flush at random; every
    frame of every flush checked against the oracle when its ticket completes.
    With `pauses` (ABI 9) the server is paused and resumed about every 50
    flushes, with batches in flight or with new ones handed over while it is
    paused."""
    rng = np.random.default_rng(0x5EED + seed + (1000 if pauses else 0))
    nt, nmb = 1024, 600
    tmpl, _ = _frames(nt, 4242, short=True)              # templates: data segments, ACKs, a few short
    tmpl_arr = tmpl.array[:nt * 2048].copy()
    tmpl.free()
    ref = tmpl_arr.copy()
    oracle.tcp4_batch(ref, nt, stride=2048, inplace=True)
    tv, rv = tmpl_arr.reshape(nt, 2048), ref.reshape(nt, 2048)
    xsum.server_start(0)
    cx = _Ctxs([13])
    try:
        pin = xsum.PinnedBuffer(nmb * 2048)
        cx.pins.append(pin)
        mb = pin.array[:nmb * 2048].reshape(nmb, 2048)
        xsum.register_frames(13, pin.addr, pin.nbytes)
        xsum.use_server(13)
        free = list(range(nmb))
        out = []                                         # (ticket, [(mbuf, template)])
        depth, checked = 4, 0

        def complete_oldest():
            nonlocal checked
            t, items = out.pop(0)
            xsum.flush_wait(13, t)
            for m, k in items:
                np.testing.assert_array_equal(mb[m], rv[k], err_msg=f"ticket {t} mbuf {m} template {k}")
                free.append(m)
            checked += len(items)

        # templates the server takes (a batch holding a short frame goes through
        # the context after the server's tickets: while paused it would wait)
        takes = np.array([k for k in range(nt) if k < 5 or (k - 5) % 97 != 0])

        def record(n, pool=None):
            pick = [free.pop(int(rng.integers(0, len(free)))) for _ in range(n)]
            items = []
            for m in pick:
                k = int(rng.integers(0, nt)) if pool is None else int(pool[rng.integers(0, len(pool))])
                mb[m] = tv[k]
                xsum.tcp_checksums(13, pin.addr + m * 2048)
                items.append((m, k))
            return items

        def submit_small():  # one slot's worth, while paused: never waits for a free slot
            items = record(int(rng.integers(1, 65)), takes)
            out.append((xsum.flush_submit(13), items))

        npause = 0
        for f in range(1500):
            if f % 100 == 0:
                depth = int(rng.integers(1, 9))
            if pauses and (rng.random() < 0.02 or f % 100 == 50):
                drained = rng.random() < 0.5
                while drained and out:
                    complete_oldest()
                _pause_now(rng, drained, submit_small)
                npause += 1
            n = int(rng.integers(1, 33)) if rng.random() < 0.9 else int(rng.integers(33, 131))
            while len(out) >= depth or len(free) < n:
                complete_oldest()
            items = record(n)
            if rng.random() < 0.1:                       # a synchronous tx_flush now and then
                while out:
                    complete_oldest()
                xsum.tx_flush(13)
                for m, k in items:
                    np.testing.assert_array_equal(mb[m], rv[k])
                    free.append(m)
                checked += len(items)
            else:
                out.append((xsum.flush_submit(13), items))
        while out:
            complete_oldest()
        assert checked > 30000
        assert xsum.server_flushes(13) > 1000            # batches with a short frame go through the context
        assert npause > 10 if pauses else npause == 0
        xsum.use_server(13, False)
        xsum.server_stop(0)
    finally:
        cx.close()


@pytest.mark.parametrize("pauses", [False, True])
@pytest.mark.parametrize("seed", STRESS_SEEDS)
def test_server_tx_segments_random_groups(oracle, seed, pauses):
    """TX segment slots under a seeded random walk: 4,096 segments of 64 flows
    (odd buffer bases and lengths, payloads of 0-1448 B, circular-buffer
    wraps) handed over in groups of 1-90 (groups over 41 take several slots)
    with 1-8 flushes in flight; every frame equals the oracle's flow_tx_read +
    tcp_checksums.  With `pauses` (ABI 9) the server is paused and resumed
    every ~12 groups, with groups in flight or with new ones (of one slot)
    handed over while it is paused."""
    rng = np.random.default_rng(0x7E57 + seed)
    n = 4096
    pay = rng.integers(0, pktgen.TCP_MSS + 1, n)
    pay[rng.random(n) < 0.2] = pktgen.TCP_MSS
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=16384, nflows=64, odd=True, seed=0xA11 + seed,
                                           room=pktgen.MBUF_ROOM)
    exp_fr = fr.copy()
    oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    xsum.server_start(0)
    cx = _Ctxs([15])
    try:
        hf = xsum.PinnedBuffer(fr.size + 4096)
        hs = xsum.PinnedBuffer(sl + 64)
        cx.pins += [hf, hs]
        hs.array[:sl] = shm[:sl]
        hf.array[:] = 0
        hf.array[:fr.size] = fr
        xsum.register_frames(15, hf.addr, hf.nbytes)
        xsum.register_shm(15, hs.addr, sl)
        xsum.use_server(15)
        out, i, depth, npause, since = [], 0, 4, 0, 0

        def submit_small():  # one slot, while paused
            nonlocal i
            if i < n:
                g = min(int(rng.integers(1, 42)), n - i)
                out.append(xsum.server_tx_segments(15, segs[i:i + g]))
                i += g

        while i < n:
            if rng.random() < 0.05:
                depth = int(rng.integers(1, 9))
            since += 1
            if pauses and (rng.random() < 0.08 or since >= 15):
                since = 0
                drained = rng.random() < 0.5
                while drained and out:
                    xsum.flush_wait(15, out.pop(0))
                _pause_now(rng, drained, submit_small)
                npause += 1
                if i >= n:
                    break
            g = min(int(rng.integers(1, 91)), n - i)
            while len(out) >= depth:
                xsum.flush_wait(15, out.pop(0))
            out.append(xsum.server_tx_segments(15, segs[i:i + g]))
            i += g
        for t in out:
            xsum.flush_wait(15, t)
        np.testing.assert_array_equal(hf.array[:fr.size], exp_fr)
        assert npause >= 3 if pauses else npause == 0
        xsum.use_server(15, False)
        xsum.server_stop(0)
    finally:
        cx.close()


def test_server_pause_lets_frees_through(oracle):
    """ABI 9: HIP's frees wait for every kernel of the device, the server's
    too (profiles/r05 r05free: hipFree, hipHostFree, hipHostUnregister and
    torch.cuda.empty_cache each waited for the stop).  Paused, the server lets
    them through with its context still attached: a torch empty_cache returns
    at once, libtasx's own frees work instead of -EBUSY, batches handed over
    meanwhile stay "not done", and after the resume they and later batches
    come out bit-exact; pause/resume refuse what they cannot do."""
    n, nb = 32, 6
    xsum.server_start(0)
    cx = _Ctxs([9])
    try:
        pin, frames = _frames(nb * n, 1900, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nb * n)
        xsum.register_frames(9, pin.addr, pin.nbytes)
        xsum.use_server(9)
        extra = xsum.PinnedBuffer(1 << 20)
        for i in range(n):                               # a batch before the pause
            xsum.tcp_checksums(9, pin.addr + i * 2048)
        xsum.tx_flush(9)
        with pytest.raises(xsum.TasxError) as e:
            xsum.server_resume(0)                        # not paused
        assert e.value.code == -errno.EINVAL
        extra.free()
        assert extra.addr != 0                           # refused (-EBUSY) while the kernel runs
        xsum.server_pause(0)
        with pytest.raises(xsum.TasxError) as e:
            xsum.server_pause(0)
        assert e.value.code == -errno.EALREADY
        x = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        x.fill_(1)
        torch.cuda.synchronize()
        del x
        t0 = time.perf_counter()
        torch.cuda.empty_cache()                         # hipFree: does not wait for the paused server
        assert time.perf_counter() - t0 < 0.5
        extra.free()
        assert extra.addr == 0                           # libtasx's own free works while paused
        tickets = []
        for b in range(1, 4):                            # handed over while paused
            for i in range(n):
                xsum.tcp_checksums(9, pin.addr + (b * n + i) * 2048)
            tickets.append(xsum.flush_submit(9))
        time.sleep(0.05)
        assert not any(xsum.flush_poll(9, t) for t in tickets)
        assert not np.array_equal(pin.array[n * 2048:4 * n * 2048], ref[n * 2048:4 * n * 2048])
        xsum.server_resume(0)
        xsum.flush_wait(9, tickets[-1])
        np.testing.assert_array_equal(pin.array[:4 * n * 2048], ref[:4 * n * 2048])
        for b in range(4, nb):                           # and on as before
            for i in range(n):
                xsum.tcp_checksums(9, pin.addr + (b * n + i) * 2048)
            xsum.tx_flush(9)
        np.testing.assert_array_equal(pin.array[:ref.size], ref)
        xsum.server_pause(0)                             # a paused server stops once detached
        with pytest.raises(xsum.TasxError) as e:
            xsum.server_stop(0)                          # contexts attached
        assert e.value.code == -errno.EBUSY
        xsum.server_resume(0)
        xsum.use_server(9, False)
        xsum.server_pause(0)
        xsum.server_stop(0)
        with pytest.raises(xsum.TasxError) as e:
            xsum.server_pause(0)                         # not running
        assert e.value.code == -errno.EINVAL
    finally:
        cx.close()
        _stop_if_running()


def test_server_abort_while_paused_hands_back(oracle):
    """ABI 8 across ABI 9: batches handed to a paused server that is then
    aborted (never resumed) come back through tasx_take_unfinished, and
    finished on the CPU every frame equals the oracle's; the batch finished
    before the pause is not handed back; a resume after the abort is refused."""
    n, nb = 32, 4
    xsum.server_start(0)
    cx = _Ctxs([10])
    try:
        pin, frames = _frames(nb * n, 2100, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nb * n)
        xsum.register_frames(10, pin.addr, pin.nbytes)
        xsum.use_server(10)
        for i in range(n):
            xsum.tcp_checksums(10, pin.addr + i * 2048)
        xsum.tx_flush(10)
        xsum.server_pause(0)
        for b in range(1, nb):
            for i in range(n):
                xsum.tcp_checksums(10, pin.addr + (b * n + i) * 2048)
            xsum.flush_submit(10)
        assert not xsum.flush_poll(10, nb)
        xsum.server_abort(0)
        with pytest.raises(xsum.TasxError) as e:
            xsum.server_resume(0)
        assert e.value.code == -errno.EIO
        with pytest.raises(xsum.TasxError):
            xsum.flush_wait(10, nb)
        back = xsum.take_unfinished(10)
        offs = _finish_on_cpu(oracle, pin, back)
        assert sorted(offs.tolist()) == [k * 2048 for k in range(n, nb * n)]
        np.testing.assert_array_equal(pin.array[:ref.size], ref)
        xsum.server_stop(0)                              # detached by the settle
    finally:
        cx.close()
        _stop_if_running()


def test_server_epochs_bound_device_wide_waits(oracle):
    """ABI 10: the server runs in epochs of
    5 ms with the next launch queued behind the running one, so the HIP calls
    that wait for all of the device's work -- a device-wide synchronize, a
    free (torch.cuda.empty_cache), a copy to pageable host memory -- return
    while it serves (no pause), even with a fast-path thread flushing through
    it the whole time; the epochs go on, and every frame is right."""
    n, nb = 32, 400
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    xsum.server_start(0)
    cx = _Ctxs([12])
    try:
        pin, frames = _frames(nb * n, 2600, short=False)
        cx.pins.append(pin)
        ref = _ref(oracle, frames, nb * n)
        xsum.register_frames(12, pin.addr, pin.nbytes)
        xsum.use_server(12)
        err = []

        def flusher():
            try:
                last = None
                for b in range(nb):
                    for i in range(n):
                        xsum.tcp_checksums(12, pin.addr + (b * n + i) * 2048)
                    last = xsum.flush_submit(12)
                    time.sleep(0.0005)
                xsum.flush_wait(12, last)
            except Exception as e:  # reported below
                err.append(repr(e))
        th = threading.Thread(target=flusher)
        th.start()
        took = {}
        for k in range(20):
            x = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")
            x.fill_(k)
            t = time.perf_counter()
            torch.cuda.synchronize()                     # hipDeviceSynchronize
            took.setdefault("synchronize", []).append(time.perf_counter() - t)
            t = time.perf_counter()
            h = x[:1 << 20].cpu()                        # a copy to pageable memory
            took.setdefault("copy", []).append(time.perf_counter() - t)
            assert int(h[0]) == k
            del x, h
            t = time.perf_counter()
            torch.cuda.empty_cache()                     # hipFree of the segment
            took.setdefault("free", []).append(time.perf_counter() - t)
        th.join(60)
        assert not err, err
        assert not th.is_alive()
        np.testing.assert_array_equal(pin.array[:ref.size], ref)
        worst = {k: max(v) for k, v in took.items()}
        assert all(v < 0.5 for v in worst.values()), worst
        epochs, slow, max_ms = xsum.server_epochs(0)
        assert epochs >= 2, epochs
        xsum.use_server(12, False)
        xsum.server_stop(0)
    finally:
        cx.close()
        _stop_if_running()


def test_server_pause_under_tight_submission(oracle):
    """the kernel looks at the stop word before it takes a ready
    slot, so a pause returns while fast-path threads keep every ring busy
    (taking first, a workgroup whose ring never ran empty never saw the stop
    word and the pause ran into its 5 s bound).  Four threads submit 32-frame
    batches back to back with up to 4 in flight; the main thread pauses and
    resumes the server three times meanwhile; every frame comes out bit-exact."""
    ids, n, nb = (4, 5, 6, 7), 32, 48
    xsum.server_start(0)
    cx = _Ctxs(ids)
    try:
        refs, pins = {}, {}
        for k, c in enumerate(ids):
            pin, frames = _frames(nb * n, 2500 + k, short=False)
            cx.pins.append(pin)
            pins[c], refs[c] = pin, _ref(oracle, frames, nb * n)
            xsum.register_frames(c, pin.addr, pin.nbytes)
            xsum.use_server(c)
        errs, started = [], threading.Barrier(len(ids) + 1)

        def body(c):
            try:
                started.wait()
                last = None
                for b in range(nb):
                    for i in range(n):
                        xsum.tcp_checksums(c, pins[c].addr + (b * n + i) * 2048)
                    last = xsum.flush_submit(c)      # completes the oldest when 4 are out
                xsum.flush_wait(c, last)
            except Exception as e:  # reported below
                errs.append(repr(e))
        ths = [threading.Thread(target=body, args=(c,)) for c in ids]
        for t in ths:
            t.start()
        started.wait()
        pauses = []
        for _ in range(3):
            time.sleep(0.01)
            t0 = time.perf_counter()
            xsum.server_pause(0)                     # refused with -EIO if a workgroup never saw the stop word
            pauses.append(time.perf_counter() - t0)
            time.sleep(0.01)
            xsum.server_resume(0)
        for t in ths:
            t.join(60)
        assert not errs, errs
        assert max(pauses) < 1.0, pauses
        for c in ids:
            np.testing.assert_array_equal(pins[c].array[:refs[c].size], refs[c])
            xsum.use_server(c, False)
        xsum.server_stop(0)
    finally:
        cx.close()
        _stop_if_running()


def test_pin_overlapping_another_context_refused():
    """a frame region that starts inside a region another context
    pinned but runs past its end is refused (-EINVAL): HIP would map only the
    part inside the pin, and that pin's release would unmap it under the second
    context.  A region lying inside the pin shares it (counted)."""
    cx = _Ctxs([3, 8])
    raw = np.zeros(6 * 4096, np.uint8)
    try:
        base = raw.ctypes.data + (-raw.ctypes.data) % 4096
        xsum.register_frames(3, base, 2 * 4096)
        with pytest.raises(xsum.TasxError) as e:
            xsum.register_frames(8, base, 4 * 4096)
        assert e.value.code == -errno.EINVAL
        with pytest.raises(xsum.TasxError) as e:
            xsum.register_frames(8, base + 4096, 2 * 4096)
        assert e.value.code == -errno.EINVAL
        xsum.register_frames(8, base + 4096, 4096)      # inside: the same pin, counted
    finally:
        cx.close()
    del raw
