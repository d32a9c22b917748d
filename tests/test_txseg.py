"""Fused TX segment build: flow_tx_segment()'s
payload copy from the flow's circular TX buffer (flow_tx_read,
/root/reference/tas/fast/fast_flows.c:833-846, :930-933) fused with
tcp_checksums() (:936 -> :1058-1069).

CPU tests pin the C oracle against the committed fixture (made by the numpy
restatement) and against the numpy restatement on seeded batches.  GPU tests
run tasx_tx_segment_batch_dev through the C ABI and compare the WHOLE frames
buffer (payload copy, checksum fields, and every byte the build must leave
alone) and the per-segment results with the oracle, bit-exact.
"""
import numpy as np
import pytest

from tas_amd import pktgen

GOLDEN = "txseg_vectors.npz"


@pytest.fixture(scope="module")
def txseg_golden():
    from conftest import GOLDEN as G
    with np.load(G / GOLDEN) as z:
        return {k: z[k] for k in z.files}


def _segs(g):
    return g["segs"].view(pktgen.TX_SEG_DTYPE)


# ---------------------------------------------------------------------------
# oracle (CPU)

def test_oracle_txseg_golden(oracle, txseg_golden):
    g = txseg_golden
    fr = g["frames_in"].copy()
    out = oracle.tx_segment_batch(g["shm"], int(g["shm_len"]), fr, _segs(g))
    np.testing.assert_array_equal(out, g["expected"])
    np.testing.assert_array_equal(fr, g["frames_out"])
    assert (out == 0).sum() == 4  # the four rejected descriptors


@pytest.mark.parametrize("odd", [False, True])
def test_oracle_txseg_vs_numpy(oracle, odd):
    from oracle import xsum_ref as R
    pay = (np.arange(150) * 37) % 1449
    shm, fr, segs, sl = pktgen.tx_segments(150, payload=pay, tx_len=2000, nflows=9, odd=odd, seed=0x1234 + odd)
    a, b = fr.copy(), fr.copy()
    np.testing.assert_array_equal(oracle.tx_segment_batch(shm, sl, a, segs), R.tx_segment(shm, sl, b, segs))
    np.testing.assert_array_equal(a, b)


def test_oracle_txseg_matches_tcp4_path(oracle):
    """After the build, the frames' checksums are what tcp_checksums gives the
    finished frames (the fused op is copy-then-checksum)."""
    shm, fr, segs, sl = pktgen.tx_segments(64, tx_len=3000, nflows=4)
    out = oracle.tx_segment_batch(shm, sl, fr, segs)
    again = oracle.tcp4_batch(fr.copy(), 64, stride=pktgen.MBUF_ROOM)
    np.testing.assert_array_equal(out, again.view(np.uint32))


def test_generator_wraps_and_flows():
    shm, fr, segs, sl = pktgen.tx_segments(4096, tx_len=16384, nflows=512)
    wraps = (segs["pos"].astype(np.int64) + segs["payload"]) > segs["tx_len"]
    assert 0 < wraps.sum() < 4096 // 4
    assert (segs["pos"] < segs["tx_len"]).all()
    assert segs.dtype.itemsize == 32 and sl == len(shm)


# ---------------------------------------------------------------------------
# GPU parity

# The comparison form of libtasx_ab.so that runs here beside the product
# (tx_segment_lds_kernel) on every TAS-layout case: "r2" =
# tasx_ab_tx_segment_form(30, ...), the round-2 product tx_segment_tas_kernel
# (unaligned non-temporal window loads).  Round 6 deleted the two forms that
# left this list in round 5 (ds_read_b128 windows, LDS-DMA staging through
# inline asm that moved M0): profiles/r06/INDEX.md.
IMPLS = ["product", "r2"]


def _gpu_run(shm, shm_len, frames, segs, ip_off=14, l4_off=34, frame_shift=0, impl="product"):
    if impl == "product" or (ip_off, l4_off) != (14, 34):
        return _gpu_run1(shm, shm_len, frames, segs, ip_off, l4_off, frame_shift)
    return _gpu_run1(shm, shm_len, frames, segs, ip_off, l4_off, frame_shift, form=30)


def _download(t):
    """t's bytes on the host, in three steps that each name themselves when a
    GPU fault surfaces in them (r05end and r06e saw hipErrorIllegalAddress at
    this copy after a clean synchronize): the synchronize after the kernel, a
    second one 50 ms later (a fault in the kernel reported late surfaces here),
    and the device-to-host copy itself."""
    import time
    import torch
    for stage in ("synchronize after the kernel", "synchronize 50 ms later", "device-to-host copy"):
        try:
            if stage == "device-to-host copy":
                return t.cpu().numpy()
            if stage == "synchronize 50 ms later":
                time.sleep(0.05)
            torch.cuda.synchronize()
        except Exception as e:
            raise AssertionError(f"GPU error surfaced at the {stage}: {e}") from e


def _gpu_run1(shm, shm_len, frames, segs, ip_off=14, l4_off=34, frame_shift=0, form=None):
    import torch
    from tas_amd import xsum
    dev = "cuda:0"
    # Host <-> device copies of whole buffers whose size is a multiple of 16
    # (r05end, r06e and r06k: hipErrorIllegalAddress surfaced at this test's
    # pageable copies of 1.55 MB at odd sizes and a 3-byte offset -- once at
    # the upload below, before any kernel of this library had run; see
    # profiles/r06/INDEX.md)
    def pad16(a, lead=0):
        h = np.zeros((lead + a.size + 16 + 15) // 16 * 16, np.uint8)
        h[lead:lead + a.size] = a
        return h
    dshm = torch.from_numpy(pad16(np.ascontiguousarray(shm).reshape(-1).view(np.uint8))).to(dev)
    fr = np.ascontiguousarray(frames)
    dfr = torch.from_numpy(pad16(fr, frame_shift)).to(dev)
    s = segs.copy()
    s["frame_off"] += np.uint64(frame_shift)
    dsegs = torch.from_numpy(s.view(np.uint8).copy()).to(dev)
    if form is None:
        out = xsum.tx_segment_batch(dshm[:shm_len], dfr, dsegs, len(s), ip_off=ip_off, l4_off=l4_off)
    else:
        out = torch.zeros(max(len(s), 1), dtype=torch.int32, device=dev)
        with xsum.using_library(xsum.AB_LIB_PATH) as ab:
            rc = ab.tasx_ab_tx_segment_form(form, dshm.data_ptr(), shm_len, dfr.data_ptr(), dsegs.data_ptr(), len(s),
                                            ip_off, l4_off, out.data_ptr(), xsum._stream(None))
            assert rc == 0, ab.tasx_last_error()
            assert xsum.last_kernel() == "tx_segment_tas_kernel", xsum.last_kernel()
    got = _download(dfr)
    assert not got[:frame_shift].any() and not got[frame_shift + fr.size:].any(), "wrote outside the frames"
    return out.cpu().numpy().view(np.uint32), got[frame_shift:frame_shift + fr.size]


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("shift", [0, 1, 2, 7])
def test_gpu_txseg_golden(txseg_golden, shift, impl):
    g = txseg_golden
    out, fr = _gpu_run(g["shm"], int(g["shm_len"]), g["frames_in"], _segs(g), frame_shift=shift, impl=impl)
    np.testing.assert_array_equal(out, g["expected"])
    np.testing.assert_array_equal(fr, g["frames_out"])


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("room", [0, pktgen.MBUF_ROOM])
@pytest.mark.parametrize("odd,tx_len,nflows", [(False, 16384, 512), (True, 16384, 512), (True, 1500, 7),
                                               (False, 1448, 3)])
def test_gpu_txseg_vs_oracle(oracle, odd, tx_len, nflows, room, impl):
    n = 4096
    pay = np.where(np.arange(n) % 5 == 0, (np.arange(n) * 131) % 1449, pktgen.TCP_MSS)
    pay = np.minimum(pay, tx_len - (7 if odd else 0))
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=tx_len, nflows=nflows, odd=odd,
                                           seed=0xC0FFEE + tx_len, room=room)
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    out, got = _gpu_run(shm, sl, fr, segs, impl=impl)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(got, exp_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
def test_gpu_txseg_packed_odd_frames(oracle, impl):
    """Frames packed back to back at an odd stride (chunks shared between
    neighbours): the build must not clobber a neighbour's bytes."""
    n, stride = 1024, 1515
    pay = (np.arange(n) * 7) % 1449
    shm, fr0, segs, sl = pktgen.tx_segments(n, payload=pay, stride=2048, tx_len=3001, nflows=13, odd=True)
    fr = np.zeros(n * stride + 1, np.uint8)
    for i in range(n):  # repack to the odd stride, trailing bytes random
        fr[i * stride:(i + 1) * stride] = fr0[i * 2048:i * 2048 + stride]
    segs["frame_off"] = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    out, got = _gpu_run(shm, sl, fr, segs, frame_shift=3, impl=impl)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(got, exp_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
def test_gpu_txseg_tso(oracle, impl):
    """64 KB segments: payload 65483 (ip.len 65535), wrap inside."""
    n, pay = 64, 65535 - 52
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, stride=65536 + 64, tx_len=98304 + 5, nflows=8,
                                           odd=True)
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    out, got = _gpu_run(shm, sl, fr, segs, impl=impl)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(got, exp_fr)
    # with the mbuf room given, the same frames (tail chunks written whole)
    segs["room"] = 65536 + 64
    out, got = _gpu_run(shm, sl, fr, segs, impl=impl)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(got, exp_fr)


@pytest.mark.gpu
def test_gpu_txseg_other_layouts(oracle):
    """Staged-record layout (ip_off 0, l4_off 20) and a gap between IP and TCP."""
    for ip_off, l4_off in ((0, 20), (14, 40)):
        n = 512
        shm, fr, segs, sl = pktgen.tx_segments(n, tx_len=5000, nflows=11, odd=True, seed=ip_off + l4_off)
        segs["hdrs_len"] = l4_off + 32
        fr = fr.reshape(n, -1)
        # rebuild each header at the layout: ip header copied to ip_off, ip.len for this hdrs_len
        hdr = fr[:, 14:34].copy()
        fr[:, ip_off:ip_off + 20] = hdr
        tl = segs["hdrs_len"].astype(np.int64) - ip_off + segs["payload"]
        fr[:, ip_off + 2] = (tl >> 8) & 0xFF
        fr[:, ip_off + 3] = tl & 0xFF
        fr = fr.reshape(-1)
        exp_fr = fr.copy()
        exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs, ip_off=ip_off, l4_off=l4_off)
        out, got = _gpu_run(shm, sl, fr, segs, ip_off=ip_off, l4_off=l4_off)
        np.testing.assert_array_equal(out, exp)
        np.testing.assert_array_equal(got, exp_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("room", [0, 2048])
def test_gpu_txseg_wrap_positions_and_region_edges(oracle, room, impl):
    """Every buffer wrap after 1..60 payload bytes (inside the frame's chunk 4,
    on chunk boundaries, in the first whole payload chunks) and payloads at the
    very start and the very end of the shared region (windows that would reach
    outside it are gathered byte by byte), for TAS segments and for segments
    with other header lengths (general body)."""
    tx_len, nfl = 1600, 64
    shm_len = tx_len * nfl
    shm = pktgen.random_bytes(77, shm_len)
    rows = [(w % nfl, tx_len - w, 1448, 66) for w in range(1, 61)]
    rows += [(0, 0, 1448, 66), (0, 0, 5, 66), (0, 1, 13, 66),              # region start
             (nfl - 1, tx_len - 1448, 1448, 66), (nfl - 1, tx_len - 3, 3, 66),  # region end
             (nfl - 1, tx_len - 10, 1448, 66), (nfl - 1, tx_len - 1, 1448, 66),
             (0, 0, 1448, 54), (nfl - 1, tx_len - 7, 1448, 80), (5, tx_len - 20, 700, 67)]
    n = len(rows)
    pay = np.array([r[2] for r in rows])
    hl = np.array([r[3] for r in rows])
    fr = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=78)
    f = fr.reshape(n, 2048)
    tl = hl - 14 + pay                       # ip.total_length for each header length
    f[:, 16] = (tl >> 8) & 0xFF
    f[:, 17] = tl & 0xFF
    segs = np.zeros(n, pktgen.TX_SEG_DTYPE)
    segs["frame_off"] = np.arange(n, dtype=np.uint64) * np.uint64(2048)
    segs["tx_base"] = [r[0] * tx_len for r in rows]
    segs["tx_len"] = tx_len
    segs["pos"] = [r[1] for r in rows]
    segs["payload"] = pay
    segs["hdrs_len"] = hl
    segs["room"] = room
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, shm_len, exp_fr, segs)
    out, got = _gpu_run(shm, shm_len, fr, segs, impl=impl)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(got, exp_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["shm", "shm+frames", "all"])
def test_gpu_txseg_host_memory(oracle, where):
    """SURVEY 8f row 1 as TAS would run it: the app's TX buffers (tas_shm) in
    pinned host memory mapped for the GPU, optionally the mbuf frames and the
    descriptors too; the kernel gathers and writes over PCIe."""
    import torch
    from tas_amd import xsum
    dev = "cuda:0"
    n = 2048
    pay = np.where(np.arange(n) % 7 == 0, (np.arange(n) * 53) % 1449, pktgen.TCP_MSS)
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=16384, nflows=256, odd=True, seed=0x5EED,
                                           room=pktgen.MBUF_ROOM)
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    pins = []
    try:
        hs = xsum.PinnedBuffer(sl)
        pins.append(hs)
        hs.array[:] = shm[:sl]
        if where == "shm":
            dfr = torch.from_numpy(fr.copy()).to(dev)
            frames = dfr
        else:
            hf = xsum.PinnedBuffer(fr.size)
            pins.append(hf)
            hf.array[:] = fr
            frames = hf.dev_addr
        if where == "all":
            hd = xsum.PinnedBuffer(segs.nbytes)
            pins.append(hd)
            hd.array[:] = segs.view(np.uint8)
            dsegs = hd.dev_addr
        else:
            dsegs = torch.from_numpy(segs.view(np.uint8).copy()).to(dev)
        out = xsum.tx_segment_batch(hs.dev_addr, frames, dsegs, n, shm_len=sl)
        torch.cuda.synchronize()
        assert xsum.last_kernel() == "tx_segment_lds_kernel"
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
        got = dfr.cpu().numpy() if where == "shm" else pins[1].array.copy()
        np.testing.assert_array_equal(got, exp_fr)
    finally:
        for pb in pins:
            pb.free()


@pytest.mark.gpu
@pytest.mark.parametrize("pages", ["huge", "4k"])
def test_gpu_txseg_registered_pages(oracle, pages):
    """The TX build over host memory as TAS allocates it: `tas_shm` is
    hugepage-backed by default (fp_hugepages, /root/reference/tas/config.c:591,
    tas/shm.c:51-64) and DPDK's mbuf pool lives in hugepages; here anonymous
    memory with transparent huge pages asked for (MADV_HUGEPAGE on 2 MiB
    boundaries; plain pages where the host disables THP) or refused, pinned by
    tasx_host_register, with the frames at an odd 2 MiB-page offset."""
    import ctypes
    import mmap
    from tas_amd import xsum
    huge = 2 << 20
    n = 4096
    pay = np.where(np.arange(n) % 5 == 0, (np.arange(n) * 29) % 1449, pktgen.TCP_MSS)
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=16384, nflows=512, odd=True, seed=0x70A,
                                           room=pktgen.MBUF_ROOM)
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    lib = xsum.lib()
    maps, regs = [], []

    def region(nbytes, shift=0):
        size = (nbytes + shift + huge - 1) // huge * huge
        mm = mmap.mmap(-1, size + huge, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        maps.append(mm)
        base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
        off = (-base) % huge
        mm.madvise(mmap.MADV_HUGEPAGE if pages == "huge" else mmap.MADV_NOHUGEPAGE, off, size)
        arr = np.frombuffer(mm, dtype=np.uint8, count=size, offset=off)
        arr[:] = 0
        assert lib.tasx_host_register(ctypes.c_void_p(base + off), ctypes.c_size_t(size)) == 0
        regs.append(base + off)
        dev = lib.tasx_host_device_pointer(ctypes.c_void_p(base + off))
        assert dev
        return arr[shift:shift + nbytes], dev + shift

    try:
        hs, ds = region(sl)
        hs[:] = shm[:sl]
        hf, df = region(fr.size, shift=3 * 4096 + 16 * 7)  # frames 16-byte aligned, off any page start
        hf[:] = fr
        hd, dd = region(segs.nbytes)
        hd[:] = segs.view(np.uint8)
        out = xsum.tx_segment_batch(ds, df, dd, n, shm_len=sl)
        got = out.cpu().numpy().view(np.uint32)
        assert xsum.last_kernel() == "tx_segment_lds_kernel"
        np.testing.assert_array_equal(got, exp)
        np.testing.assert_array_equal(hf.copy(), exp_fr)
    finally:
        import torch
        torch.cuda.synchronize()
        for a in regs:
            assert lib.tasx_host_unregister(ctypes.c_void_p(a)) == 0
        hs = hf = hd = None
        for mm in maps:
            try:
                mm.close()
            except BufferError:  # a view still held (by a failure's traceback): the process frees it
                pass


@pytest.mark.gpu
def test_gpu_txseg_errors():
    import torch
    from tas_amd import xsum
    dev = "cuda:0"
    shm = torch.zeros(4096, dtype=torch.uint8, device=dev)
    fr = torch.zeros(4096, dtype=torch.uint8, device=dev)
    segs = torch.zeros(64, dtype=torch.uint8, device=dev)
    with pytest.raises(xsum.TasxError):
        xsum.tx_segment_batch(shm, fr, segs, 1, ip_off=14, l4_off=30)   # l4 inside the IP header
    with pytest.raises(xsum.TasxError):
        xsum.tx_segment_batch(shm, fr, segs[8:], 1)                      # misaligned descriptors
    assert xsum.tx_segment_batch(shm, fr, segs, 0).numel() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("shift", [0, 16, 48])
def test_gpu_txseg_scratch_room(oracle, shift, impl):
    """room | TASX_TXSEG_SCRATCH (the mbuf holds nothing past data_len): frames
    bit-exact up to their end, results equal, and only the bytes from each
    frame's end to the end of its 128-byte block (counted from `frames`, within
    the room) may differ -- everything else in the buffer is untouched."""
    import torch
    from tas_amd import xsum
    n = 3000
    pay = np.where(np.arange(n) % 3 == 0, (np.arange(n) * 97) % 1449, pktgen.TCP_MSS)
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=16384, nflows=97, seed=0x5C2A + shift,
                                           room=pktgen.MBUF_ROOM)
    segs["room"] = np.uint32(pktgen.MBUF_ROOM | xsum.TXSEG_SCRATCH)
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    out, got = _gpu_run(shm, sl, fr, segs, frame_shift=shift, impl=impl)
    np.testing.assert_array_equal(out, exp)
    mask = np.ones(fr.size, bool)
    fend = segs["frame_off"].astype(np.int64) + pktgen.HDRS_LEN + segs["payload"].astype(np.int64)
    bend = (fend + shift + 127) // 128 * 128 - shift                   # block end, counted from `frames`
    lim = segs["frame_off"].astype(np.int64) + pktgen.MBUF_ROOM
    for a, b in zip(fend, np.minimum(bend, lim)):
        mask[a:b] = False
    np.testing.assert_array_equal(got[mask], exp_fr[mask])
    assert (~mask).sum() > 0
