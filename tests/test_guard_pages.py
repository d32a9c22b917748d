"""The product kernels over buffers fenced by unmapped guard pages (round 6,
VERDICT r05 item 1).

Every buffer a kernel reads or writes -- frames, the TX buffers' shared region,
the segment descriptors, the flow tables -- is placed flush against the end
(or the start) of a mapping whose neighbouring pages are not mapped
(tests/guarded.py).  A kernel that touched even one byte beyond the bounds
include/tasx_xsum.h promises (whole 16-byte aligned chunks holding a byte of
the packet, the hinted range or the room; the shm region's clamp; the
descriptor array) would fault here instead of silently reading a neighbour.
Each case also checks its results and frames bit-exact against the C oracle,
so the placements exercise the real code paths at the buffers' edges:

* TX segment build (tx_segment_lds_kernel + its general body, the flush
  server's row): the round-5 failure's own input (1,024 frames packed at the
  odd stride 1,515, mostly off 16-byte alignment), every wrap position and the
  shm region's first and last bytes, 64 KB TSO segments;
* TCP4 checksums: no hint, the uniform hint, per-frame hints, a room, offsets;
* RX verification with received lengths; RAW in stride, uniform-length and
  lengths modes; the flow lookup and the one-pass RX with their tables fenced.

r05end's hipErrorIllegalAddress surfaced at a copy after a clean device
synchronize, with no fault address in its record; profiles/r06/INDEX.md
records what these placements show.
"""
import numpy as np
import pytest
import torch

from guarded import Guarded
from tas_amd import pktgen, xsum

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    xsum.lib()
    yield
    torch.cuda.synchronize()


def _fenced(a: np.ndarray, at: str) -> Guarded:
    g = Guarded(a.nbytes, at=at)
    g.upload(a)
    return g


def _sync_u32(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


# ---------------------------------------------------------------------------
# TX segment build

def _txseg_fenced(oracle, shm, sl, fr, segs, frames_at, shm_at, impl="product"):
    """fr trimmed to its furthest frame byte, all three buffers fenced.
    impl "r2": the comparison build's round-2 kernel (tx_segment_tas_kernel,
    tasx_ab_tx_segment_form 30), the form r06e's fault surfaced after."""
    fend = int((segs["frame_off"].astype(np.int64) + segs["hdrs_len"] + segs["payload"]).max())
    fr = np.ascontiguousarray(fr[:fend])
    exp_fr = fr.copy()
    exp = oracle.tx_segment_batch(shm, sl, exp_fr, segs)
    with _fenced(fr, frames_at) as gf, _fenced(np.ascontiguousarray(shm[:sl]), shm_at) as gs, \
            _fenced(segs.view(np.uint8), "end") as gd:
        assert gd.addr % 16 == 0
        if impl == "product":
            out = xsum.tx_segment_batch(gs.addr, gf.addr, gd.addr, len(segs), shm_len=sl)
            got_out = _sync_u32(out)
            got_fr = gf.download()
            kernel = xsum.last_kernel()
        else:
            out = torch.zeros(len(segs), dtype=torch.int32, device=DEV)
            with xsum.using_library(xsum.AB_LIB_PATH) as ab:
                rc = ab.tasx_ab_tx_segment_form(30, gs.addr, sl, gf.addr, gd.addr, len(segs), 14, 34, out.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream)
                assert rc == 0, ab.tasx_last_error()
                got_out = _sync_u32(out)
                got_fr = gf.download()
                kernel = xsum.last_kernel()
    np.testing.assert_array_equal(got_out, exp)
    np.testing.assert_array_equal(got_fr, exp_fr)
    return kernel


@pytest.mark.parametrize("impl", ["product", "r2"])
@pytest.mark.parametrize("frames_at", ["start", "end"])
@pytest.mark.parametrize("shm_at", ["start", "end"])
def test_guard_txseg_packed_odd_frames(oracle, frames_at, shm_at, impl):
    """r05end's failing input: frames packed at stride 1515 (15 of 16 off
    16-byte alignment: the general body; 1 of 16 aligned: the LDS rows)."""
    n, stride = 1024, 1515
    pay = (np.arange(n) * 7) % 1449
    shm, fr0, segs, sl = pktgen.tx_segments(n, payload=pay, stride=2048, tx_len=3001, nflows=13, odd=True)
    fr = np.zeros(n * stride + 1, np.uint8)
    for i in range(n):
        fr[i * stride:(i + 1) * stride] = fr0[i * 2048:i * 2048 + stride]
    segs["frame_off"] = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    for shift in (0, 3):   # the whole batch moved by 3 bytes, as r05end's frame_shift
        s = segs.copy()
        s["frame_off"] += np.uint64(shift)
        f = np.concatenate([np.zeros(shift, np.uint8), fr])
        kernel = _txseg_fenced(oracle, shm, sl, f, s, frames_at, shm_at, impl)
        assert kernel == ("tx_segment_lds_kernel" if impl == "product" else "tx_segment_tas_kernel")


@pytest.mark.parametrize("impl", ["product", "r2"])
@pytest.mark.parametrize("shm_at", ["start", "end"])
def test_guard_txseg_wraps_and_region_edges(oracle, shm_at, impl):
    """Every buffer wrap after 1..60 payload bytes, payloads at the very start
    and the very end of the shm region, other header lengths (general body)."""
    tx_len, nfl = 1600, 64
    shm_len = tx_len * nfl
    shm = pktgen.random_bytes(77, shm_len)
    rows = [(w % nfl, tx_len - w, 1448, 66) for w in range(1, 61)]
    rows += [(0, 0, 1448, 66), (0, 0, 5, 66), (0, 1, 13, 66), (nfl - 1, tx_len - 1448, 1448, 66),
             (nfl - 1, tx_len - 3, 3, 66), (nfl - 1, tx_len - 10, 1448, 66), (nfl - 1, tx_len - 1, 1448, 66),
             (0, 0, 1448, 54), (nfl - 1, tx_len - 7, 1448, 80), (5, tx_len - 20, 700, 67)]
    n = len(rows)
    pay = np.array([r[2] for r in rows])
    hl = np.array([r[3] for r in rows])
    fr = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=78)
    f = fr.reshape(n, 2048)
    tl = hl - 14 + pay
    f[:, 16] = (tl >> 8) & 0xFF
    f[:, 17] = tl & 0xFF
    segs = np.zeros(n, pktgen.TX_SEG_DTYPE)
    segs["frame_off"] = np.arange(n, dtype=np.uint64) * np.uint64(2048)
    segs["tx_base"] = [r[0] * tx_len for r in rows]
    segs["tx_len"] = tx_len
    segs["pos"] = [r[1] for r in rows]
    segs["payload"] = pay
    segs["hdrs_len"] = hl
    # the last frame is the furthest one: a 1448-byte TAS segment ending at the fence
    segs[-1], segs[-4] = segs[-4].copy(), segs[-1].copy()
    f[[-1, -4]] = f[[-4, -1]]
    segs["frame_off"] = np.arange(n, dtype=np.uint64) * np.uint64(2048)
    _txseg_fenced(oracle, shm, shm_len, fr, segs, "end", shm_at, impl)


@pytest.mark.parametrize("impl", ["product", "r2"])
@pytest.mark.parametrize("odd,tx_len,nflows", [(True, 1500, 7), (False, 16384, 512)])
def test_guard_txseg_random(oracle, odd, tx_len, nflows, impl):
    n = 4096
    pay = np.where(np.arange(n) % 5 == 0, (np.arange(n) * 131) % 1449, pktgen.TCP_MSS)
    pay = np.minimum(pay, tx_len - (7 if odd else 0))
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, tx_len=tx_len, nflows=nflows, odd=odd, seed=0xFE11 + tx_len)
    _txseg_fenced(oracle, shm, sl, fr, segs, "end", "end", impl)


def test_guard_txseg_tso(oracle):
    n, pay = 16, 65535 - 52
    shm, fr, segs, sl = pktgen.tx_segments(n, payload=pay, stride=65536 + 64, tx_len=98304 + 5, nflows=4, odd=True)
    _txseg_fenced(oracle, shm, sl, fr, segs, "end", "start")


# ---------------------------------------------------------------------------
# TCP4 checksums and RX verification

def _frames_to_end(n, pay, stride, seed):
    """n TAS frames at `stride`, the buffer cut right after the last datagram."""
    fr = pktgen.tcp4_frames(n, payload=pay, stride=stride, seed=seed)
    end = (n - 1) * stride + 14 + 52 + int(np.broadcast_to(pay, (n,))[-1])
    return np.ascontiguousarray(fr[:end])


@pytest.mark.parametrize("form", ["frames_only", "uniform_hint", "per_frame_hints", "offsets"])
def test_guard_tcp4(oracle, form):
    n, stride = 4096, 2048
    if form == "uniform_hint":
        pay = np.full(n, pktgen.TCP_MSS)          # the headline batch: one MTU for all
    else:
        rng = np.random.default_rng(11)
        pay = np.where(rng.random(n) < 0.5, 0, rng.integers(1, pktgen.TCP_MSS + 1, n))
        pay[-1] = 0                               # a 66-byte ACK last, at the fence
    fr = _frames_to_end(n, pay, stride, 0x6A7D)
    exp = oracle.tcp4_batch(np.concatenate([fr, np.zeros(stride, np.uint8)]), n, stride=stride)
    out = torch.empty(2 * n, dtype=torch.int16, device=DEV)
    with _fenced(fr, "end") as g:
        kw = dict(stride=stride)
        if form == "uniform_hint":
            kw["frame_len"] = 14 + 52 + pktgen.TCP_MSS
        elif form == "per_frame_hints":
            kw["frame_len"] = torch.from_numpy((14 + 52 + pay).astype(np.int32)).to(DEV)
        elif form == "offsets":
            kw = dict(offsets=torch.from_numpy(np.arange(n, dtype=np.int64) * stride).to(DEV))
        xsum.tcp4_cksum_batch(g.addr, n, out=out, **kw)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint16)
        xsum.tcp4_cksum_batch(g.addr, n, inplace=True, want_out=False, **kw)   # the fields stored in place
        torch.cuda.synchronize()
        back = g.download()
    np.testing.assert_array_equal(got, exp)
    f = np.concatenate([back, np.zeros(stride, np.uint8)]).reshape(-1)[:n * stride].reshape(n, stride)
    np.testing.assert_array_equal(f[:, 24:26].copy().view(np.uint16).ravel(), exp[0::2])
    np.testing.assert_array_equal(f[:, 50:52].copy().view(np.uint16).ravel(), exp[1::2])


def test_guard_tcp4_room(oracle):
    """A room of the full stride: the batch ends at the last room's end."""
    n, stride = 4096, 2048
    fr = pktgen.tcp4_frames(n, payload=(np.arange(n) * 37) % 1449, stride=stride, seed=0x600D)
    exp = oracle.tcp4_batch(fr.copy(), n, stride=stride)
    out = torch.empty(2 * n, dtype=torch.int16, device=DEV)
    with _fenced(fr, "end") as g:
        xsum.tcp4_cksum_batch(g.addr, n, stride=stride, out=out, room=stride)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp)


@pytest.mark.parametrize("bound", ["per_frame", "uniform"])
def test_guard_verify(oracle, bound):
    n, stride = 4096, 2048
    rng = np.random.default_rng(5)
    pay = rng.integers(0, pktgen.TCP_MSS + 1, n) if bound == "per_frame" else np.full(n, pktgen.TCP_MSS)
    fr = pktgen.tcp4_frames(n, payload=pay, stride=stride, seed=0x7E1)
    oracle.tcp4_batch(fr, n, stride=stride, inplace=True)
    fr[3 * stride + 60] ^= 1                                   # one bad L4 sum
    rlen = (14 + 52 + pay).astype(np.int64)
    end = (n - 1) * stride + int(rlen[-1])
    fr = np.ascontiguousarray(fr[:end])
    exp = oracle.tcp4_verify_batch_bounded(np.concatenate([fr, np.zeros(stride, np.uint8)]), n,
                                           rlen.astype(np.uint32) if bound == "per_frame" else int(rlen[0]),
                                           stride=stride)
    out = torch.empty(n, dtype=torch.uint8, device=DEV)
    with _fenced(fr, "end") as g:
        fl = torch.from_numpy(rlen.astype(np.int32)).to(DEV) if bound == "per_frame" else int(rlen[0])
        xsum.tcp4_verify_batch(g.addr, n, stride=stride, out=out, frame_len=fl)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
    np.testing.assert_array_equal(got, exp)
    assert got[3] == 1 and (np.delete(got, 3) == 3).all()


# ---------------------------------------------------------------------------
# RAW

@pytest.mark.parametrize("form", ["stride", "uniform_s32", "lengths"])
def test_guard_raw(oracle, form):
    out = torch.empty(1 << 16, dtype=torch.int16, device=DEV)
    if form == "lengths":
        buf, offs, lens = pktgen.raw_mixed(20000, seed=0x9A1, odd=True)
        n = len(lens)
        end = int(offs[-1] + lens[-1])
        buf = np.ascontiguousarray(buf[:end])
        exp = oracle.raw_batch(np.concatenate([buf, np.zeros(16, np.uint8)]), n, offsets=offs, lengths=lens)
        with _fenced(buf, "end") as g:
            xsum.raw_cksum_batch(g.addr, n, offsets=torch.from_numpy(offs.astype(np.int64)).to(DEV),
                                 lengths=torch.from_numpy(lens.astype(np.int32)).to(DEV), out=out)
            torch.cuda.synchronize()
            got = out[:n].cpu().numpy().view(np.uint16)
    else:
        n, L = 40000, 1500 if form == "uniform_s32" else 1499
        buf = pktgen.random_bytes(0x5EA, n * L)
        exp = oracle.raw_batch(buf, n, stride=L, len0=L)
        with _fenced(buf, "end") as g:
            xsum.raw_cksum_batch(g.addr, n, stride=L, len0=L, out=out)
            torch.cuda.synchronize()
            got = out[:n].cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(got, exp)


# ---------------------------------------------------------------------------
# RX flow lookup and the one-pass RX

@pytest.mark.parametrize("call", ["lookup", "rx_pass"])
def test_guard_flow(oracle, call):
    nflows, ent, n = 4096, 8192, 20000
    keys = pktgen.flow_keys(nflows, seed=21)
    fs = pktgen.flow_state(keys, seed=21)
    fr_all = pktgen.rx_frames(keys, stride=128, seed=21)
    hashes, _ = oracle.flow_lookup_batch(fr_all, nflows, np.zeros(2, np.uint32), fs, fs_num=nflows, stride=128)
    ht, ok = pktgen.flow_table(hashes, ent)
    rng = np.random.default_rng(22)
    fkeys = keys[rng.integers(0, nflows, n)].copy()
    stride = 2048 if call == "rx_pass" else 128
    fr = pktgen.rx_frames(fkeys, stride=stride, seed=23)
    if call == "rx_pass":
        oracle.tcp4_batch(fr, n, stride=stride, inplace=True)
        fr = np.ascontiguousarray(fr[:(n - 1) * stride + 66])      # the last ACK ends at the fence
    else:
        fr = np.ascontiguousarray(fr[:(n - 1) * stride + 54])      # the last key's bytes end inside it
    pad = np.concatenate([fr, np.zeros(stride, np.uint8)])
    eh, ef = oracle.flow_lookup_batch(pad, n, ht, fs, fs_num=nflows, stride=stride)
    with _fenced(fr, "end") as gf, _fenced(ht.view(np.uint8), "end") as gh, _fenced(fs, "end") as gs:
        if call == "lookup":
            h, fid = xsum.flow_lookup_batch(gf.addr, n, gh.addr, gs.addr, nflows, stride=stride, ht_entries=ent)
            flags = None
        else:
            flags, h, fid = xsum.rx_batch(gf.addr, n, gh.addr, gs.addr, nflows, stride=stride, ht_entries=ent,
                                          frame_len=66)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), eh)
        np.testing.assert_array_equal(fid.cpu().numpy().view(np.uint32), ef)
        if flags is not None:
            assert (flags.cpu().numpy() == 3).all()
