"""Parity against the Linux TCP/IP stack's own checksums
(tests/golden/linux_frames.npz, made by tests/golden/gen_linux_frames.py).

The reference's end-to-end test pins TAS's software checksums by running TAS
with --fp-no-xsumoffload against the Linux stack, which drops segments with a
wrong checksum (/root/reference/tests/full/fulltest.c:103).  The fixture holds
one TCP connection over a TUN device: the frames Linux sent (its checksums,
computed in software) and the frames checksummed by the C oracle that Linux
accepted.  Here every frame gets its checksum fields overwritten and
recomputed -- by the C oracle, the numpy restatement and the GPU kernels in
each batch form -- and must come out as on the wire; and every frame must
verify.
"""
from pathlib import Path

import numpy as np
import pytest

from oracle import xsum_ref

FIX = Path(__file__).resolve().parent / "golden" / "linux_frames.npz"
ROOM = 2048


def _load():
    d = np.load(FIX)
    n = len(d["lens"])
    frames = d["frames"].reshape(n, ROOM)
    wire_ip = frames[:, 24:26].copy().view(np.uint16).ravel()
    wire_tcp = frames[:, 50:52].copy().view(np.uint16).ravel()
    scrubbed = frames.copy()
    scrubbed[:, 24:26] = 0x5A  # stale checksum fields, as tcp_checksums() finds them
    scrubbed[:, 50:52] = 0xA5
    return n, frames.ravel().copy(), scrubbed.ravel().copy(), d["lens"].astype(np.uint32), d["origin"], \
        wire_ip, wire_tcp


def test_fixture_shape():
    n, frames, _, lens, origin, _, _ = _load()
    assert n >= 60 and (origin == 0).sum() >= 30 and (origin == 1).sum() >= 20
    assert ((lens == 1514) & (origin == 0)).sum() >= 10          # TAS-sized MSS segments from Linux
    f = frames.reshape(n, ROOM)
    assert (f[:, 14] == 0x45).all() and (f[:, 23] == 6).all()     # IPv4, IHL 5, TCP: TAS's layout
    tl = f[:, 16].astype(np.uint32) << 8 | f[:, 17]
    np.testing.assert_array_equal(tl + 14, lens)
    assert len(set(tl.tolist())) >= 20 and (tl % 2 == 1).any()   # many lengths, odd ones included


def test_oracle_reproduces_linux(oracle):
    n, _, scrubbed, _, _, wire_ip, wire_tcp = _load()
    out = oracle.tcp4_batch(scrubbed, n, stride=ROOM)
    np.testing.assert_array_equal(out[0::2], wire_ip)
    np.testing.assert_array_equal(out[1::2], wire_tcp)


def test_numpy_restatement_reproduces_linux():
    n, _, scrubbed, _, _, wire_ip, wire_tcp = _load()
    f = scrubbed.reshape(n, ROOM)
    for i in range(n):
        fr = bytearray(f[i].tobytes())
        ip, tcp = xsum_ref.tcp_checksums(fr)
        assert (ip, tcp) == (wire_ip[i], wire_tcp[i]), i


def test_oracle_verifies_linux_frames(oracle):
    n, frames, _, lens, _, _, _ = _load()
    assert (oracle.tcp4_verify_batch(frames, n, stride=ROOM) == 3).all()
    assert (oracle.tcp4_verify_batch_bounded(frames, n, lens, stride=ROOM) == 3).all()


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["frames", "hints", "room", "offsets", "inplace"])
def test_gpu_reproduces_linux(form):
    import torch
    from tas_amd import xsum
    n, _, scrubbed, lens, _, wire_ip, wire_tcp = _load()
    dev = torch.from_numpy(scrubbed).cuda()
    kw = {"stride": ROOM}
    if form == "hints":
        kw["frame_len"] = torch.from_numpy(lens.astype(np.int32)).cuda()
    elif form == "room":
        kw["room"] = ROOM
    elif form == "offsets":
        kw = {"offsets": torch.from_numpy(np.arange(n, dtype=np.int64) * ROOM).cuda()}
    if form == "inplace":
        xsum.tcp4_cksum_batch(dev, n, stride=ROOM, inplace=True, want_out=False)
        torch.cuda.synchronize()
        f = dev.cpu().numpy().reshape(n, ROOM)
        np.testing.assert_array_equal(f[:, 24:26].copy().view(np.uint16).ravel(), wire_ip)
        np.testing.assert_array_equal(f[:, 50:52].copy().view(np.uint16).ravel(), wire_tcp)
        return
    out = xsum.tcp4_cksum_batch(dev, n, **kw)
    torch.cuda.synchronize()
    assert xsum.last_kernel().startswith("tcp4_tas14_kernel")
    o = out.cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(o[0::2], wire_ip)
    np.testing.assert_array_equal(o[1::2], wire_tcp)


@pytest.mark.gpu
def test_gpu_verifies_linux_frames():
    import torch
    from tas_amd import xsum
    n, frames, _, lens, _, _, _ = _load()
    dev = torch.from_numpy(frames).cuda()
    hints = torch.from_numpy(lens.astype(np.int32)).cuda()
    flags = xsum.tcp4_verify_batch(dev, n, stride=ROOM, frame_len=hints)
    torch.cuda.synchronize()
    assert (flags.cpu().numpy() == 3).all()
    flags2 = xsum.tcp4_verify_batch(dev, n, stride=ROOM)
    torch.cuda.synchronize()
    assert (flags2.cpu().numpy() == 3).all()


def _txseg_case():
    """The Linux data segments (66-byte headers: TCP with NOP NOP timestamp,
    TAS's layout) rebuilt by the TX segment build (SURVEY.md section 8f row 1,
    flow_tx_read + tcp_checksums, /root/reference/tas/fast/fast_flows.c:930-936):
    each payload placed in its own 4 KiB ring in a shared region -- every third
    one wrapping around its ring's end -- the frames handed over with the
    payload and both checksum fields scrambled, a descriptor per frame.  The
    build must give back Linux's frames byte for byte."""
    from tas_amd import pktgen
    n, frames, _, lens, origin, _, _ = _load()
    f = frames.reshape(n, ROOM)
    doff = f[:, 46] >> 4
    pay = lens.astype(np.int64) - 66
    sel = np.nonzero((origin == 0) & (doff == 8) & (pay > 0))[0]
    m = len(sel)
    ring = 4096
    shm = np.zeros(m * ring + 16, np.uint8)
    segs = np.zeros(m, pktgen.TX_SEG_DTYPE)
    want = f[sel].copy()
    got = want.copy()
    rng = np.random.default_rng(5)
    for j, i in enumerate(sel):
        p = int(pay[i])
        body = f[i, 66:66 + p]
        pos = ring - max(1, p // 2) if j % 3 == 0 else int(rng.integers(0, ring - p))
        base = j * ring
        idx = (pos + np.arange(p)) % ring
        shm[base + idx] = body
        got[j, 66:66 + p] = rng.integers(0, 256, p, dtype=np.uint8)
        got[j, 24:26] = 0x5A
        got[j, 50:52] = 0xA5
        segs[j] = (j * ROOM, base, ring, pos, p, 66, ROOM)
    wraps = int((segs["pos"].astype(np.int64) + segs["payload"] > ring).sum())
    return shm, len(shm), got.ravel().copy(), segs, want, wraps


def test_oracle_txseg_rebuilds_linux_frames(oracle):
    shm, sl, fr, segs, want, wraps = _txseg_case()
    assert len(segs) >= 20 and wraps >= 5 and (segs["payload"] == 1448).sum() >= 10
    out = oracle.tx_segment_batch(shm, sl, fr, segs)
    np.testing.assert_array_equal(fr.reshape(want.shape), want)
    np.testing.assert_array_equal(out & 0xFFFF, want[:, 24:26].copy().view(np.uint16).ravel())
    np.testing.assert_array_equal(out >> 16, want[:, 50:52].copy().view(np.uint16).ravel())


@pytest.mark.gpu
def test_gpu_txseg_rebuilds_linux_frames():
    import torch
    from tas_amd import xsum
    shm, sl, fr, segs, want, _ = _txseg_case()
    dshm = torch.from_numpy(shm).cuda()
    dfr = torch.from_numpy(fr).cuda()
    dsegs = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
    out = xsum.tx_segment_batch(dshm, dfr, dsegs, len(segs), shm_len=sl)
    torch.cuda.synchronize()
    assert xsum.last_kernel() == "tx_segment_lds_kernel"
    np.testing.assert_array_equal(dfr.cpu().numpy().reshape(want.shape), want)
    o = out.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(o & 0xFFFF, want[:, 24:26].copy().view(np.uint16).ravel())
    np.testing.assert_array_equal(o >> 16, want[:, 50:52].copy().view(np.uint16).ravel())


def _rx_tables(oracle):
    """A flow table holding the captured connection as the receiving end at
    10.77.0.2 sees it (local = ip.dest / tcp.dest, remote = ip.src / tcp.src of
    Linux's frames) among 63 other flows."""
    from tas_amd import pktgen
    n, frames, _, _, origin, _, _ = _load()
    f = frames.reshape(n, ROOM)
    i = int(np.nonzero(origin == 0)[0][0])
    conn = np.concatenate([f[i, 30:34], f[i, 26:30], f[i, 36:38], f[i, 34:36]]).astype(np.uint8)
    keys = np.concatenate([conn[None, :], pktgen.flow_keys(63, seed=77)])
    fs = pktgen.flow_state(keys, seed=77)
    hashes, _ = oracle.flow_lookup_batch(pktgen.rx_frames(keys, stride=128, seed=78), len(keys),
                                         np.zeros(2, np.uint32), fs, fs_num=len(keys), stride=128)
    ht, ok = pktgen.flow_table(hashes, 1024)
    assert ok[0]                                   # the connection is in the table
    return ht, fs, len(keys)


def test_oracle_rx_lookup_linux_frames(oracle):
    """The flow lookup finds the connection for every frame Linux sent and for
    none of the frames sent the other way."""
    n, frames, _, _, origin, _, _ = _load()
    ht, fs, nf = _rx_tables(oracle)
    _, fid = oracle.flow_lookup_batch(frames, n, ht, fs, fs_num=nf, stride=ROOM)
    assert (fid[origin == 0] == 0).all() and (fid[origin == 1] == 0xFFFFFFFF).all()


@pytest.mark.gpu
@pytest.mark.parametrize("uniform", [False, True])
def test_gpu_rx_pass_linux_frames(oracle, uniform):
    """One RX pass (tasx_rx_batch_dev) over the captured connection: every frame
    verifies, Linux's frames find their flow, the others do not -- against
    both oracles.  uniform: only Linux's full-MSS segments, with their received
    length as the uniform hint."""
    import torch
    from tas_amd import xsum
    n, frames, _, lens, origin, _, _ = _load()
    ht, fs, nf = _rx_tables(oracle)
    if uniform:
        sel = np.nonzero((origin == 0) & (lens == 1514))[0]
        frames = frames.reshape(n, ROOM)[sel].ravel().copy()
        n, lens, origin = len(sel), lens[sel], origin[sel]
        kw = {"frame_len": 1514}
    else:
        kw = {"frame_len": torch.from_numpy(lens.astype(np.int32)).cuda()}
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    flags, h, fid = xsum.rx_batch(t(frames), n, t(ht), t(fs), nf, stride=ROOM, **kw)
    torch.cuda.synchronize()
    assert xsum.last_kernel() == ("tcp4_tas14_kernel<hint,verify,flow>" if uniform
                                  else "tcp4_tas14_kernel<hints,verify,flow>")
    assert (flags.cpu().numpy() == 3).all()
    eh, ef = oracle.flow_lookup_batch(frames, n, ht, fs, fs_num=nf, stride=ROOM)
    np.testing.assert_array_equal(fid.cpu().numpy().view(np.uint32), ef)
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), eh)
    assert (ef[origin == 0] == 0).all() and (ef[origin == 1] == 0xFFFFFFFF).all()
