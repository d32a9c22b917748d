"""One RX pass (tasx_rx_batch_dev): checksum verification (SURVEY.md section
8f row 3) and the flow lookup of fast_flows_packet_fss()
(/root/reference/tas/fast/fast_flows.c:1084-1163, row 4) of the same frames.
The product must equal the two calls in turn: flags against the bounded
verification oracle, hashes and flow ids against the lookup oracle, on RX
bursts of data segments and pure ACKs with corrupted, padded and truncated
frames and unknown flows, in every row-kernel form and the general fallback.
"""
import numpy as np
import pytest

from tas_amd import pktgen


def _burst(oracle, n, stride, seed, uniform=False, nflows=4096, ent=8192):
    """n received TAS frames with flow keys (10 % unknown), valid checksums
    except where corrupted, the received lengths, and the flow tables."""
    keys = pktgen.flow_keys(nflows, seed=seed)
    fs = pktgen.flow_state(keys, seed=seed)
    hashes, _ = oracle.flow_lookup_batch(pktgen.rx_frames(keys, stride=128, seed=seed), nflows,
                                         np.zeros(2, np.uint32), fs, fs_num=nflows, stride=128)
    ht, ok = pktgen.flow_table(hashes, ent)
    rng = np.random.default_rng(seed)
    fkeys = keys[rng.integers(0, nflows, n)].copy()
    miss = rng.random(n) < 0.1
    fkeys[miss, 4] ^= 0x5A                                          # unknown remote ip
    if uniform:
        pay = np.full(n, pktgen.TCP_MSS, np.int64)
    else:
        pay = np.where(rng.random(n) < 0.5, 0, rng.integers(1, pktgen.TCP_MSS + 1, n)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=stride, seed=seed + 1)
    pktgen.set_flow_keys(frames, fkeys, stride)
    oracle.tcp4_batch(frames, n, stride=stride, inplace=True)
    f = frames.reshape(n, stride)
    rcv = 14 + 52 + pay
    if not uniform:
        pad = np.arange(n) % 7 == 1
        rcv[pad] = np.maximum(rcv[pad], 60) + 4 + (np.arange(n)[pad] % 9)
        trunc = np.arange(n) % 11 == 2
        rcv[trunc] = np.maximum(rcv[trunc] - 1 - np.arange(n)[trunc] % 40, 20)
    bad = np.arange(n) % 5 == 3
    pos = 14 + 38 + (rng.integers(0, 10 ** 6, n) % np.maximum(rcv - 14 - 38, 1))   # past the key bytes
    f[np.nonzero(bad)[0], np.minimum(pos[bad], stride - 1)] ^= 0x20
    f[4::13, 24] ^= 0x01                                            # ip.chksum
    f[6::17, 50] ^= 0x80                                            # tcp.chksum
    return frames, rcv, ht, fs, nflows, miss


FORMS = {  # form: (stride, offsets, bound, uniform, kernel)
    "hint": (2048, False, "uniform", True, "tcp4_tas14_kernel<hint,verify,flow>"),
    "hints": (2048, False, "len", False, "tcp4_tas14_kernel<hints,verify,flow>"),
    "tl_first": (2048, False, "none", False, "tcp4_tas14_kernel<tl_first,verify,flow>"),
    "room": (2048, False, "room", False, "tcp4_tas14_kernel<tl_first,verify,flow>"),
    "hints_offs": (2048, True, "len", False, "tcp4_tas14_kernel<hints,verify,offs,flow>"),
    "tl_first_offs": (2048, True, "none", False, "tcp4_tas14_kernel<tl_first,verify,offs,flow>"),
    "general": (2056, False, "len", False, "tcp4 verify + flow_lookup_kernel"),
}


@pytest.mark.gpu
@pytest.mark.parametrize("form", list(FORMS))
def test_rx_fused_forms(oracle, form):
    import torch
    from tas_amd import xsum
    stride, offs, bound, uniform, kernel = FORMS[form]
    n = 8192
    frames, rcv, ht, fs, nflows, miss = _burst(oracle, n, stride, seed=300 + len(form), uniform=uniform)
    dev = "cuda:0"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    kw = dict(offsets=t(np.arange(n, dtype=np.int64) * stride)) if offs else dict(stride=stride)
    if bound == "uniform":
        kw["frame_len"] = int(rcv[0])
        b = int(rcv[0])
    elif bound == "len":
        kw["frame_len"] = t(rcv.astype(np.int32))
        b = rcv.astype(np.uint32)
    elif bound == "room":
        kw["room"] = stride
        b = stride
    else:
        b = 0 if offs else stride
    exp_flags = oracle.tcp4_verify_batch_bounded(frames, n, b, stride=stride)
    exp_h, exp_fid = oracle.flow_lookup_batch(frames, n, ht, fs, fs_num=nflows, stride=stride)
    flags, h, fid = xsum.rx_batch(t(frames), n, t(ht), t(fs), nflows, **kw)
    torch.cuda.synchronize()
    assert xsum.last_kernel() == kernel
    np.testing.assert_array_equal(flags.cpu().numpy(), exp_flags)
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), exp_h)
    np.testing.assert_array_equal(fid.cpu().numpy().view(np.uint32), exp_fid)
    assert (fid.cpu().numpy().view(np.uint32)[miss] == 0xFFFFFFFF).all()
    assert 0.2 < (exp_flags == 3).mean() < 0.95                       # both verdicts present
    # without hashes, and against the two separate calls
    _, h2, fid2 = xsum.rx_batch(t(frames), n, t(ht), t(fs), nflows, want_hash=False, **kw)
    assert h2 is None
    sep_flags = xsum.tcp4_verify_batch(t(frames), n, **kw)
    sep_h, sep_fid = xsum.flow_lookup_batch(t(frames), n, t(ht), t(fs), nflows,
                                            offsets=kw.get("offsets"), stride=0 if offs else stride)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fid2.cpu().numpy(), sep_fid.cpu().numpy())
    np.testing.assert_array_equal(flags.cpu().numpy(), sep_flags.cpu().numpy())
    np.testing.assert_array_equal(h.cpu().numpy(), sep_h.cpu().numpy())


@pytest.mark.gpu
def test_rx_fused_ragged_and_errors():
    """Batch sizes that leave partial rows and blocks, n = 0, and the argument
    checks of both halves."""
    import torch
    from tas_amd import xsum
    dev = "cuda:0"
    fr = torch.zeros(64 * 2048, dtype=torch.uint8, device=dev)
    ht = torch.zeros(16, dtype=torch.int32, device=dev)
    fs = torch.zeros(128 * 4, dtype=torch.uint8, device=dev)
    for n in (1, 3, 17, 63):
        flags, _, fid = xsum.rx_batch(fr, n, ht, fs, 4, stride=2048, frame_len=1514)
        sep = xsum.tcp4_verify_batch(fr, n, stride=2048, frame_len=1514)
        torch.cuda.synchronize()
        assert (fid.cpu().numpy().view(np.uint32) == 0xFFFFFFFF).all()      # no valid entries
        np.testing.assert_array_equal(flags.cpu().numpy(), sep.cpu().numpy())
    assert xsum.rx_batch(fr, 0, ht, fs, 4, stride=2048)[2].numel() == 0
    with pytest.raises(xsum.TasxError):
        xsum.rx_batch(fr, 4, ht, fs, 0, stride=2048)                        # empty flow state
    with pytest.raises(xsum.TasxError):
        xsum.rx_batch(fr, 4, ht, fs, 4, stride=2048, fs_stride=130)         # misaligned flow table
    with pytest.raises(xsum.TasxError):
        xsum.rx_batch(fr, 4, ht, fs, 4, stride=2048, room=4096)             # room past the stride


@pytest.mark.gpu
@pytest.mark.parametrize("ent", [1, 2, 3, 5])
def test_rx_fused_tiny_tables(oracle, ent):
    """the lookup probes bucket entries (h + j) % ht_entries;
    tables smaller than a bucket (1-3 entries) wrap more than once, and every
    probe stays inside the table."""
    import torch
    from tas_amd import xsum
    n, stride = 600, 2048
    frames, rcv, _, fs, nflows, _ = _burst(oracle, n, stride, seed=950 + ent, nflows=8, ent=64)
    keys = pktgen.flow_keys(8, seed=950 + ent)
    hashes, _ = oracle.flow_lookup_batch(pktgen.rx_frames(keys, stride=128, seed=950 + ent), 8,
                                         np.zeros(2, np.uint32), fs, fs_num=8, stride=128)
    ht, _ = pktgen.flow_table(hashes, ent)
    dev = "cuda:0"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    exp_h, exp_fid = oracle.flow_lookup_batch(frames, n, ht, fs, fs_num=nflows, stride=stride)
    exp_flags = oracle.tcp4_verify_batch_bounded(frames, n, stride, stride=stride)
    flags, h, fid = xsum.rx_batch(t(frames), n, t(ht), t(fs), nflows, stride=stride)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(flags.cpu().numpy(), exp_flags)
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), exp_h)
    np.testing.assert_array_equal(fid.cpu().numpy().view(np.uint32), exp_fid)
    assert (fid.cpu().numpy().view(np.uint32) != 0xFFFFFFFF).any()


@pytest.mark.gpu
def test_rx_fused_uniform_batch_edges(oracle):
    """the uniform-received-length grid (XCD-matched lookup
    blocks with two frames per lane) at the same batch edges."""
    import torch
    from tas_amd import xsum
    frames, rcv, ht, fs, nflows, _ = _burst(oracle, 4200, 2048, seed=913, uniform=True)
    assert np.all(rcv == rcv[0])
    dev = "cuda:0"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    fr = t(frames)
    for n in (1, 15, 16, 17, 255, 256, 257, 511, 512, 513, 1024, 1300, 2047, 2048, 2049, 4095, 4096, 4097, 4200):
        exp_h, exp_fid = oracle.flow_lookup_batch(frames, n, ht, fs, fs_num=nflows, stride=2048)
        exp_flags = oracle.tcp4_verify_batch_bounded(frames, n, int(rcv[0]), stride=2048)
        flags, h, fid = xsum.rx_batch(fr, n, t(ht), t(fs), nflows, stride=2048, frame_len=int(rcv[0]))
        torch.cuda.synchronize()
        assert xsum.last_kernel() == "tcp4_tas14_kernel<hint,verify,flow>"
        np.testing.assert_array_equal(flags.cpu().numpy(), exp_flags)
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), exp_h)
        np.testing.assert_array_equal(fid.cpu().numpy().view(np.uint32), exp_fid)


@pytest.mark.gpu
def test_rx_fused_batch_edges(oracle):
    """Batch sizes around row, block and lookup-block boundaries (16 frames
    per verify block, 256 / 512 frames per lookup block, 2048 / 4096 frames per
    8 XCD-matched lookup blocks or per 128-block group): every frame verified
    and looked up once, in the product's split grid (lookup blocks first, each
    over the frames of the verify blocks on its own XCD)."""
    import torch
    from tas_amd import xsum
    frames, rcv, ht, fs, nflows, _ = _burst(oracle, 4200, 2048, seed=911)
    dev = "cuda:0"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    fr = t(frames)
    for n in (1, 15, 16, 17, 255, 256, 257, 511, 512, 513, 1024, 1300, 2047, 2048, 2049, 4095, 4096, 4097, 4200):
        exp_h, exp_fid = oracle.flow_lookup_batch(frames, n, ht, fs, fs_num=nflows, stride=2048)
        exp_flags = oracle.tcp4_verify_batch_bounded(frames, n, rcv[:n].astype(np.uint32), stride=2048)
        flags, h, fid = xsum.rx_batch(fr, n, t(ht), t(fs), nflows, stride=2048, frame_len=t(rcv[:n].astype(np.int32)))
        torch.cuda.synchronize()
        assert xsum.last_kernel() == "tcp4_tas14_kernel<hints,verify,flow>"
        np.testing.assert_array_equal(flags.cpu().numpy(), exp_flags)
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), exp_h)
        np.testing.assert_array_equal(fid.cpu().numpy().view(np.uint32), exp_fid)
