"""The timed call is the tested call.  For each BASELINE.json config and each
extra bench.py leg, bench.py's own workload object and C launch loop -- the
same entry point, hint, room, stride, batch size and alignment bench.py times
-- run once and are compared bit-exact with the oracle (out of place and in
place where the call writes frames), and the kernel the call launched is
asserted (tasx_last_kernel).  Reference interface: tcp_checksums() flag-off
branch, /root/reference/tas/fast/fast_flows.c:1058-1069.
"""
import numpy as np
import pytest
import torch

import bench
from tas_amd import benchloop, pktgen, xsum

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    xsum.lib()
    yield
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy()


def test_bench_config2_headline(oracle):
    """Config 2 (the headline): 65,536 TAS frames (ip.len 1500) at the 2048 B
    mbuf stride, tasx_tcp4_cksum_batch_dev_hint with flen0 = 1514, the batch
    rank 0 times first -- out of place, then in place."""
    wl = bench.Tcp4Workload(1, pktgen.SEED)
    assert (wl.n, wl.stride, wl.hint) == (65536, 2048, 1514)
    wl.loop(benchloop.HINT)(0, 1)
    assert xsum.last_kernel() == "tcp4_tas14_kernel<hint>"
    exp = oracle.tcp4_batch(wl.host.copy(), wl.n, stride=wl.stride)
    np.testing.assert_array_equal(host(wl.outs[0]).view(np.uint16), exp)
    wl.loop(benchloop.HINT, inplace=True)(0, 1)
    ref = wl.host.copy()
    oracle.tcp4_batch(ref, wl.n, stride=wl.stride, inplace=True)
    np.testing.assert_array_equal(host(wl.bufs[0]), ref)


def test_bench_config2_drop_in_forms(oracle):
    """The bench's tcp4_nohint (no hint, room = the mbuf data room) and
    tcp4_frames_only (tasx_tcp4_cksum_batch_dev) legs on the headline frames,
    and its rx_verify leg on the checksummed frames."""
    wl = bench.Tcp4Workload(1, pktgen.SEED + 1)
    exp = oracle.tcp4_batch(wl.host.copy(), wl.n, stride=wl.stride)
    for which, kw, name in ((benchloop.ROOM, dict(flen0=0, room=bench.STRIDE), "tcp4_tas14_kernel<room>"),
                            (benchloop.DEV, dict(flen0=0), "tcp4_tas14_kernel<tl_first>")):
        wl.outs[0].zero_()
        wl.loop(which, **kw)(0, 1)
        assert xsum.last_kernel() == name
        np.testing.assert_array_equal(host(wl.outs[0]).view(np.uint16), exp, err_msg=name)
    wl.loop(benchloop.ROOM, flen0=0, room=bench.STRIDE, inplace=True)(0, 1)
    ref = wl.host.copy()
    oracle.tcp4_batch(ref, wl.n, stride=wl.stride, inplace=True)
    np.testing.assert_array_equal(host(wl.bufs[0]), ref)
    rv = bench.RxVerifyWorkload(wl)
    rv.loop()(0, 1)
    assert xsum.last_kernel() == "tcp4_tas14_kernel<hint,verify>"
    got = host(wl.rx_flags[0])
    np.testing.assert_array_equal(got, oracle.tcp4_verify_batch_bounded(ref, wl.n, bench.FRAME_LEN, stride=wl.stride))
    assert np.all(got == 3)


def test_bench_flush_mix(oracle):
    """The flush_mix leg: 64K frames, half data segments and half pure ACKs,
    per-frame hints and the mbuf room (tasx_tcp4_cksum_batch_dev_room)."""
    mw = bench.FlushMixWorkload(1, pktgen.SEED + 500)
    mw.loop()(0, 1)
    assert xsum.last_kernel() == "tcp4_tas14_kernel<hints>"
    exp = oracle.tcp4_batch(mw.host.copy(), mw.n, stride=mw.stride)
    np.testing.assert_array_equal(host(mw.outs[0]).view(np.uint16), exp)


def test_bench_rx_mix(oracle):
    """The rx_verify_mix leg: the flush_mix frames after their TX checksums,
    verified with per-frame received lengths (tasx_tcp4_verify_batch_dev_hint)
    -- every frame verifies, bit-exact against the bounded oracle."""
    mw = bench.FlushMixWorkload(1, pktgen.SEED + 500)
    rm = bench.RxMixWorkload(mw)
    rm.loop()(0, 1)
    assert xsum.last_kernel() == "tcp4_tas14_kernel<hints,verify>"
    frames = host(mw.bufs[0])
    got = host(rm.flags[0])
    np.testing.assert_array_equal(got, oracle.tcp4_verify_batch_bounded(frames, mw.n, host(mw.flen).astype(np.uint32),
                                                                        stride=mw.stride))
    assert np.all(got == 3)


@pytest.mark.parametrize("ws,rank", [(1, 0), (4, 3)])
def test_bench_config3_mixed_mtu(oracle, ws, rank):
    """Config 3: 1,048,576 RAW packets, {64, 576, 1500, 9000} B in random order,
    per-packet offsets and lengths (tasx_raw_cksum_batch_dev); and rank 3's
    byte-balanced shard of it at N = 4."""
    wl = bench.mixed_workload(ws, rank)
    if ws == 1:
        assert wl.n == 1 << 20
    wl.loop()(0, 1)
    assert xsum.last_kernel() == "raw_wave_kernel"
    offs = host(wl.off).astype(np.uint64)
    lens = host(wl.lens).astype(np.uint32)
    exp = oracle.raw_batch(host(wl.bufs[0]), wl.n, offsets=offs, lengths=lens)
    np.testing.assert_array_equal(host(wl.outs[0]).view(np.uint16), exp)


@pytest.mark.parametrize("rank", [0, 7])
def test_bench_config4_shard(oracle, rank):
    """Config 4: one GPU's shard of 8,388,608 x 1500 B at N = 8 (1,048,576
    packets, stride mode), as rank `rank` of bench.py --gpus 8 --workload
    shard8m builds it."""
    wl = bench.shard8m_workload(8, rank)
    assert wl.n == 1 << 20
    wl.loop()(0, 1)
    assert xsum.last_kernel() == "raw_sad_kernel<s32>"
    exp = oracle.raw_batch(host(wl.bufs[0]), wl.n, stride=wl.len0, len0=wl.len0)
    np.testing.assert_array_equal(host(wl.outs[0]).view(np.uint16), exp)


def test_bench_config4_whole_on_one_gpu(oracle):
    """Config 4 at N = 1: all 8,388,608 x 1500 B (12.6 GB) on one GPU, as
    bench.py --workload shard8m --gpus 1 times it: 524,288 blocks, so the grid
    runs in XCD runs of 256 blocks (xcd_run, round 5); every packet compared
    with the oracle."""
    wl = bench.shard8m_workload(1, 0)
    assert wl.n == bench.SHARD8M_N == 1 << 23
    wl.loop()(0, 1)
    assert xsum.last_kernel() == "raw_sad_kernel<s32>"
    got = host(wl.outs[0]).view(np.uint16)
    buf = host(wl.bufs[0])
    exp = oracle.raw_batch(buf, wl.n, stride=wl.len0, len0=wl.len0)
    np.testing.assert_array_equal(got, exp)


def test_bench_config5_tso(oracle):
    """Config 5: 16,384 TSO segments (ip.len 65535, L4 65,515 B) in 65,552 B
    rooms, the frame length 65,549 as the uniform hint; out of place, then in
    place."""
    wl = bench.tso_workload(0)
    assert (wl.n, wl.stride, wl.hint) == (16384, 65552, 65549)
    wl.loop(benchloop.HINT)(0, 1)
    assert xsum.last_kernel() == "tcp4_tas_kernel"
    frames = host(wl.bufs[0])
    exp = oracle.tcp4_batch(frames.copy(), wl.n, stride=wl.stride)
    np.testing.assert_array_equal(host(wl.outs[0]).view(np.uint16), exp)
    wl.loop(benchloop.HINT, inplace=True)(0, 1)
    oracle.tcp4_batch(frames, wl.n, stride=wl.stride, inplace=True)
    np.testing.assert_array_equal(host(wl.bufs[0]), frames)


def test_bench_raw_leg(oracle):
    """The raw leg: 64K x 1500 B packed payloads, stride mode."""
    rw = bench.RawWorkload(1, pktgen.SEED + 1000)
    rw.loop()(0, 1)
    assert xsum.last_kernel() == "raw_sad_kernel<s32>"
    exp = oracle.raw_batch(host(rw.bufs[0]), rw.n, stride=rw.len0, len0=rw.len0)
    np.testing.assert_array_equal(host(rw.outs[0]).view(np.uint16), exp)


def test_bench_tx_segment_leg():
    """The tx_segment leg: 64K segments from 8192 flows' circular TX buffers;
    the built frames against the oracle's flow_tx_read + tcp_checksums."""
    tw = bench.TxSegWorkload(1, pktgen.SEED + 2000)
    tw.loop()(0, 1)
    assert xsum.last_kernel() == "tx_segment_lds_kernel"
    assert tw.cpu_check(0.05)["parity_vs_gpu"] == "bit-exact"


def test_bench_flow_lookup_leg():
    """The flow_lookup leg: 256K RX frames in a TAS-sized flow table."""
    fw = bench.FlowLookupWorkload(1, pktgen.SEED + 3000)
    fw.loop()(0, 1)
    assert xsum.last_kernel() == "flow_lookup_kernel"
    assert fw.cpu_check(0.05)["parity_vs_gpu"] == "bit-exact"


def test_bench_rx_pass_leg(oracle):
    """The rx_pass leg as timed: tasx_rx_batch_dev on 64K received frames (50%
    data / 50% ACKs, per-frame received lengths) in the TAS-sized flow table,
    and the two calls it replaces (RX_SEPARATE) -- both bit-exact against the
    oracles."""
    from tas_amd import benchloop
    fw = bench.FlowLookupWorkload(1, pktgen.SEED + 3000)
    rp = bench.RxPassWorkload(fw, 1, pktgen.SEED + 4000)
    frames = host(rp.bufs[0])
    flen = host(rp.flen).astype(np.uint32)
    exp_flags = oracle.tcp4_verify_batch_bounded(frames, rp.n, flen, stride=bench.STRIDE)
    exp_h, exp_fid = oracle.flow_lookup_batch(frames, rp.n, fw.ht_np, fw.fs_np, fs_num=fw.NFLOWS,
                                              stride=bench.STRIDE)
    assert np.all(exp_flags == 3)
    for which, kernel in ((benchloop.RX_FUSED, "tcp4_tas14_kernel<hints,verify,flow>"),
                          (benchloop.RX_SEPARATE, "flow_lookup_kernel")):
        for a in (rp.flags[0], rp.fids[0], rp.hashes[0]):
            a.fill_(0x5A)
        rp.loop(which)(0, 1)
        assert xsum.last_kernel() == kernel
        np.testing.assert_array_equal(host(rp.flags[0]), exp_flags)
        np.testing.assert_array_equal(host(rp.hashes[0]).view(np.uint32), exp_h)
        np.testing.assert_array_equal(host(rp.fids[0]).view(np.uint32), exp_fid)
