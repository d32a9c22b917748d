"""GPU parity: the HIP kernels (through libtasx's C ABI) against the CPU oracle
and the committed golden fixtures, bit-exact, at BASELINE.json's full sizes
plus the edge cases the reference path has (odd starts / tails, empty and
short segments, total_length < 20, the 0 -> 0xffff rules, in-place stores).

Run on the MI355X box:  python -m pytest tests -m gpu -x -q
"""
import contextlib
import ctypes

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


# the product's kernel selections (tasx_set_kernel_variant; round 6 retired the
# comparison build's variants)
VARIANTS = (0, 2, 3, 6, 7)


@contextlib.contextmanager
def kernel_variant(v: int):
    """Run the block with kernel variant v selected."""
    xsum.set_kernel_variant(v)
    try:
        yield
    finally:
        xsum.set_kernel_variant(0)


def to_dev(a: np.ndarray) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:
        a = a.copy()
    return torch.from_numpy(a).to(DEV)


def u16(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def dev_random(nbytes: int, seed: int) -> torch.Tensor:
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=DEV, generator=g)


# ---------------------------------------------------------------------------
# golden fixtures

def test_golden_raw(raw_golden):
    g = raw_golden
    n = len(g["lengths"])
    out = xsum.raw_cksum_batch(to_dev(g["buf"]), n, offsets=to_dev(g["offsets"].astype(np.int64)),
                               lengths=to_dev(g["lengths"].astype(np.int32)))
    np.testing.assert_array_equal(u16(out), g["expected"])


def test_kat_ipv4_header_public(oracle):
    """The published IPv4 header example inside a frame (ip at 14): ip.chksum
    bytes b8 61 from the GPU, every kernel variant, with and without a hint."""
    import json
    from pathlib import Path
    kat = json.loads((Path(__file__).parent / "golden" / "kat.json").read_text())["ipv4_header_public"]
    frame = np.zeros(2048, np.uint8)
    frame[14:34] = np.frombuffer(bytes.fromhex(kat["header_hex"]), np.uint8)
    frame[34:14 + 115] = np.arange(95, dtype=np.uint8) * 7
    exp = oracle.tcp4_batch(frame.copy(), 1, stride=2048)
    for v in (0, 2, 3, 6):
        with kernel_variant(v):
            for hint in (None, 14 + 115):
                got = u16(xsum.tcp4_cksum_batch(to_dev(frame), 1, stride=2048, frame_len=hint))
                assert int(got[0]).to_bytes(2, "little").hex() == kat["ip_chksum_bytes"]
                np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 15])
def test_golden_tcp4(tcp4_golden, shift):
    g = tcp4_golden
    n = len(g["offsets"])
    buf = torch.zeros(g["frames"].size + 64, dtype=torch.uint8, device=DEV)
    buf[shift:shift + g["frames"].size] = to_dev(g["frames"])
    out = xsum.tcp4_cksum_batch(buf[shift:], n, stride=int(g["stride"]))
    np.testing.assert_array_equal(u16(out), g["expected"])
    # not in place: frames untouched
    np.testing.assert_array_equal(buf[shift:shift + g["frames"].size].cpu().numpy(), g["frames"])


def test_golden_tcp4_inplace(tcp4_golden, oracle):
    g = tcp4_golden
    n, stride = len(g["offsets"]), int(g["stride"])
    dbuf = to_dev(g["frames"])
    out = xsum.tcp4_cksum_batch(dbuf, n, stride=stride, inplace=True)
    ref = g["frames"].copy()
    oracle.tcp4_batch(ref, n, stride=stride, inplace=True)
    np.testing.assert_array_equal(dbuf.cpu().numpy(), ref)
    np.testing.assert_array_equal(u16(out), g["expected"])
    # in place with no result array
    dbuf2 = to_dev(g["frames"])
    assert xsum.tcp4_cksum_batch(dbuf2, n, stride=stride, inplace=True, want_out=False) is None
    np.testing.assert_array_equal(dbuf2.cpu().numpy(), ref)


def test_kat_frame_on_gpu():
    f = np.frombuffer(bytes(pktgen.kat_frame()) + bytes(30), np.uint8)
    out = u16(xsum.tcp4_cksum_batch(to_dev(f), 1, stride=96))
    assert (int(out[0]), int(out[1])) == (pktgen.KAT_IP_CHKSUM, pktgen.KAT_TCP_CHKSUM)


# ---------------------------------------------------------------------------
# RAW edge sweeps

def test_raw_all_short_lengths_all_alignments(oracle):
    lens, offs = [], []
    pos = 0
    for L in range(0, 300):
        for sh in range(16):
            pos = (pos + 15) // 16 * 16 + sh
            offs.append(pos)
            lens.append(L)
            pos += L
    buf = pktgen.random_bytes(5, pos + 32)
    offs = np.asarray(offs, np.int64)
    lens = np.asarray(lens, np.int32)
    n = len(lens)
    exp = oracle.raw_batch(buf, n, offsets=offs, lengths=lens)
    got = u16(xsum.raw_cksum_batch(to_dev(buf), n, offsets=to_dev(offs), lengths=to_dev(lens)))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("fill", [0x00, 0xFF, 0x01])
def test_raw_constant_buffers(fill):
    """All-zero -> 0, all-0xff -> 0xffff (never 0), long buffers up to TASX_RAW_MAX_LEN."""
    for L in (1, 2, 15, 16, 17, 1500, 65535, 131072, 131073):
        buf = torch.full((L + 32,), fill, dtype=torch.uint8, device=DEV)
        exp = _raw_np(bytes([fill]) * L)
        for sh in (0, 1):
            out = u16(xsum.raw_cksum_batch(buf[sh:], 1, len0=L, stride=0))
            assert int(out[0]) == exp, (L, sh)
        if fill == 0:
            assert exp == 0
        if fill == 0xFF and L % 2 == 0:
            assert exp == 0xFFFF


def _raw_np(b: bytes) -> int:
    from oracle import xsum_ref
    return xsum_ref.raw_cksum(b)


def test_raw_uniform_stride_mode(oracle):
    for L, stride in ((1500, 1500), (1500, 1504), (1499, 1501), (64, 64), (9000, 9000)):
        n = 3000
        buf = pktgen.random_bytes(L * 7 + stride, n * stride + 16)
        exp = oracle.raw_batch(buf, n, stride=stride, len0=L)
        got = u16(xsum.raw_cksum_batch(to_dev(buf), n, stride=stride, len0=L))
        np.testing.assert_array_equal(got, exp, err_msg=f"L={L} stride={stride}")


def test_raw_mixed_odd(oracle):
    buf, offs, lens = pktgen.raw_mixed(20000, seed=11, odd=True)
    n = len(lens)
    exp = oracle.raw_batch(buf, n, offsets=offs, lengths=lens)
    got = u16(xsum.raw_cksum_batch(to_dev(buf), n, offsets=to_dev(offs.astype(np.int64)),
                                   lengths=to_dev(lens.astype(np.int32))))
    np.testing.assert_array_equal(got, exp)


# ---------------------------------------------------------------------------
# BASELINE.json configs at full size, bit-exact against the C oracle

def test_config2_raw_64k_1500(oracle):
    n, L = 65536, 1500
    d = dev_random(n * L, 2)
    h = d.cpu().numpy()
    exp = oracle.raw_batch(h, n, stride=L, len0=L)
    got = u16(xsum.raw_cksum_batch(d, n, stride=L, len0=L))
    np.testing.assert_array_equal(got, exp)


def test_config2_tcp4_64k_tas_frames(oracle):
    n = 65536
    frames = pktgen.tcp4_frames(n, payload=pktgen.TCP_MSS, stride=2048)
    exp = oracle.tcp4_batch(frames, n, stride=2048)
    got = u16(xsum.tcp4_cksum_batch(to_dev(frames), n, stride=2048))
    np.testing.assert_array_equal(got, exp)


def test_concurrent_contexts_on_streams(oracle):
    """Independent batches of several fast-path contexts in flight at once, on
    their own streams (bench.py's two_contexts leg): every batch bit-exact."""
    n, S = 8192, 4
    pays = [np.where(np.arange(n) % 3 == 0, (np.arange(n) * (7 + s)) % 1449, pktgen.TCP_MSS) for s in range(S)]
    frames = [pktgen.tcp4_frames(n, payload=pays[s], stride=2048, seed=100 + s) for s in range(S)]
    exp = [oracle.tcp4_batch(f, n, stride=2048) for f in frames]
    dev = [to_dev(f) for f in frames]
    hints = [to_dev((66 + p).astype(np.int32)) for p in pays]
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = [torch.empty(2 * n, dtype=torch.int16, device=DEV) for _ in range(S)]
    torch.cuda.synchronize()
    for rep in range(3):
        for s in range(S):
            xsum.tcp4_cksum_batch(dev[s], n, stride=2048, frame_len=hints[s] if rep != 1 else None,
                                  out=outs[s], stream=streams[s])
    torch.cuda.synchronize()
    for s in range(S):
        np.testing.assert_array_equal(u16(outs[s]), exp[s])


def test_config3_mixed_mtu_1M(oracle):
    n = 1 << 20
    lens = pktgen.mixed_lengths(n, seed=3).astype(np.int64)
    slot = (lens + 15) // 16 * 16
    offs = np.zeros(n, np.int64)
    np.cumsum(slot[:-1], out=offs[1:])
    total = int(offs[-1] + slot[-1])
    d = dev_random(total, 3)
    h = d.cpu().numpy()
    exp = oracle.raw_batch(h, n, offsets=offs, lengths=lens)
    got = u16(xsum.raw_cksum_batch(d, n, offsets=to_dev(offs), lengths=to_dev(lens.astype(np.int32))))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 4099])
def test_raw_wave_descriptor_orders(oracle, n):
    """raw_wave_kernel (a wave's 4 packets as one chunk sequence): packets in
    descending, repeated and interleaved order, empty and maximum-length
    (TASX_RAW_MAX_LEN) packets, batch sizes that leave a wave partly empty."""
    rng = np.random.default_rng(n)
    total = 3 << 20
    d = dev_random(total, 70 + n)
    h = d.cpu().numpy()
    lens = rng.choice([0, 1, 2, 15, 16, 17, 1500, 9000, 65535, 131073], n).astype(np.int64)  # 131073 = TASX_RAW_MAX_LEN
    offs = rng.integers(0, total - 131073, n).astype(np.int64)
    if n > 3:
        offs[1::4] = offs[0::4][:len(offs[1::4])]           # repeated packet
        offs[2::4] = np.sort(offs[2::4])[::-1]               # descending
    exp = oracle.raw_batch(h, n, offsets=offs, lengths=lens)
    for v in (0, 7):
        with kernel_variant(v):
            got = u16(xsum.raw_cksum_batch(d, n, offsets=to_dev(offs), lengths=to_dev(lens.astype(np.int32))))
        np.testing.assert_array_equal(got, exp, err_msg=f"variant {v}")


def test_raw_wave_span_beyond_4gib(oracle):
    """A wave whose packets lie more than 4 GiB apart takes raw_wave_kernel's
    64-bit addressing path (the 32-bit-offset path covers spans below 4 GiB)."""
    far = (4 << 30) + 4093                                   # odd: misaligned far packets
    big = torch.empty(far + 20000, dtype=torch.uint8, device=DEV)
    near = dev_random(20000, 81)
    big[:20000] = near
    big[far:far + 20000] = dev_random(20000, 82)
    lens = np.array([1500, 9000, 17, 9001, 64, 0, 1, 576], np.int64)
    offs = np.array([0, far, 3, far + 7, far + 10001, 5, 19999, 11], np.int64)
    hn = near.cpu().numpy()
    hf = big[far:far + 20000].cpu().numpy()
    exp = np.array([oracle.raw_batch(hf if o >= far else hn, 1, offsets=np.array([o - far if o >= far else o]),
                                     lengths=np.array([ln]))[0] for o, ln in zip(offs, lens)], np.uint16)
    got = u16(xsum.raw_cksum_batch(big, len(lens), offsets=to_dev(offs), lengths=to_dev(lens.astype(np.int32))))
    del big
    torch.cuda.empty_cache()
    np.testing.assert_array_equal(got, exp)


def test_config4_shard_1M_1500(oracle):
    """One GPU's shard of the 8M x 1500 B 8-GPU config (1,048,576 packets)."""
    n, L = 1 << 20, 1500
    d = dev_random(n * L, 4)
    h = d.cpu().numpy()
    exp = oracle.raw_batch(h, n, stride=L, len0=L)
    got = u16(xsum.raw_cksum_batch(d, n, stride=L, len0=L))
    np.testing.assert_array_equal(got, exp)


def test_config5_tso_64k_segments(oracle):
    """16,384 TSO-sized segments, ip.len 65535 (L4 65,515 B, odd tail)."""
    n, stride = 16384, 65552
    frames = pktgen.tcp4_frames(n, payload=0, stride=stride, seed=5, ip_total_len=65535)
    exp = oracle.tcp4_batch(frames, n, stride=stride)
    d = to_dev(frames)
    got = u16(xsum.tcp4_cksum_batch(d, n, stride=stride))
    np.testing.assert_array_equal(got, exp)
    # receiver-side property on the device: after in-place stores every IP header sums to 0xffff
    xsum.tcp4_cksum_batch(d, n, stride=stride, inplace=True, want_out=False)
    hdr = u16(xsum.raw_cksum_batch(d[14:], n, stride=stride, len0=20))
    assert np.all(hdr == 0xFFFF)


# ---------------------------------------------------------------------------
# TCP4 edges

def test_tcp4_varied_payloads_offsets(oracle):
    n = 4096
    pay = (pktgen.splitmix64(77, n) % np.uint64(1449)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=77)
    # scatter the frames to random (odd and even) offsets in a bigger buffer
    shift = (pktgen.splitmix64(78, n) % np.uint64(200)).astype(np.int64)
    offs = np.arange(n, dtype=np.int64) * 2304 + shift
    big = np.zeros(n * 2304 + 2048, np.uint8)
    for i in range(n):
        big[offs[i]:offs[i] + 2048] = frames[i * 2048:(i + 1) * 2048]
    exp = oracle.tcp4_batch(big, n, offsets=offs)
    got = u16(xsum.tcp4_cksum_batch(to_dev(big), n, offsets=to_dev(offs)))
    np.testing.assert_array_equal(got, exp)


def test_tcp4_ack_sized_and_short(oracle):
    """ACKs (ip.len 52), SYN-sized (56), and total_length 0..60."""
    n = 61 * 8
    tl = np.tile(np.arange(61), 8)
    frames = pktgen.tcp4_frames(n, payload=0, stride=128, seed=9, ip_total_len=tl)
    exp = oracle.tcp4_batch(frames, n, stride=128)
    got = u16(xsum.tcp4_cksum_batch(to_dev(frames), n, stride=128))
    np.testing.assert_array_equal(got, exp)


def test_tcp4_nonstandard_offsets(oracle):
    """ip/l4 offsets other than TAS's 14/34 (e.g. VLAN-tagged, IP options)."""
    n = 1024
    frames = pktgen.tcp4_frames(n, payload=700, stride=2048, seed=12)
    exp = oracle.tcp4_batch(frames, n, stride=2048, ip_off=14, l4_off=38)
    got = u16(xsum.tcp4_cksum_batch(to_dev(frames), n, stride=2048, ip_off=14, l4_off=38))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("variant", [0])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 4099])
@pytest.mark.parametrize("ack_frac", [0.0, 0.5, 0.9])
def test_tcp4_flush_mix_per_frame_hints(oracle, n, ack_frac, variant):
    """tx_flush-shaped batches with per-frame hints (automatic: tcp4_tas_kernel;
    8: tcp4_wave_kernel): data segments among pure ACKs (ip.len 52), ragged batch
    ends, a few hints that disagree with ip.total_length or do not cover ip + 40,
    in place and to the output array."""
    with kernel_variant(variant):
        _flush_mix(oracle, n, ack_frac)


def _flush_mix(oracle, n, ack_frac):
    rng = np.random.default_rng(n * 7 + int(ack_frac * 10))
    pay = np.where(rng.random(n) < ack_frac, 0, rng.integers(1, pktgen.TCP_MSS + 1, n)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=n + 3)
    hint = (14 + 52 + pay).astype(np.int32)
    hint[5::37] -= 1           # short hint: the row body redoes the frame
    hint[6::37] += 7           # long hint
    hint[7::37] = 40           # does not cover tcp.chksum
    exp = oracle.tcp4_batch(frames.copy(), n, stride=2048)
    d = to_dev(frames)
    got = u16(xsum.tcp4_cksum_batch(d, n, stride=2048, frame_len=to_dev(hint)))
    np.testing.assert_array_equal(got, exp)
    xsum.tcp4_cksum_batch(d, n, stride=2048, frame_len=to_dev(hint), inplace=True, want_out=False)
    f = d.cpu().numpy().reshape(n, 2048)
    np.testing.assert_array_equal(f[:, 24:26].copy().view(np.uint16).ravel(), exp[0::2])
    np.testing.assert_array_equal(f[:, 50:52].copy().view(np.uint16).ravel(), exp[1::2])


def test_tcp4_wave_odd_offsets(oracle):
    """Per-frame hints with frames at odd and even offsets (odd IPv4 headers go
    to the row body, even ones are flattened)."""
    n = 2048
    pay = np.where(np.arange(n) % 3 == 0, 0, 1448 - (np.arange(n) % 200)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=81)
    shift = (pktgen.splitmix64(82, n) % np.uint64(100)).astype(np.int64)
    offs = np.arange(n, dtype=np.int64) * 2176 + shift
    big = np.zeros(n * 2176 + 2048, np.uint8)
    for i in range(n):
        big[offs[i]:offs[i] + 2048] = frames[i * 2048:(i + 1) * 2048]
    exp = oracle.tcp4_batch(big, n, offsets=offs)
    hint = (14 + 52 + pay).astype(np.int32)
    for v in (0, 2):
        with kernel_variant(v):
            got = u16(xsum.tcp4_cksum_batch(to_dev(big), n, offsets=to_dev(offs), frame_len=to_dev(hint)))
        np.testing.assert_array_equal(got, exp, err_msg=f"variant {v}")


@pytest.mark.parametrize("variant", VARIANTS)
def test_tcp4_all_variants_and_hints(oracle, variant):
    """Every kernel variant, with and without frame-length hints (exact, short,
    long, zero, garbage): results follow ip.total_length only."""
    n = 3000
    pay = (pktgen.splitmix64(55, n) % np.uint64(1449)).astype(np.int64)
    pay[::97] = 0
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=55)
    tl = 52 + pay
    tl[::101] = 10     # total_length < 20
    tl[1::101] = 20
    tl[2::101] = 37
    f = frames.reshape(n, 2048)
    f[:, 16] = (tl >> 8) & 0xFF
    f[:, 17] = tl & 0xFF
    exp = oracle.tcp4_batch(frames.copy(), n, stride=2048)
    d = to_dev(frames)
    exact = (14 + tl).astype(np.int32)
    noise = (pktgen.splitmix64(56, n) % np.uint64(4000)).astype(np.int32)
    with kernel_variant(variant):
        for hint in (None, 1514, 64, 2048, 0, to_dev(exact), to_dev(noise), to_dev(exact // 2)):
            got = u16(xsum.tcp4_cksum_batch(d, n, stride=2048, frame_len=hint))
            np.testing.assert_array_equal(got, exp, err_msg=f"variant {variant} hint {hint if isinstance(hint, (int, type(None))) else 'array'}")


@pytest.mark.parametrize("variant", VARIANTS)
def test_raw_all_variants(oracle, variant):
    buf, offs, lens = pktgen.raw_mixed(6000, seed=57, sizes=(0, 1, 3, 64, 255, 576, 1500, 1501, 9000), odd=True)
    n = len(lens)
    exp = oracle.raw_batch(buf, n, offsets=offs, lengths=lens)
    with kernel_variant(variant):
        got = u16(xsum.raw_cksum_batch(to_dev(buf), n, offsets=to_dev(offs.astype(np.int64)),
                                       lengths=to_dev(lens.astype(np.int32))))
        np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("variant", [0, 3])
def test_tso_with_hints(oracle, variant):
    n, stride = 512, 65552
    frames = pktgen.tcp4_frames(n, payload=0, stride=stride, seed=58,
                                ip_total_len=np.where(np.arange(n) % 3 == 0, 65535, 30000))
    exp = oracle.tcp4_batch(frames.copy(), n, stride=stride)
    d = to_dev(frames)
    with kernel_variant(variant):
        for hint in (None, 65549, 1514, stride):
            np.testing.assert_array_equal(u16(xsum.tcp4_cksum_batch(d, n, stride=stride, frame_len=hint)), exp)


@pytest.mark.parametrize("variant", [0, 6])
def test_tcp4_uniform_hint_every_size(oracle, variant):
    """Uniform-MTU batches (one frame-length hint for the batch, as bench.py
    passes it): every datagram size the headline kernel takes (ip.len 64..1522)
    and the sizes around it, in place and to the result array; then the same
    hint over frames whose total_length disagrees with it (the general body
    redoes those groups)."""
    with kernel_variant(variant):
        for tl in list(range(40, 1540, 7)) + [63, 64, 65, 1500, 1521, 1522, 1523]:
            n = 48
            frames = pktgen.tcp4_frames(n, payload=0, stride=1536 + 64, seed=tl, ip_total_len=tl)
            exp = oracle.tcp4_batch(frames.copy(), n, stride=1600)
            d = to_dev(frames)
            got = u16(xsum.tcp4_cksum_batch(d, n, stride=1600, frame_len=14 + tl))
            np.testing.assert_array_equal(got, exp, err_msg=f"ip.len {tl}")
            xsum.tcp4_cksum_batch(d, n, stride=1600, frame_len=14 + tl, inplace=True, want_out=False)
            f = d.cpu().numpy().reshape(n, 1600)
            ipc = f[:, 24].astype(np.uint16) | (f[:, 25].astype(np.uint16) << 8)
            tcpc = f[:, 50].astype(np.uint16) | (f[:, 51].astype(np.uint16) << 8)
            np.testing.assert_array_equal(ipc, exp[0::2], err_msg=f"in place ip.len {tl}")
            np.testing.assert_array_equal(tcpc, exp[1::2], err_msg=f"in place ip.len {tl}")
        # one hint, mixed total_length: every 5th frame disagrees with it
        n = 4096
        tl = np.full(n, 1500)
        tl[::5] = (pktgen.splitmix64(3, n)[::5] % np.uint64(1600)).astype(np.int64)
        frames = pktgen.tcp4_frames(n, payload=1448, stride=2048, seed=4, ip_total_len=tl)
        exp = oracle.tcp4_batch(frames.copy(), n, stride=2048)
        got = u16(xsum.tcp4_cksum_batch(to_dev(frames), n, stride=2048, frame_len=1514))
        np.testing.assert_array_equal(got, exp)


def test_deterministic_and_n0():
    frames = pktgen.tcp4_frames(1000, stride=2048)
    d = to_dev(frames)
    a = u16(xsum.tcp4_cksum_batch(d, 1000, stride=2048))
    b = u16(xsum.tcp4_cksum_batch(d, 1000, stride=2048))
    np.testing.assert_array_equal(a, b)
    assert xsum.raw_cksum_batch(d, 0, len0=5).numel() == 0


# ---------------------------------------------------------------------------
# host-memory surfaces: deferred tcp_checksums()/tx_flush and end-to-end batches

def test_deferred_tcp_checksums_flush(oracle):
    xsum.ctx_init(0, 0, 1 << 20)
    try:
        n = 32  # TXBUF_SIZE, tas/include/fastpath.h:38
        pay = np.arange(n) * 45
        frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=21)
        ref = frames.copy()
        oracle.tcp4_batch(ref, n, stride=2048, inplace=True)
        base = frames.ctypes.data
        for i in range(n):
            if i % 2:
                xsum.tcp_checksums(0, base + i * 2048)
            else:
                xsum.fast_flows_kernelxsums(0, base + i * 2048)
        assert xsum.pending(0) == n
        xsum.tx_flush(0)
        assert xsum.pending(0) == 0
        np.testing.assert_array_equal(frames, ref)
        # many flushes of varying size, including a frame larger than a slot's share
        for k in (1, 7, 200):
            fr = pktgen.tcp4_frames(k, payload=1448, stride=2048, seed=100 + k)
            rf = fr.copy()
            oracle.tcp4_batch(rf, k, stride=2048, inplace=True)
            for i in range(k):
                xsum.defer_tcp4(0, fr.ctypes.data + i * 2048)
            xsum.tx_flush(0)
            np.testing.assert_array_equal(fr, rf)
    finally:
        xsum.ctx_destroy(0)


def test_host_batch_end_to_end(oracle):
    xsum.ctx_init(1, 0, 8 << 20)  # small slots: many pipelined chunks
    try:
        n = 20000
        frames = pktgen.tcp4_frames(n, stride=2048, seed=31)
        pin = xsum.PinnedBuffer(frames.size)
        pin.array[:] = frames
        out = np.empty(2 * n, np.uint16)
        xsum.tcp4_cksum_batch_host(1, pin.addr, 2048, n, out.ctypes.data, inplace=True)
        ref = frames.copy()
        exp = oracle.tcp4_batch(ref, n, stride=2048, inplace=True)
        np.testing.assert_array_equal(out, exp)
        np.testing.assert_array_equal(pin.array, ref)
        pin.free()
        raw, stride = pktgen.raw_uniform(30000, 1500, seed=32)
        pin = xsum.PinnedBuffer(raw.size)
        pin.array[:] = raw
        out = np.empty(30000, np.uint16)
        xsum.raw_cksum_batch_host(1, pin.addr, 1500, 1500, 30000, out.ctypes.data)
        np.testing.assert_array_equal(out, oracle.raw_batch(raw, 30000, stride=1500, len0=1500))
        pin.free()
    finally:
        xsum.ctx_destroy(1)


def test_zero_copy_flush(oracle):
    """Frames in a registered host region: tasx_flush reads them over PCIe and
    stores the checksums in place with no staging copies."""
    xsum.ctx_init(3, 0, 1 << 20)
    try:
        n = 32
        pay = (np.arange(n) * 47) % 1449
        frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=61)
        ref = frames.copy()
        oracle.tcp4_batch(ref, n, stride=2048, inplace=True)
        pin = xsum.PinnedBuffer(frames.size)
        pin.array[:] = frames
        xsum.register_frames(3, pin.addr, pin.nbytes)
        for rnd in range(3):  # reuse of the same frames (stale-cache check)
            pin.array[:] = frames
            for i in range(n):
                xsum.tcp_checksums(3, pin.addr + i * 2048)
            xsum.tx_flush(3)
            np.testing.assert_array_equal(pin.array, ref)
        z, st = xsum.ctx_stats(3)
        assert z == 3 and st == 0
        # a frame outside the region takes the staged path
        outside = pktgen.tcp4_frames(1, payload=100, stride=2048, seed=62)
        ref1 = outside.copy()
        oracle.tcp4_batch(ref1, 1, stride=2048, inplace=True)
        pin.array[:] = frames
        xsum.tcp_checksums(3, pin.addr)
        xsum.tcp_checksums(3, outside.ctypes.data)
        xsum.tx_flush(3)
        np.testing.assert_array_equal(outside, ref1)
        np.testing.assert_array_equal(pin.array[:2048], ref[:2048])
        assert xsum.ctx_stats(3) == (3, 1)
        pin.free()
    finally:
        xsum.ctx_destroy(3)


@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("shift", [0, 1, 9])
def test_flush_records_as_frame_starts(oracle, zero_copy, shift):
    """tasx_flush hands its records over as TAS frame starts (IPv4 at 14, TCP
    at 34, per-frame hints 14 + total_length) so both flush paths take
    tcp4_tas14_kernel<hints,offs>: frames shifted off 16-byte alignment (rows
    redone by the general row body), total_length 0..60 next to data
    segments, and -- zero-copy -- a region that starts at a frame's IPv4
    header (no room for the 14-byte lead: that flush keeps header records)."""
    ctx = 6
    xsum.ctx_init(ctx, 0, 1 << 20)
    try:
        n = 40
        pay = np.where(np.arange(n) % 4 == 0, 0, (np.arange(n) * 37) % 1449)
        frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=81 + shift)
        f = frames.reshape(n, 2048)
        short = np.arange(0, n, 5)
        tl = (np.arange(len(short)) * 7) % 61           # 0, 7, ..., 56: the general body's cases
        f[short, 16] = tl >> 8
        f[short, 17] = tl & 0xFF
        buf = np.zeros(n * 2048 + 64, np.uint8)
        if zero_copy:
            pin = xsum.PinnedBuffer(buf.size)
            buf, base = pin.array, pin.addr
        else:
            base = buf.ctypes.data
        view = buf[shift:shift + n * 2048].reshape(n, 2048)
        view[:] = f
        ref = f.copy()
        oracle.tcp4_batch(ref.reshape(-1), n, stride=2048, inplace=True)
        if zero_copy:
            # the region starts at frame 0's IPv4 header: frame 0 has no lead
            xsum.register_frames(ctx, base + shift + 14, n * 2048 - 14)
        addrs = [base + shift + i * 2048 for i in range(n)]
        for i in range(1, n):
            xsum.tcp_checksums(ctx, addrs[i])
        xsum.tx_flush(ctx)
        assert xsum.last_kernel() == "tcp4_tas14_kernel<hints,offs>"
        np.testing.assert_array_equal(view[1:], ref[1:])
        xsum.tcp_checksums(ctx, addrs[0])
        xsum.tx_flush(ctx)
        assert xsum.last_kernel() == ("tcp4_frame_kernel" if zero_copy else "tcp4_tas14_kernel<hints,offs>")
        np.testing.assert_array_equal(view, ref)
        z, st = xsum.ctx_stats(ctx)
        assert (z, st) == ((2, 0) if zero_copy else (0, 2))
        if zero_copy:
            pin.free()
    finally:
        xsum.ctx_destroy(ctx)


def _feeder_frames(nframes: int, seed: int):
    """tx_flush-shaped frames (data segments, ACKs, short total_length) in a
    pinned region with their expected in-place checksums."""
    pay = np.where(np.arange(nframes) % 3 == 0, 0, (np.arange(nframes) * 53 + seed) % 1449)
    frames = pktgen.tcp4_frames(nframes, payload=pay, stride=2048, seed=seed)
    f = frames.reshape(nframes, 2048)
    short = np.arange(5, nframes, 97)
    f[short, 16], f[short, 17] = 0, (np.arange(len(short)) * 7) % 38   # total_length < 38: general body
    ref = frames.copy()
    oracle_ref = ref  # filled by the caller's oracle
    pin = xsum.PinnedBuffer(frames.size + 4096)
    pin.array[:] = 0
    pin.array[:frames.size] = frames
    return pin, frames, oracle_ref


def test_shared_feeder(oracle):
    """tasx_feeder_start + tasx_ctx_use_feeder: three contexts' flushes,
    submitted interleaved, served by the GPU's one feeder thread (one launch
    per sweep, absolute frame addresses from several regions); completions in
    each context's ticket order; a batch with a frame outside the region is
    flushed by its context after its feeder tickets; stop refuses while
    contexts are attached; detach, stop."""
    ctxs, nb, n = (8, 9, 10), 12, 32
    xsum.feeder_start(0)
    pins = []
    try:
        with pytest.raises(xsum.TasxError):
            xsum.feeder_start(0)                       # one feeder per GPU
        for k, c in enumerate(ctxs):
            xsum.ctx_init(c, 0, 1 << 20)
            pin, frames, ref = _feeder_frames(nb * n, 300 + k)
            oracle.tcp4_batch(ref, nb * n, stride=2048, inplace=True)
            with pytest.raises(xsum.TasxError):
                xsum.use_feeder(c)                     # no frame region yet
            xsum.register_frames(c, pin.addr, pin.nbytes)
            xsum.use_feeder(c)
            pins.append((pin, ref))
        tickets = {c: [] for c in ctxs}
        for b in range(nb):
            for k, c in enumerate(ctxs):
                for i in range(n):
                    xsum.tcp_checksums(c, pins[k][0].addr + (b * n + i) * 2048)
                tickets[c].append(xsum.flush_submit(c))
        for c in ctxs:
            assert tickets[c] == list(range(1, nb + 1))
            xsum.flush_wait(c, tickets[c][-1])
            assert all(xsum.flush_poll(c, t) for t in tickets[c])
            assert xsum.feeder_flushes(c) == nb and xsum.ctx_stats(c) == (0, 0)
        for k, c in enumerate(ctxs):
            pin, ref = pins[k]
            np.testing.assert_array_equal(pin.array[:ref.size], ref)
        sweeps, frames_done = xsum.feeder_stats(0)
        assert frames_done == len(ctxs) * nb * n and 1 <= sweeps <= len(ctxs) * nb
        # a frame outside the region: that batch goes through the context itself
        outside = pktgen.tcp4_frames(2, payload=np.array([100, 1448]), stride=2048, seed=401)
        ref_out = outside.copy()
        oracle.tcp4_batch(ref_out, 2, stride=2048, inplace=True)
        pin, ref = pins[0]
        pin.array[:2048] = 0
        pin.array[:2048] = ref[:2048]
        pin.array[24:26] = 0                                                  # stale field
        xsum.tcp_checksums(ctxs[0], pin.addr)                                 # a feeder batch
        t1 = xsum.flush_submit(ctxs[0])
        xsum.tcp_checksums(ctxs[0], outside.ctypes.data)
        xsum.tcp_checksums(ctxs[0], outside.ctypes.data + 2048)
        t2 = xsum.flush_submit(ctxs[0])
        assert t2 == t1 + 1
        xsum.flush_wait(ctxs[0], t2)
        np.testing.assert_array_equal(outside, ref_out)
        np.testing.assert_array_equal(pin.array[:2048], ref[:2048])
        assert xsum.ctx_stats(ctxs[0]) == (0, 1) and xsum.feeder_flushes(ctxs[0]) == nb + 1
        with pytest.raises(xsum.TasxError):
            xsum.feeder_stop(0)                                               # contexts attached
        for c in ctxs:
            xsum.use_feeder(c, False)
        xsum.feeder_stop(0)
    finally:
        for c in ctxs:
            try:
                xsum.ctx_destroy(c)
            except xsum.TasxError:
                pass
        try:
            xsum.feeder_stop(0)
        except xsum.TasxError:
            pass
        for pin, _ in pins:
            pin.free()


def test_shared_feeder_threads(oracle):
    """Four fast-path threads, each with its own context bound
    (tasx_set_thread_ctx) and attached to the feeder, each submitting 60
    tx_flush batches with up to 3 in flight (poll, then wait for the oldest),
    concurrently: every frame of every thread checksummed exactly."""
    import threading
    ctxs, nb, n = (11, 12, 13, 14), 60, 32
    xsum.feeder_start(0)
    pins, errs = [], []
    try:
        for k, c in enumerate(ctxs):
            xsum.ctx_init(c, 0, 1 << 20)
            pin, frames, ref = _feeder_frames(nb * n, 500 + k)
            oracle.tcp4_batch(ref, nb * n, stride=2048, inplace=True)
            xsum.register_frames(c, pin.addr, pin.nbytes)
            xsum.use_feeder(c)
            pins.append((pin, ref))

        def core(k, c):
            try:
                xsum.set_thread_ctx(c)
                inflight = []
                for b in range(nb):
                    for i in range(n):
                        xsum.tcp_checksums(xsum.CTX_SELF, pins[k][0].addr + (b * n + i) * 2048)
                    inflight.append(xsum.flush_submit(xsum.CTX_SELF))
                    while inflight and xsum.flush_poll(xsum.CTX_SELF, inflight[0]):
                        inflight.pop(0)
                    if len(inflight) >= 3:
                        xsum.flush_wait(xsum.CTX_SELF, inflight.pop(0))
                if inflight:
                    xsum.flush_wait(xsum.CTX_SELF, inflight[-1])
                xsum.set_thread_ctx(xsum.CTX_SELF)
            except Exception as e:  # reported below
                errs.append(e)
        th = [threading.Thread(target=core, args=(k, c)) for k, c in enumerate(ctxs)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert not errs, errs
        for k, c in enumerate(ctxs):
            pin, ref = pins[k]
            np.testing.assert_array_equal(pin.array[:ref.size], ref)
            assert xsum.feeder_flushes(c) == nb
        for c in ctxs:
            xsum.use_feeder(c, False)
        xsum.feeder_stop(0)
    finally:
        for c in ctxs:
            try:
                xsum.ctx_destroy(c)
            except xsum.TasxError:
                pass
        try:
            xsum.feeder_stop(0)
        except xsum.TasxError:
            pass
        for pin, _ in pins:
            pin.free()


@pytest.mark.parametrize("offs", [False, True])
def test_offload_branch_phdr(oracle, offs):
    """tasx_tcp4_offload_batch_dev, the fp_xsumoffload branch of tcp_checksums
    (network_ip_phdr_xsum via tx_xsum_enable, not inverted, ip.chksum zeroed):
    random addresses, total_length 0..65535 (the 16-bit l3_paylen wraps below
    20), odd frame starts; against the oracle's restatement, out of place and in
    place (nothing else in the frame changes)."""
    n, stride = 5003, 96
    rng = np.random.default_rng(33 + offs)
    buf = rng.integers(0, 256, n * stride + 64, dtype=np.uint8)
    starts = np.arange(n, dtype=np.int64) * stride + (np.arange(n) % 3 if offs else 0)
    tl = rng.integers(0, 65536, n)
    tl[:40] = np.arange(40)
    for k, st in enumerate(starts):
        buf[st + 16], buf[st + 17] = tl[k] >> 8, tl[k] & 0xFF
    exp = np.array([oracle.ip_phdr_xsum(int(buf[st + 26:st + 30].view(np.uint32)[0]),
                                        int(buf[st + 30:st + 34].view(np.uint32)[0]), 6, int(tl[k] - 20) & 0xFFFF)
                    for k, st in enumerate(starts)], np.uint16)
    d = to_dev(buf)
    kw = dict(offsets=to_dev(starts)) if offs else dict(stride=stride)
    got = u16(xsum.tcp4_offload_batch(d, n, **kw))
    assert xsum.last_kernel() == "tcp4_offload_kernel"
    np.testing.assert_array_equal(got, exp)
    xsum.tcp4_offload_batch(d, n, inplace=True, want_out=False, **kw)
    h = d.cpu().numpy()
    want = buf.copy()
    for k, st in enumerate(starts):
        want[st + 24:st + 26] = 0
        want[st + 50:st + 52] = np.frombuffer(int(exp[k]).to_bytes(2, "little"), np.uint8)
    np.testing.assert_array_equal(h, want)


def test_zero_copy_needs_chunk_slack(oracle):
    """A frame whose datagram ends less than 16 bytes before the registered
    region's end is not read in place (rows read whole 16-byte chunks): that
    flush goes through staging, and its checksums are still exact."""
    ctx = 7
    xsum.ctx_init(ctx, 0, 1 << 20)
    try:
        frames = pktgen.tcp4_frames(2, payload=np.array([1448, 100]), stride=2048, seed=91)
        ref = frames.copy()
        oracle.tcp4_batch(ref, 2, stride=2048, inplace=True)
        pin = xsum.PinnedBuffer(frames.size)
        pin.array[:] = frames
        end1 = 2048 + 14 + 152                       # frame 1's datagram end (ip.len 152)
        xsum.register_frames(ctx, pin.addr, end1 + 8)  # 8 bytes of slack only
        xsum.tcp_checksums(ctx, pin.addr)
        xsum.tx_flush(ctx)
        assert xsum.ctx_stats(ctx) == (1, 0)
        xsum.tcp_checksums(ctx, pin.addr + 2048)
        xsum.tx_flush(ctx)
        assert xsum.ctx_stats(ctx) == (1, 1)
        np.testing.assert_array_equal(pin.array, ref)
        pin.free()
    finally:
        xsum.ctx_destroy(ctx)


@pytest.mark.parametrize("zero_copy", [False, True])
def test_async_flush_pipeline(oracle, zero_copy):
    """tasx_flush_submit / _poll / _wait: tx_flush-sized batches (32 frames,
    data segments and ACK sizes) submitted back to back with up to 3 in flight
    per context (the 4th submit completes the 1st), completions in ticket
    order, each batch's frames finished only when its ticket completes; the
    staged path and the zero-copy one (frames in a registered pool)."""
    ctx = 5
    xsum.ctx_init(ctx, 0, 1 << 20)
    try:
        nb, n = 7, 32
        pay = np.where(np.arange(nb * n) % 3 == 0, 0, (np.arange(nb * n) * 53) % 1449)
        frames = pktgen.tcp4_frames(nb * n, payload=pay, stride=2048, seed=73)
        ref = frames.copy()
        oracle.tcp4_batch(ref, nb * n, stride=2048, inplace=True)
        if zero_copy:
            pin = xsum.PinnedBuffer(frames.size)
            pin.array[:] = frames
            xsum.register_frames(ctx, pin.addr, pin.nbytes)
            buf, addr = pin.array, pin.addr
        else:
            buf, addr = frames, frames.ctypes.data
        assert xsum.flush_submit(ctx) == 0 and xsum.flush_poll(ctx, 0)   # nothing submitted yet
        tickets = []
        for b in range(nb):
            for i in range(n):
                xsum.tcp_checksums(ctx, addr + (b * n + i) * 2048)
            tickets.append(xsum.flush_submit(ctx))
            assert xsum.pending(ctx) == 0
        assert tickets == list(range(1, nb + 1))
        with pytest.raises(xsum.TasxError):
            xsum.flush_poll(ctx, nb + 1)                               # not submitted
        # poll the last ticket until it completes; earlier ones are then done too
        while not xsum.flush_poll(ctx, tickets[-1]):
            pass
        assert all(xsum.flush_poll(ctx, t) for t in tickets)
        np.testing.assert_array_equal(buf, ref)
        assert xsum.flush_submit(ctx) == nb                            # empty: the last ticket
        xsum.flush_wait(ctx, nb)
        z, st = xsum.ctx_stats(ctx)
        assert (z, st) == ((nb, 0) if zero_copy else (0, nb))
        if zero_copy:
            pin.free()
    finally:
        xsum.ctx_destroy(ctx)


@pytest.mark.parametrize("pages", ["4k", "huge"])
def test_zero_copy_pageable_region(oracle, pages):
    """hipHostRegister of ordinary (numpy) memory as the frame region; `huge`:
    anonymous memory on a 2 MiB transparent huge page (MADV_HUGEPAGE), as a
    DPDK hugepage mempool's mbufs would be."""
    import ctypes
    import mmap
    xsum.ctx_init(4, 0, 1 << 20)
    mm = None
    try:
        n = 64
        if pages == "huge":
            huge = 2 << 20
            mm = mmap.mmap(-1, 2 * huge, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
            mm.madvise(mmap.MADV_HUGEPAGE, (-base) % huge, huge)
            raw = np.frombuffer(mm, dtype=np.uint8, count=huge, offset=(-base) % huge)
            raw[:] = 0
            start = 0
        else:
            raw = np.zeros(n * 2048 + 8192, np.uint8)
            start = (-raw.ctypes.data) % 4096
        region = raw[start:start + n * 2048]
        region[:] = pktgen.tcp4_frames(n, payload=1448, stride=2048, seed=63)
        ref = region.copy()
        oracle.tcp4_batch(ref, n, stride=2048, inplace=True)
        xsum.register_frames(4, region.ctypes.data, region.size)
        for i in range(n):
            xsum.fast_flows_kernelxsums(4, region.ctypes.data + i * 2048)
        xsum.tx_flush(4)
        np.testing.assert_array_equal(region, ref)
        assert xsum.ctx_stats(4)[0] == 1
    finally:
        xsum.ctx_destroy(4)  # unregisters the region
        raw = region = None
        if mm is not None:
            try:
                mm.close()
            except BufferError:  # a view still held (by a failure's traceback): the process frees it
                pass


def test_device_batch_on_pinned_host_memory(oracle):
    """The device batch entry point on pinned host memory (zero-copy over PCIe)."""
    n = 4096
    frames = pktgen.tcp4_frames(n, payload=1448, stride=2048, seed=64)
    pin = xsum.PinnedBuffer(frames.size)
    pin.array[:] = frames
    out = torch.empty(2 * n, dtype=torch.int16, device=DEV)
    xsum.tcp4_cksum_batch(pin.dev_addr, n, stride=2048, out=out, frame_len=1514)
    np.testing.assert_array_equal(u16(out), oracle.tcp4_batch(frames.copy(), n, stride=2048))
    pin.free()


def test_ctx_errors():
    with pytest.raises(xsum.TasxError):
        xsum.ctx_init(0, 99)
    xsum.ctx_init(2, 0, 1 << 20)
    try:
        with pytest.raises(xsum.TasxError):
            xsum.ctx_init(2, 0)
        f = np.zeros(64, np.uint8)
        with pytest.raises(xsum.TasxError):
            xsum.defer_tcp4(2, f.ctypes.data, 14, 20)  # l4_off < ip_off + 20
    finally:
        xsum.ctx_destroy(2)


# ---------------------------------------------------------------------------
# receive-side verification

def test_verify_roundtrip_64k(oracle):
    """TX kernel stores -> RX verification kernel: every frame verifies; random
    single-bit corruption is caught exactly as the oracle reports it."""
    n = 65536
    frames = pktgen.tcp4_frames(n, payload=(np.arange(n) * 7) % 1449, stride=2048, seed=81)
    d = to_dev(frames)
    xsum.tcp4_cksum_batch(d, n, stride=2048, inplace=True, want_out=False)
    flags = xsum.tcp4_verify_batch(d, n, stride=2048)
    torch.cuda.synchronize()
    assert bool((flags == 3).all())
    h = d.cpu().numpy()
    rng = pktgen.splitmix64(82, n)
    tl = 52 + (np.arange(n) * 7) % 1449
    pos = 14 + (rng % tl.astype(np.uint64)).astype(np.int64)
    bit = (rng >> np.uint64(61)).astype(np.int64)
    sel = np.arange(0, n, 3)
    h2 = h.copy()
    h2[sel * 2048 + pos[sel]] ^= (1 << bit[sel]).astype(np.uint8)
    got = xsum.tcp4_verify_batch(to_dev(h2), n, stride=2048).cpu().numpy()
    exp = oracle.tcp4_verify_batch_bounded(h2, n, 2048, stride=2048)  # RX bound: the stride slot
    np.testing.assert_array_equal(got, exp)
    assert np.all(got[sel] != 3) and np.all(np.delete(got, sel) == 3)


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_verify_edges(oracle, tcp4_golden, shift):
    g = tcp4_golden
    n, stride = len(g["offsets"]), int(g["stride"])
    good = g["frames"].copy()
    oracle.tcp4_batch(good, n, stride=stride, inplace=True)
    mixed = np.concatenate([good, g["frames"]])  # checksummed + raw (random fields) frames
    f = mixed.reshape(2 * n, stride)
    f[::5, 14] = 0x46                          # IHL 6
    f[1::7, 16:18] = 0                         # total_length 0
    buf = torch.zeros(mixed.size + 64, dtype=torch.uint8, device=DEV)
    buf[shift:shift + mixed.size] = to_dev(mixed)
    got = xsum.tcp4_verify_batch(buf[shift:], 2 * n, stride=stride).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.tcp4_verify_batch_bounded(mixed, 2 * n, stride, stride=stride))


@pytest.mark.parametrize("stride", [80, 128, 2048])
def test_tcp4_and_verify_short_frames_no_hint(oracle, stride):
    """Frames with total_length 0..90 (ACK and SYN sizes among them) without a
    hint: tcp4_tas14_kernel takes 38..1522 itself, the rest goes to the general
    body; TX checksums, then verification of the checksummed frames and of
    frames with random checksum fields."""
    tl = np.tile(np.arange(91), 9)
    n = len(tl)
    frames = pktgen.tcp4_frames(n, payload=0, stride=stride, seed=stride, ip_total_len=np.minimum(tl, stride - 14))
    f = frames.reshape(n, stride)
    f[:, 16] = (tl >> 8) & 0xFF
    f[:, 17] = tl & 0xFF       # total_length may exceed the room: the bytes past it are the next frame's
    big = np.concatenate([frames, np.zeros(128, np.uint8)])
    exp = oracle.tcp4_batch(big.copy(), n, stride=stride)
    d = to_dev(big)
    np.testing.assert_array_equal(u16(xsum.tcp4_cksum_batch(d, n, stride=stride)), exp)
    vexp = oracle.tcp4_verify_batch_bounded(big.copy(), n, stride, stride=stride)  # RX reads stay in the slot
    np.testing.assert_array_equal(xsum.tcp4_verify_batch(d, n, stride=stride).cpu().numpy(), vexp)
    xsum.tcp4_cksum_batch(d, n, stride=stride, inplace=True, want_out=False)
    good = d.cpu().numpy()
    np.testing.assert_array_equal(xsum.tcp4_verify_batch(d, n, stride=stride).cpu().numpy(),
                                  oracle.tcp4_verify_batch_bounded(good, n, stride, stride=stride))


@pytest.mark.parametrize("hinted", [False, True])
def test_tcp4_offsets_aligned_rooms_mix(oracle, hinted):
    """Frames by an offsets array over 16-byte aligned rooms in shuffled order
    (tcp4_tas14_kernel<OFFS>): data segments, ACKs and total_length 0..90, a few
    rooms shifted off alignment (general body), in place and to the output."""
    n = 6000
    rng = np.random.default_rng(11)
    pay = np.where(rng.random(n) < 0.5, 0, rng.integers(1, pktgen.TCP_MSS + 1, n)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=11)
    tl = 52 + pay
    tl[::13] = np.arange(len(tl[::13])) % 91
    f = frames.reshape(n, 2048)
    f[:, 16] = (tl >> 8) & 0xFF
    f[:, 17] = tl & 0xFF
    perm = rng.permutation(n)
    big = np.zeros((n + 1) * 2048, np.uint8)
    offs = perm.astype(np.int64) * 2048
    offs[::17] += (np.arange(len(offs[::17])) % 15) + 1       # misaligned frames
    for i in range(n):
        big[offs[i]:offs[i] + 2048] = f[i]
    exp = oracle.tcp4_batch(big.copy(), n, offsets=offs)
    d = to_dev(big)
    hint = to_dev(np.minimum(14 + tl, 2048).astype(np.int32)) if hinted else None
    np.testing.assert_array_equal(u16(xsum.tcp4_cksum_batch(d, n, offsets=to_dev(offs), frame_len=hint)), exp)
    xsum.tcp4_cksum_batch(d, n, offsets=to_dev(offs), frame_len=hint, inplace=True, want_out=False)
    got = d.cpu().numpy()
    ipc = np.array([int(got[o + 24]) | (int(got[o + 25]) << 8) for o in offs], np.uint16)
    tcpc = np.array([int(got[o + 50]) | (int(got[o + 51]) << 8) for o in offs], np.uint16)
    np.testing.assert_array_equal(ipc, exp[0::2])
    np.testing.assert_array_equal(tcpc, exp[1::2])


def test_tcp4_flush_mix_no_hint(oracle):
    """Data segments among pure ACKs, no hint (each row reads its own total_length)."""
    n = 8192
    rng = np.random.default_rng(5)
    pay = np.where(rng.random(n) < 0.5, 0, pktgen.TCP_MSS).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=5)
    exp = oracle.tcp4_batch(frames.copy(), n, stride=2048)
    np.testing.assert_array_equal(u16(xsum.tcp4_cksum_batch(to_dev(frames), n, stride=2048)), exp)


@pytest.mark.parametrize("variant", [0, 2])
def test_verify_uniform_hint(oracle, variant):
    """Received uniform-MTU batches with one frame-length hint (the headline
    kernel's verify mode): good frames, single-bit corruption anywhere in the
    datagram (checksum fields included), IHL 6, and total_length disagreeing
    with the hint (general body); then every datagram size it takes."""
    with kernel_variant(variant):
        n = 8192
        frames = pktgen.tcp4_frames(n, payload=1448, stride=2048, seed=91)
        d = to_dev(frames)
        xsum.tcp4_cksum_batch(d, n, stride=2048, inplace=True, want_out=False)
        h = d.cpu().numpy()
        rng = pktgen.splitmix64(92, n)
        pos = 14 + (rng % np.uint64(1500)).astype(np.int64)
        bit = (rng >> np.uint64(61)).astype(np.int64)
        sel = np.arange(0, n, 3)
        h[sel * 2048 + pos[sel]] ^= (1 << bit[sel]).astype(np.uint8)
        f = h.reshape(n, 2048)
        f[1::11, 14] = 0x46                         # IHL 6
        f[2::13, 16:18] = [0x05, 0x00]              # total_length 1280 (hint disagrees)
        f[4::17, 24:26] ^= 0xFF                     # ip.chksum flipped
        f[5::19, 50:52] = 0                         # tcp.chksum zeroed
        exp = oracle.tcp4_verify_batch_bounded(h, n, 1514, stride=2048)  # the received length bounds reads
        got = xsum.tcp4_verify_batch(to_dev(h), n, stride=2048, frame_len=1514).cpu().numpy()
        np.testing.assert_array_equal(got, exp)
        for tl in list(range(40, 1540, 11)) + [64, 1500, 1522, 1523]:
            m = 32
            fr = pktgen.tcp4_frames(m, payload=0, stride=1600, seed=tl, ip_total_len=tl)
            oracle.tcp4_batch(fr, m, stride=1600, inplace=True)
            fr.reshape(m, 1600)[::4, 40] ^= 0x10        # corrupt a quarter (a tcp header byte)
            exp = oracle.tcp4_verify_batch_bounded(fr, m, 14 + tl, stride=1600)
            got = xsum.tcp4_verify_batch(to_dev(fr), m, stride=1600, frame_len=14 + tl).cpu().numpy()
            np.testing.assert_array_equal(got, exp, err_msg=f"ip.len {tl}")


# ---------------------------------------------------------------------------
# rooms: rows that load ahead of their total_length (tasx_tcp4_cksum_batch_dev_room)

@pytest.mark.parametrize("room", [80, 1536, 2048])
@pytest.mark.parametrize("variant", [0, 2, 3])
def test_tcp4_rooms_every_row_mode(oracle, room, variant):
    """Stride-mode TAS frames in 2048 B rooms with a room contract: the
    automatic selection (each row mode the room and the hints select: whole
    room, total_length first, per-frame hints, the uniform hint) and the
    general kernels, over data segments, ACKs, total_length 0..90 and
    1523..2034 (rows the fast path hands to the general body), with no hint,
    per-frame hints (exact, short, long) and a uniform hint; out of place and
    in place."""
    n = 5000
    rng = np.random.default_rng(room + variant)
    pay = np.where(rng.random(n) < 0.4, 0, rng.integers(1, pktgen.TCP_MSS + 1, n)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=room)
    tl = 52 + pay
    tl[::11] = np.arange(len(tl[::11])) % 91
    tl[5::97] = 1523 + np.arange(len(tl[5::97])) % 500
    f = frames.reshape(n, 2048)
    f[:, 16] = (tl >> 8) & 0xFF
    f[:, 17] = tl & 0xFF
    exp = oracle.tcp4_batch(frames.copy(), n, stride=2048)
    exact = (14 + tl).astype(np.int32)
    noise = (14 + tl + rng.integers(-30, 30, n)).clip(0, 2048).astype(np.int32)
    with kernel_variant(variant):
        for hint in (None, to_dev(exact), to_dev(noise), 1514):
            d = to_dev(frames)
            got = u16(xsum.tcp4_cksum_batch(d, n, stride=2048, frame_len=hint, room=room))
            tag = f"room {room} variant {variant} hint {'array' if isinstance(hint, torch.Tensor) else hint}"
            np.testing.assert_array_equal(got, exp, err_msg=tag)
            xsum.tcp4_cksum_batch(d, n, stride=2048, frame_len=hint, room=room, inplace=True, want_out=False)
            h = d.cpu().numpy().reshape(n, 2048)
            np.testing.assert_array_equal(h[:, 24:26].copy().view(np.uint16).ravel(), exp[0::2], err_msg=tag)
            np.testing.assert_array_equal(h[:, 50:52].copy().view(np.uint16).ravel(), exp[1::2], err_msg=tag)


def test_tcp4_room_selects_row_mode():
    """Which tcp4_tas14_kernel mode a call takes (tasx_last_kernel): a full-MTU
    room and no per-frame hints -> whole-room rows; per-frame hints -> each
    row's hint as its geometry; neither -> total_length first; a uniform hint -> the hinted kernel; an offsets
    array -> the OFFS forms."""
    n = 64
    frames = to_dev(pktgen.tcp4_frames(n, stride=2048))
    flen = to_dev(np.full(n, 1514, np.int32))
    offs = to_dev(np.arange(n, dtype=np.int64) * 2048)
    cases = [
        (dict(stride=2048), "tcp4_tas14_kernel<tl_first>"),
        (dict(stride=2048, room=2048), "tcp4_tas14_kernel<room>"),
        (dict(stride=2048, room=1536), "tcp4_tas14_kernel<room>"),
        (dict(stride=2048, room=1535), "tcp4_tas14_kernel<tl_first>"),
        (dict(stride=2048, room=79), "tcp4_tas14_kernel<tl_first>"),
        (dict(stride=2048, room=2048, frame_len=flen), "tcp4_tas14_kernel<hints>"),
        (dict(stride=2048, frame_len=flen), "tcp4_tas14_kernel<hints>"),
        (dict(stride=2048, room=2048, frame_len=1514), "tcp4_tas14_kernel<hint>"),
        (dict(offsets=offs, room=2048), "tcp4_tas14_kernel<room,offs>"),
        (dict(offsets=offs, room=2048, frame_len=flen), "tcp4_tas14_kernel<hints,offs>"),
        (dict(offsets=offs), "tcp4_tas14_kernel<tl_first,offs>"),
        (dict(stride=2048, ip_off=14, l4_off=38), "tcp4_frame_kernel"),
    ]
    for kw, name in cases:
        xsum.tcp4_cksum_batch(frames, n, **kw)
        assert xsum.last_kernel() == name, (kw, xsum.last_kernel())
    torch.cuda.synchronize()


@pytest.mark.parametrize("ip_off", [14, 30])
@pytest.mark.parametrize("absolute", [False, True])
@pytest.mark.parametrize("room", [0, 80, 2048])
def test_tcp4_offsets_rooms_ipoff_absolute(oracle, ip_off, absolute, room):
    """Frames by an offsets array (tcp4_tas14_kernel<OFFS>) with the IPv4 header
    at 14 and at 30 (an (ip_off & ~15) term in the frame start), offsets from a
    base or absolute device addresses (base NULL), some frames misaligned, with
    and without a room, per-frame hints."""
    n = 3000
    rng = np.random.default_rng(ip_off * 7 + room + int(absolute))
    pay = np.where(rng.random(n) < 0.5, 0, rng.integers(1, 1400, n)).astype(np.int64)
    raw = pktgen.tcp4_frames(n, payload=pay, stride=2048, seed=ip_off).reshape(n, 2048)
    frames = np.zeros((n, 2048 + 16), np.uint8)
    frames[:, ip_off - 14:ip_off - 14 + 2048] = raw     # shift: IPv4 header at ip_off
    perm = rng.permutation(n)
    big = np.zeros((n + 2) * 2080, np.uint8)
    offs = perm.astype(np.int64) * 2080
    offs[::19] += (np.arange(len(offs[::19])) % 15) + 1       # misaligned frames
    for i in range(n):
        big[offs[i]:offs[i] + 2064] = frames[i]
    exp = oracle.tcp4_batch(big.copy(), n, offsets=offs, ip_off=ip_off, l4_off=ip_off + 20)
    d = to_dev(big)
    hint = to_dev((ip_off + 52 + pay).astype(np.int32))
    if absolute:
        base, o = None, to_dev(offs + d.data_ptr())
    else:
        base, o = d, to_dev(offs)
    out = torch.empty(2 * n, dtype=torch.int16, device=DEV)
    rc = xsum.lib().tasx_tcp4_cksum_batch_dev_room(None if base is None else base.data_ptr(), o.data_ptr(), 0,
                                                   hint.data_ptr(), 0, room, n, ip_off, ip_off + 20,
                                                   out.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, xsum.last_error()
    assert xsum.last_kernel().startswith("tcp4_tas14_kernel")
    np.testing.assert_array_equal(u16(out), exp)
    rc = xsum.lib().tasx_tcp4_cksum_batch_dev_room(None if base is None else base.data_ptr(), o.data_ptr(), 0,
                                                   hint.data_ptr(), 0, room, n, ip_off, ip_off + 20,
                                                   None, xsum.TASX_F_INPLACE, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    got = d.cpu().numpy()
    ipc = np.array([int(got[x + ip_off + 10]) | (int(got[x + ip_off + 11]) << 8) for x in offs], np.uint16)
    tcpc = np.array([int(got[x + ip_off + 36]) | (int(got[x + ip_off + 37]) << 8) for x in offs], np.uint16)
    np.testing.assert_array_equal(ipc, exp[0::2])
    np.testing.assert_array_equal(tcpc, exp[1::2])


def test_tcp4_room_tso_rows(oracle):
    """Whole-room rows over TSO-sized frames (ip.len 1523..65535 in 65,552 B
    rooms): every row goes to the general body, results still exact."""
    n, stride = 256, 65552
    tl = np.where(np.arange(n) % 2 == 0, 65535, 1523 + np.arange(n) * 17)
    frames = pktgen.tcp4_frames(n, payload=0, stride=stride, seed=59, ip_total_len=tl)
    exp = oracle.tcp4_batch(frames.copy(), n, stride=stride)
    got = u16(xsum.tcp4_cksum_batch(to_dev(frames), n, stride=stride, room=stride))
    assert xsum.last_kernel() == "tcp4_tas14_kernel<room>"
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("variant", [0])
@pytest.mark.parametrize("offs", [False, True])
@pytest.mark.parametrize("bound", ["len", "room", "none"])
def test_verify_mix_received_lengths(oracle, variant, offs, bound):
    """An RX burst of data segments and pure ACKs: honest frames,
    Ethernet-padded short frames (received length > 14 + total_length),
    truncated frames, corrupted bytes and checksum fields; stride mode and an
    offsets array; bounded by each frame's received length (its hint: row mode
    <hints,verify>), by a 2048 B room or by nothing but the stride slot / the
    frame's own total_length (both <tl_first,verify>).  Bit-exact against the
    bounded oracle."""
    n, stride = 8192, 2048
    rng = np.random.default_rng(17 + variant + 2 * offs)
    pay = np.where(rng.random(n) < 0.5, 0, rng.integers(1, pktgen.TCP_MSS + 1, n)).astype(np.int64)
    frames = pktgen.tcp4_frames(n, payload=pay, stride=stride, seed=170)
    oracle.tcp4_batch(frames, n, stride=stride, inplace=True)
    f = frames.reshape(n, stride)
    rcv = 14 + 52 + pay
    pad = np.arange(n) % 7 == 1
    rcv[pad] = np.maximum(rcv[pad], 60) + 4 + (np.arange(n)[pad] % 9)   # padding / trailer bytes
    trunc = np.arange(n) % 11 == 2
    rcv[trunc] = np.maximum(rcv[trunc] - 1 - np.arange(n)[trunc] % 40, 20)
    bad = np.arange(n) % 5 == 3
    pos = 14 + (rng.integers(0, 10 ** 6, n) % (rcv - 14))
    f[np.nonzero(bad)[0], pos[bad]] ^= 0x20
    f[4::13, 24] ^= 0x01                                                   # ip.chksum
    f[6::17, 50] ^= 0x80                                                   # tcp.chksum
    kw = dict(offsets=to_dev(np.arange(n, dtype=np.int64) * stride)) if offs else dict(stride=stride)
    if bound == "len":
        kw["frame_len"] = to_dev(rcv.astype(np.int32))
        b, mode = rcv.astype(np.uint32), "hints"
    elif bound == "room":
        kw["room"] = stride
        b, mode = stride, "tl_first"
    else:
        b, mode = (0 if offs else stride), "tl_first"
    exp = oracle.tcp4_verify_batch_bounded(frames, n, b, stride=stride)
    with kernel_variant(variant):
        got = xsum.tcp4_verify_batch(to_dev(frames), n, **kw)
        name = f"tcp4_tas14_kernel<{mode},verify{',offs' if offs else ''}>"
        assert xsum.last_kernel() == name
        np.testing.assert_array_equal(got.cpu().numpy(), exp)


# ---------------------------------------------------------------------------
# RX: received frames are untrusted (forged total_length)

@pytest.mark.parametrize("form", ["flen", "flen0", "stride", "room_offs"])
def test_verify_forged_total_length_bounded(oracle, form):
    """Short received frames whose total_length claims far more than arrived
    (up to 65535), packed at the END of their allocation: reads stay inside
    each frame's bound (received length, uniform length, stride slot, room) and
    L4 fails for them; honest frames still verify.  Bit-exact against the
    bounded oracle."""
    n, stride = 4096, 128
    rng = np.random.default_rng(len(form))
    frames = pktgen.tcp4_frames(n, payload=rng.integers(0, 60, n), stride=stride, seed=71)
    oracle.tcp4_batch(frames, n, stride=stride, inplace=True)
    f = frames.reshape(n, stride)
    rcv = (66 + (f[:, 17].astype(np.int64) - 52)).clip(66, stride)       # what arrived: the frame's bytes
    forged = np.arange(n) % 3 == 0
    forged[-1] = True                                                   # the batch's last frame too
    fake = np.where(np.arange(n) % 2 == 0, 65535, 1500 + np.arange(n) % 500)
    f[forged, 16] = (fake[forged] >> 8) & 0xFF
    f[forged, 17] = fake[forged] & 0xFF
    host = frames.copy()
    # the frames end exactly where the allocation ends
    d = torch.empty(host.size, dtype=torch.uint8, device=DEV)
    d.copy_(torch.from_numpy(host))
    if form == "flen":
        got = xsum.tcp4_verify_batch(d, n, stride=stride, frame_len=to_dev((14 + 52 + rcv - 66).astype(np.int32)))
        bound = (14 + 52 + rcv - 66).astype(np.uint32)
    elif form == "flen0":
        got = xsum.tcp4_verify_batch(d, n, stride=stride, frame_len=100)
        bound = 100
    elif form == "stride":
        got = xsum.tcp4_verify_batch(d, n, stride=stride)
        bound = stride
    else:
        offs = np.arange(n, dtype=np.int64) * stride
        got = xsum.tcp4_verify_batch(d, n, offsets=to_dev(offs), room=stride)
        bound = stride
    got = got.cpu().numpy()
    exp = oracle.tcp4_verify_batch_bounded(host, n, bound, stride=stride)
    np.testing.assert_array_equal(got, exp)
    assert np.all(got[forged] & xsum.RX_L4_OK == 0)
    honest = ~forged & (rcv >= 66)
    assert np.all(got[honest] == 3) or form == "flen0"
