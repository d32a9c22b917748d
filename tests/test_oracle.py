"""CPU oracle checks: known-answer vectors, golden fixtures, and the two
independent restatements (oracle/tasx_oracle.c vs oracle/xsum_ref.py) against
each other.  Parity anchors: RFC 1071 section 3 and the reference unit-test
frame (tests/golden/kat.json); the reference's own tests pin no checksum value
(tests/tas_unit/fastpath.c:206,258)."""
import json

import numpy as np
import pytest

from oracle import xsum_ref as R
from tas_amd import pktgen

from conftest import GOLDEN


def test_rfc1071_section3(oracle):
    kat = json.loads((GOLDEN / "kat.json").read_text())["rfc1071_sec3"]
    b = bytes.fromhex(kat["bytes"])
    assert oracle.raw_cksum(b) == kat["raw_cksum_native_le"] == 0xF2DD
    assert R.raw_cksum(b) == 0xF2DD
    # network-order bytes of the folded sum are dd f2, as RFC 1071 prints it
    assert oracle.raw_cksum(b).to_bytes(2, "little").hex() == kat["raw_cksum_be"]


def test_ipv4_header_public_kat(oracle):
    """rte_ipv4_cksum on the widely published IPv4 header example: b8 61."""
    kat = json.loads((GOLDEN / "kat.json").read_text())["ipv4_header_public"]
    h = bytes.fromhex(kat["header_hex"])
    assert oracle.ipv4_cksum(h).to_bytes(2, "little").hex() == kat["ip_chksum_bytes"] == "b861"
    assert R.ipv4_cksum(h) == oracle.ipv4_cksum(h)


def test_unit_test_frame_kat(oracle):
    kat = json.loads((GOLDEN / "kat.json").read_text())["tas_unit_window_update"]
    f = bytearray(bytes.fromhex(kat["frame_hex"]))
    assert f == pktgen.kat_frame()
    ipc, tcpc = oracle.tcp_checksums(f)
    assert f[24:26].hex() == kat["ip_chksum_bytes"] == "a3bb"
    assert f[50:52].hex() == kat["tcp_chksum_bytes"] == "cfd7"
    assert (ipc, tcpc) == (pktgen.KAT_IP_CHKSUM, pktgen.KAT_TCP_CHKSUM)
    g = pktgen.kat_frame()
    assert R.tcp_checksums(g) == (ipc, tcpc)
    assert g == f


def test_kat_receiver_verification(oracle):
    """A receiver summing the finished header / segment gets 0xffff (RFC 1071)."""
    f = pktgen.kat_frame()
    oracle.tcp_checksums(f)
    assert oracle.raw_cksum(bytes(f[14:34])) == 0xFFFF
    tl = int.from_bytes(f[16:18], "big")
    total = R.word_sum(bytes(f[34:14 + tl])) + oracle.ipv4_phdr_cksum(bytes(f[14:34]))
    assert R._fold_exact(total) == 0xFFFF


@pytest.mark.parametrize("buf,expect", [
    (b"", 0), (b"\0", 0), (bytes(64), 0), (b"\xff" * 64, 0xFFFF), (b"\xff", 0xFF),
    (b"\x01\x00\xfe\xff", 0xFFFF), (b"\x12", 0x12), (b"\x12\x34", 0x3412),
])
def test_raw_edges(oracle, buf, expect):
    assert oracle.raw_cksum(buf) == expect
    assert R.raw_cksum(buf) == expect


def test_raw_reduce_and_acc(oracle):
    assert oracle.L.oracle_raw_cksum_reduce(0) == 0
    assert oracle.L.oracle_raw_cksum_reduce(0xFFFF) == 0xFFFF
    assert oracle.L.oracle_raw_cksum_reduce(0x10000) == 1
    assert oracle.L.oracle_raw_cksum_reduce(0xFFFFFFFF) == 0xFFFF
    b = bytes(range(256)) * 3
    arr = np.frombuffer(b, np.uint8)
    assert oracle.L.oracle_raw_cksum_acc(arr.ctypes.data, len(b), 5) == R.word_sum(b) + 5


def test_ipv4_cksum_special(oracle):
    # all-zero header: raw 0 -> ~0 = 0xffff
    assert oracle.ipv4_cksum(bytes(20)) == 0xFFFF == R.ipv4_cksum(bytes(20))
    # raw sum folding to 0xffff is returned as 0xffff, not inverted
    h = bytearray(20)
    h[0:2] = b"\xff\xff"
    assert oracle.ipv4_cksum(bytes(h)) == 0xFFFF == R.ipv4_cksum(bytes(h))
    h[0:2] = b"\x01\x00"
    assert oracle.ipv4_cksum(bytes(h)) == 0xFFFE


def test_udptcp_short_total_length(oracle):
    ip = bytearray(20)
    for tl in (0, 1, 19):
        ip[2:4] = tl.to_bytes(2, "big")
        assert oracle.ipv4_udptcp_cksum(bytes(ip), bytes(64)) == 0 == R.ipv4_udptcp_cksum(bytes(ip), bytes(64))
    ip[2:4] = (20).to_bytes(2, "big")
    ip[9] = 6
    # empty segment: ~(phdr) with phdr = proto<<8
    assert oracle.ipv4_udptcp_cksum(bytes(ip), b"") == (~0x0600) & 0xFFFF


def test_udptcp_zero_result_becomes_ffff(oracle):
    ip = bytearray(20)
    ip[2:4] = (22).to_bytes(2, "big")
    ip[9] = 6
    phdr = oracle.ipv4_phdr_cksum(bytes(ip))
    w = (0xFFFF - phdr) % 0xFFFF
    l4 = w.to_bytes(2, "little")
    assert oracle.ipv4_udptcp_cksum(bytes(ip), l4) == 0xFFFF == R.ipv4_udptcp_cksum(bytes(ip), l4)


def test_phdr_tso_flag_and_offload_xsum(oracle):
    f = pktgen.tcp4_frames(4, payload=1448, stride=2048).reshape(4, 2048)
    for i in range(4):
        ip = bytes(f[i, 14:34])
        tl = int.from_bytes(ip[2:4], "big")
        src = int.from_bytes(ip[12:16], "little")
        dst = int.from_bytes(ip[16:20], "little")
        # network_ip_phdr_xsum (offload branch) equals rte_ipv4_phdr_cksum
        assert oracle.ip_phdr_xsum(src, dst, 6, tl - 20) == oracle.ipv4_phdr_cksum(ip)
        assert R.ip_phdr_xsum(src, dst, 6, tl - 20) == oracle.ipv4_phdr_cksum(ip)
        assert oracle.ipv4_phdr_cksum(ip, R.PKT_TX_TCP_SEG) == R.ipv4_phdr_cksum(ip, R.PKT_TX_TCP_SEG)
        assert oracle.ipv4_phdr_cksum(ip) == R.ipv4_phdr_cksum(ip)


def test_raw_golden(oracle, raw_golden):
    g = raw_golden
    got = oracle.raw_batch(g["buf"], len(g["lengths"]), offsets=g["offsets"], lengths=g["lengths"])
    np.testing.assert_array_equal(got, g["expected"])


def test_tcp4_golden(oracle, tcp4_golden):
    g = tcp4_golden
    n = len(g["offsets"])
    frames = g["frames"].copy()
    got = oracle.tcp4_batch(frames, n, stride=int(g["stride"]))
    np.testing.assert_array_equal(got, g["expected"])
    np.testing.assert_array_equal(frames, g["frames"])  # not in place: restored
    # odd frame starts give the same results (sums are relative to each header)
    odd = np.zeros(frames.size + 32, np.uint8)
    odd[1:1 + frames.size] = frames
    got = oracle.tcp4_batch(odd[1:], n, stride=int(g["stride"]))
    np.testing.assert_array_equal(got, g["expected"])


def test_tcp4_inplace_matches_reference_stores(oracle):
    buf = pktgen.tcp4_frames(64, payload=np.arange(64) * 22, stride=2048)
    ref = buf.copy()
    out = oracle.tcp4_batch(buf, 64, stride=2048, inplace=True)
    f = buf.reshape(64, 2048)
    np.testing.assert_array_equal(f[:, 24:26].copy().view("<u2")[:, 0], out[0::2])
    np.testing.assert_array_equal(f[:, 50:52].copy().view("<u2")[:, 0], out[1::2])
    for i in range(64):
        fr = bytearray(ref[i * 2048:(i + 1) * 2048].tobytes())
        assert R.tcp_checksums(fr) == (out[2 * i], out[2 * i + 1])


def test_random_cross_restatement(oracle):
    buf, offs, lens = pktgen.raw_mixed(400, seed=99, sizes=(0, 1, 2, 3, 17, 64, 577, 1500, 9001), odd=True)
    got = oracle.raw_batch(buf, len(lens), offsets=offs, lengths=lens)
    np.testing.assert_array_equal(got, R.raw_batch(buf, offs, lens))


def test_oracle_bench_runs(oracle):
    buf, stride = pktgen.raw_uniform(512, 1500)
    t = oracle.bench(0, buf, 512, stride=stride, len0=1500, threads=2, reps=3)
    assert 0 < t < 5
    fr = pktgen.tcp4_frames(256)
    t = oracle.bench(1, fr, 256, stride=2048, threads=1, reps=3)
    assert 0 < t < 5


# ---------------------------------------------------------------------------
# receive-side verification

def test_verify_kat_and_corruption(oracle):
    f = pktgen.kat_frame()
    oracle.tcp_checksums(f)
    arr = np.frombuffer(bytes(f), np.uint8).copy()
    assert oracle.tcp4_verify_batch(arr, 1, stride=len(f))[0] == 3
    assert R.tcp4_verify(bytes(f)) == 3
    for pos, expect in ((14 + 8, 2), (34 + 5, 1), (14 + 13, 0)):  # ttl; seq; src addr (in both)
        g = arr.copy()
        g[pos] ^= 0x10
        assert oracle.tcp4_verify_batch(g, 1, stride=len(f))[0] == expect, pos
        assert R.tcp4_verify(bytes(g)) == expect
    g = arr.copy()
    g[14] = 0x46  # IHL 6
    assert oracle.tcp4_verify_batch(g, 1, stride=len(f))[0] & 4


def test_verify_batch_cross_restatement(oracle):
    n = 300
    frames = pktgen.tcp4_frames(n, payload=(np.arange(n) * 5) % 1449, stride=2048, seed=71)
    good = frames.copy()
    oracle.tcp4_batch(good, n, stride=2048, inplace=True)
    flags = oracle.tcp4_verify_batch(good, n, stride=2048)
    assert np.all(flags == 3)
    bad = good.copy()
    rng = pktgen.splitmix64(72, n)
    for i in range(n):
        tl = 52 + (i * 5) % 1449
        pos = 14 + int(rng[i] % np.uint64(tl))
        bad[i * 2048 + pos] ^= 1 << int(rng[i] >> np.uint64(61))
    fl = oracle.tcp4_verify_batch(bad, n, stride=2048)
    assert np.all(fl != 3)  # a single flipped bit is always detected
    for i in range(0, n, 7):
        assert fl[i] == R.tcp4_verify(bytes(bad[i * 2048:(i + 1) * 2048]))
