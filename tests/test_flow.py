"""RX flow lookup: fast_flows_packet_fss()
(/root/reference/tas/fast/fast_flows.c:1084-1163) and its CRC32C flow_hash
(:1078-1082).

CPU tests pin the CRC32C of both restatements (oracle C table-driven, numpy
module bitwise) against RFC 3720 B.4 and the catalogue check value, and the C
lookup against the committed fixture and the Python lookup.  GPU tests run
tasx_flow_lookup_batch_dev through the C ABI against the C oracle, bit-exact
(hash and flow id of every frame).
"""
import json

import numpy as np
import pytest

from tas_amd import pktgen


@pytest.fixture(scope="module")
def flow_golden():
    from conftest import GOLDEN as G
    with np.load(G / "flow_vectors.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def kat():
    from conftest import GOLDEN as G
    return json.loads((G / "kat.json").read_text())


def _std_crc(o, b: bytes) -> int:
    c = 0xFFFFFFFF
    for i in range(0, len(b), 8):
        c = o.L.oracle_crc32c_u64(int.from_bytes(b[i:i + 8], "little"), c)
    return c ^ 0xFFFFFFFF


def test_crc32c_rfc3720(oracle, kat):
    from oracle import xsum_ref as R
    k = kat["crc32c_rfc3720_b4"]
    cases = {"zeros32": bytes(32), "ones32": b"\xff" * 32, "inc32": bytes(range(32)),
             "dec32": bytes(range(31, -1, -1))}
    for name, data in cases.items():
        exp = int(k[name], 16)
        assert _std_crc(oracle, data) == exp, name
        assert R.crc32c(data, 0xFFFFFFFF) ^ 0xFFFFFFFF == exp, name
    assert R.crc32c(b"123456789", 0xFFFFFFFF) ^ 0xFFFFFFFF == int(k["check_123456789"], 16)


def test_crc32c_word_forms(oracle):
    """crc32c_sse42_u64 then _u32 (fast path) == one pass over the 12 bytes
    (rte_hash_crc in the slow path, tas/slow/nicif.c:588-600)."""
    from oracle import xsum_ref as R
    rng = np.random.default_rng(3)
    for _ in range(50):
        b = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        h = oracle.L.oracle_crc32c_u32(int.from_bytes(b[8:], "little"),
                                       oracle.L.oracle_crc32c_u64(int.from_bytes(b[:8], "little"), 0))
        assert h == R.crc32c(b, 0)


def test_oracle_flow_golden(oracle, flow_golden):
    g = flow_golden
    n = len(g["expected_fid"])
    h, fid = oracle.flow_lookup_batch(g["frames"], n, g["flowht"], g["flowst"], fs_num=int(g["fs_num"]),
                                      stride=int(g["stride"]))
    np.testing.assert_array_equal(h, g["expected_hash"])
    np.testing.assert_array_equal(fid, g["expected_fid"])
    assert (fid != 0xFFFFFFFF).sum() >= 30 and (fid == 0xFFFFFFFF).sum() >= 10


def test_oracle_flow_vs_python(oracle):
    from oracle import xsum_ref as R
    nflows, ent = 300, 509
    keys = pktgen.flow_keys(nflows, seed=11)
    fs = pktgen.flow_state(keys, seed=11)
    hashes = np.asarray([R.crc32c(bytes(k), 0) for k in keys], np.uint64)
    ht, ok = pktgen.flow_table(hashes, ent)
    fr = pktgen.rx_frames(keys, stride=96, seed=11)
    h, fid = oracle.flow_lookup_batch(fr, nflows, ht, fs, fs_num=nflows, stride=96)
    for i in range(nflows):
        eh, ef = R.flow_lookup(fr[i * 96:(i + 1) * 96].tobytes(), ht, fs.tobytes(), nflows)
        assert (h[i], fid[i]) == (eh, ef)
    np.testing.assert_array_equal(fid[ok], np.arange(nflows)[ok])
    assert (fid[~ok] == 0xFFFFFFFF).all()


# ---------------------------------------------------------------------------
# GPU parity

def _gpu(frames, n, flowht, flowst, fs_num, stride=0, offsets=None, want_hash=True, **kw):
    import torch
    from tas_amd import xsum
    dev = "cuda:0"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    off = None if offsets is None else t(np.asarray(offsets, np.int64))
    h, fid = xsum.flow_lookup_batch(t(frames), n, t(flowht), t(flowst), fs_num, offsets=off, stride=stride,
                                    want_hash=want_hash, **kw)
    torch.cuda.synchronize()
    return (None if h is None else h.cpu().numpy().view(np.uint32)), fid.cpu().numpy().view(np.uint32)


@pytest.mark.gpu
def test_gpu_flow_golden(flow_golden):
    """The lookup on the fixture (round 6 retired the comparison variants:
    CRC forms, frames per lane, key cache policies, the partitioned lookup)."""
    from tas_amd import xsum
    g = flow_golden
    n = len(g["expected_fid"])
    h, fid = _gpu(g["frames"], n, g["flowht"], g["flowst"], int(g["fs_num"]), stride=int(g["stride"]))
    assert xsum.last_kernel() == "flow_lookup_kernel"
    np.testing.assert_array_equal(h, g["expected_hash"])
    np.testing.assert_array_equal(fid, g["expected_fid"])


@pytest.mark.gpu
def test_gpu_flow_vs_oracle_large(oracle):
    """64K flows in a TAS-sized table (2x entries), 256K frames: hits in random
    order, misses (unknown keys), hash-out off, with a ragged batch end."""
    nflows, ent, n = 65536, 131072, 262144
    keys = pktgen.flow_keys(nflows, seed=5)
    fs = pktgen.flow_state(keys, seed=5)
    fr_all = pktgen.rx_frames(keys, stride=128, seed=5)
    hashes, _ = oracle.flow_lookup_batch(fr_all, nflows, np.zeros(2, np.uint32), fs, fs_num=nflows, stride=128)
    ht, ok = pktgen.flow_table(hashes, ent)
    assert ok.mean() > 0.95
    rng = np.random.default_rng(9)
    pick = rng.integers(0, nflows, n)
    fkeys = keys[pick].copy()
    miss = rng.random(n) < 0.1
    fkeys[miss, 4] ^= 0x5A  # unknown remote ip
    fr = pktgen.rx_frames(fkeys, stride=128, seed=6)
    eh, ef = oracle.flow_lookup_batch(fr, n, ht, fs, fs_num=nflows, stride=128)
    h, fid = _gpu(fr, n, ht, fs, nflows, stride=128)
    np.testing.assert_array_equal(h, eh)
    np.testing.assert_array_equal(fid, ef)
    assert (fid[miss] == 0xFFFFFFFF).all()
    _, fid2 = _gpu(fr, n, ht, fs, nflows, stride=128, want_hash=False)
    np.testing.assert_array_equal(fid2, ef)
    m = n - 777                                          # ragged end
    h3, fid3 = _gpu(fr, m, ht, fs, nflows, stride=128)
    np.testing.assert_array_equal(fid3, ef[:m])
    np.testing.assert_array_equal(h3, eh[:m])


@pytest.mark.gpu
def test_gpu_flow_offsets_layouts(oracle, flow_golden):
    """Frames at odd offsets (offsets array), and a different header layout."""
    g = flow_golden
    n, stride = len(g["expected_fid"]), int(g["stride"])
    frames = g["frames"].reshape(n, stride)
    buf = np.zeros(n * (stride + 3) + 16, np.uint8)
    offs = np.arange(n, dtype=np.int64) * (stride + 3) + 1
    for i in range(n):
        buf[offs[i]:offs[i] + stride] = frames[i]
    h, fid = _gpu(buf, n, g["flowht"], g["flowst"], int(g["fs_num"]), offsets=offs)
    np.testing.assert_array_equal(h, g["expected_hash"])
    np.testing.assert_array_equal(fid, g["expected_fid"])
    # ip at 0, tcp at 24 (an options gap): same keys moved
    lay = np.zeros((n, 64), np.uint8)
    lay[:, 0:20] = frames[:, 14:34]
    lay[:, 24:44] = frames[:, 34:54]
    h2, fid2 = _gpu(lay.reshape(-1), n, g["flowht"], g["flowst"], int(g["fs_num"]), stride=64, ip_off=0, l4_off=24)
    np.testing.assert_array_equal(h2, g["expected_hash"])
    np.testing.assert_array_equal(fid2, g["expected_fid"])


@pytest.mark.gpu
def test_gpu_flow_errors():
    import torch
    from tas_amd import xsum
    z = torch.zeros(4096, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(xsum.TasxError):
        xsum.flow_lookup_batch(z, 1, z[:16], z, 0, stride=64)            # fs_num 0
    with pytest.raises(xsum.TasxError):
        xsum.flow_lookup_batch(z, 1, z[4:20], z, 1, stride=64)           # misaligned flowht
    with pytest.raises(xsum.TasxError):
        xsum.flow_lookup_batch(z, 1, z[:16], z, 1, stride=64, fs_stride=130)
