"""The C boundary in TAS's own terms:

* tests/c/gen_ref_frames.c builds TX frames with the reference's own wire types
  and header macros (/root/reference/include/packet_defs.h, utils.h) exactly
  as flow_tx_segment / flow_tx_ack fill them (tas/fast/fast_flows.c:886-1008),
  with static asserts on the layout the kernels assume (54-byte pkt_tcp, ip at
  14, tcp at 34); its output is the committed fixture tests/golden/ref_frames.bin
  (the unit-test frame of tests/tas_unit/fastpath.c:187-207 + a 32-frame
  tx_flush batch) with the oracle's expected checksums.
* tests/c/bin/boundary_test (tests/c/boundary_test.c, linking libtasx only)
  runs INTEGRATION.md's glue (tests/c/tas_glue.h: tcp_checksums /
  fast_flows_kernelxsums with beui32_t arguments, the thread-bound context)
  over fake mbufs and checks every frame after the tx_flush step, staged and
  zero-copy, on the GPU.
"""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

REF_INC = Path("/root/reference/include")
FIXTURE = GOLDEN / "ref_frames.bin"
BIN = ROOT / "tests" / "c" / "bin" / "boundary_test"


def load_fixture():
    b = FIXTURE.read_bytes()
    assert b[:8] == b"TASXRF01"
    n, room = struct.unpack_from("<II", b, 8)
    recs = [struct.unpack_from("<IHHI", b, 16 + 12 * i) for i in range(n)]
    frames = np.frombuffer(b, np.uint8, n * room, 16 + 12 * n).reshape(n, room)
    return n, room, recs, frames


@pytest.mark.skipif(not (REF_INC / "packet_defs.h").exists(), reason="needs /root/reference (build container)")
def test_generator_builds_with_reference_headers_and_reproduces_fixture(tmp_path):
    """The generator compiles against the reference's headers (its static
    asserts pin struct pkt_tcp's layout) and regenerates the committed fixture
    byte for byte."""
    exe = tmp_path / "gen"
    subprocess.run(["gcc", "-std=gnu99", "-O2", "-Wall", "-I", str(REF_INC), "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "c" / "gen_ref_frames.c"), str(ROOT / "oracle" / "tasx_oracle.c"),
                    "-lpthread", "-o", str(exe)], check=True)
    out = tmp_path / "ref_frames.bin"
    subprocess.run([str(exe), str(out)], check=True, capture_output=True)
    assert out.read_bytes() == FIXTURE.read_bytes()


def test_fixture_against_oracle(oracle):
    """Every fixture frame's expected checksums are the oracle's tcp_checksums()
    results; frame 0 is the unit-test KAT a3 bb / cf d7; the batch holds data
    segments, ACKs and fast_flows_kernelxsums frames."""
    n, room, recs, frames = load_fixture()
    assert n == 33 and room == 2048
    exp = oracle.tcp4_batch(frames.copy().ravel(), n, stride=room)
    assert [(r[1], r[2]) for r in recs] == [(int(exp[2 * i]), int(exp[2 * i + 1])) for i in range(n)]
    assert frames[0, 24:26].tolist() == [0, 0] and recs[0][1:3] == (0xBBA3, 0xD7CF)
    kinds = [r[3] for r in recs]
    assert kinds.count(1) == 12 and kinds.count(2) >= 2
    for i, r in enumerate(recs):                     # tx_send length = 14 + ip.len
        assert r[0] == 14 + (int(frames[i, 16]) << 8 | int(frames[i, 17]))


@pytest.mark.skipif(not (REF_INC / "packet_defs.h").exists(), reason="needs /root/reference (build container)")
def test_boundary_binary_links_only_libtasx():
    from tas_amd import build
    exe = build.build_c_tests()
    dyn = subprocess.run(["readelf", "-d", str(exe)], capture_output=True, text=True, check=True).stdout
    assert "libtasx.so" in dyn and "oracle" not in dyn


@pytest.mark.gpu
def test_c_boundary_glue_on_gpu():
    """INTEGRATION.md's glue, compiled against the reference's types, over fake
    mbufs: the unit-test frame and a 32-frame tx_flush batch, staged,
    zero-copy and through the shared feeder, bit-exact against the fixture;
    then a flush through an aborted flush server, recovered by the glue."""
    assert BIN.exists(), f"{BIN} not built (python -c 'import __graft_entry__ as g; g.build()' with /root/reference)"
    r = subprocess.run([str(BIN), str(FIXTURE)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "staged, zero-copy and feeder: OK" in r.stdout
    # ABI 8 error contract: an aborted server fails the flush, the glue finishes
    # all 33 frames on TAS's CPU path (bit-exact), the next flush is the GPU's
    assert "aborted flush server, 33 frames finished by the glue's CPU path, then the GPU again: OK" in r.stdout
