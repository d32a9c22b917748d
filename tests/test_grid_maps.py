"""The RX pass's grid arithmetic, restated on the CPU (no GPU work): the
XCD-matched split grid (tcp4_tas14_kernel<..., flow>,
tas_amd/csrc/xsum_kernels.hip, and launch_splitx) must look every frame up
exactly once, from a lookup block on the same XCD (blockIdx % 8) as the
frame's verify block; and the XCD-run block order of large grids (xcd_run,
tas_amd/csrc/xsum_device.h, round 5) must sum every block once and give each
XCD runs of consecutive blocks.  The GPU tests check the kernels at a few
batch sizes (tests/test_rx_fused.py); these sweep the formulas over many."""
import numpy as np
import pytest

ROWS = 16  # verify rows (frames) per 256-thread block


def lookup_blocks(nv: int, f: int) -> int:
    """splitx_lookup_blocks<F>: a multiple of 8 covering nv verify blocks, 16 F per lookup block."""
    return ((nv + 16 * f - 1) // (16 * f) + 7) & ~7


def splitx_frames(n: int, f: int):
    """(frame, lookup block) for every lookup lane and frame slot of the grid."""
    nv = (n + ROWS - 1) // ROWS
    nl = lookup_blocks(nv, f)
    b = np.arange(nl)[:, None, None]
    slot = np.arange(f)[None, :, None]
    t = np.arange(256)[None, None, :]
    vbk = 8 * (16 * f * (b // 8) + 16 * slot + t // 16) + (b & 7)
    i0 = vbk * ROWS + (t & 15)
    blk = np.broadcast_to(b, i0.shape)
    return i0.ravel(), blk.ravel(), nl


@pytest.mark.parametrize("f", [1, 2])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 255, 256, 257, 2047, 2048, 2049, 4095, 4096, 4097, 65536, 70007])
def test_splitx_covers_every_frame_once_on_its_xcd(n, f):
    i0, blk, nl = splitx_frames(n, f)
    assert nl % 8 == 0
    live = i0 < n
    frames = i0[live]
    assert np.array_equal(np.sort(frames), np.arange(n))  # each frame exactly once
    # the frame's verify block runs at blockIdx nl + vb: same XCD as its lookup block
    vb = frames // ROWS
    assert np.array_equal((nl + vb) % 8, blk[live] % 8)


def xcd_run(b, nb, xrun):
    """tas_amd/csrc/xsum_device.h xcd_run, restated (numpy, vectorised over b):
    dispatched block b (XCD b % 8) -> the logical block it sums.  Windows of
    8 * S blocks (S = 2^(xrun - 1)) in which XCD x takes S consecutive logical
    blocks; the blocks past the last whole window stay in grid order."""
    b = np.asarray(b, dtype=np.int64)
    if xrun == 0:
        return b
    sh = xrun - 1
    wmask = (8 << sh) - 1
    o = b & wmask
    mapped = (b & ~wmask) + ((o & 7) << sh) + (o >> 3)
    return np.where(b >= (nb & ~wmask), b, mapped)


@pytest.mark.parametrize("xrun", [0, 1, 2, 5, 7, 9, 10])
@pytest.mark.parametrize("nb", [1, 7, 8, 9, 255, 256, 2047, 2048, 2049, 16384, 16385, 65536 + 1000, 524288])
def test_xcd_run_is_a_permutation(nb, xrun):
    """Every logical block is summed exactly once, whatever the grid size
    (the product applies xrun 9 from 16,384 blocks up: config 4 is 524,288)."""
    m = xcd_run(np.arange(nb), nb, xrun)
    assert np.array_equal(np.sort(m), np.arange(nb))


@pytest.mark.parametrize("xrun", [1, 7, 9])
def test_xcd_run_gives_each_xcd_consecutive_runs(xrun):
    """Inside whole windows, the blocks the dispatcher deals to one XCD
    (b % 8 == x) sum runs of S = 2^(xrun - 1) consecutive logical blocks."""
    s = 1 << (xrun - 1)
    nb = 8 * s * 5 + 3  # five whole windows and a grid-order tail
    m = xcd_run(np.arange(nb), nb, xrun)
    for x in range(8):
        mine = m[np.arange(nb) % 8 == x][: 5 * s]
        runs = mine.reshape(5, s)
        assert (np.diff(runs, axis=1) == 1).all()          # consecutive inside a run
        assert (runs[:, 0] % s == 0).all()                 # runs start on run boundaries
    assert np.array_equal(m[8 * s * 5:], np.arange(8 * s * 5, nb))  # the tail in grid order
