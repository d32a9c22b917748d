"""Bit-exactness of an A/B kernel variant against the product on the bench's
data/ACK mix legs: the flush_mix TX checksums (tasx_tcp4_cksum_batch_dev_room
with per-frame hints) and the RX verification of the same frames
(tasx_tcp4_verify_batch_dev_hint), both forms called through the A/B build.

    python tools/ab_check.py 37 [n,n,...]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402


def main():
    v = int(sys.argv[1])
    ok = True
    for n in ([int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [bench.N_FRAMES]):
        ok &= check(v, n)
    if not ok:
        sys.exit(1)


def check(v: int, n: int) -> bool:
    mw = bench.FlushMixWorkload(1, pktgen.SEED + 500, n=n)
    res = {}
    with xsum.using_library(xsum.AB_LIB_PATH):
        for var in (0, v):
            xsum.set_kernel_variant(var)
            try:
                out = torch.full((2 * mw.n,), 0x5a5a, dtype=torch.int16, device="cuda")
                xsum.tcp4_cksum_batch(mw.bufs[0], mw.n, stride=mw.stride, frame_len=mw.flen, room=mw.stride,
                                      out=out)
                torch.cuda.synchronize()
                k_tx = xsum.last_kernel()
                fr = mw.bufs[0].clone()
                xsum.tcp4_cksum_batch(fr, mw.n, stride=mw.stride, frame_len=mw.flen, room=mw.stride, inplace=True,
                                      want_out=False)
                flags = torch.full((mw.n,), 0x5a, dtype=torch.uint8, device="cuda")
                xsum.tcp4_verify_batch(fr, mw.n, stride=mw.stride, frame_len=mw.flen, out=flags)
                torch.cuda.synchronize()
                res[var] = (out.cpu(), flags.cpu(), k_tx, xsum.last_kernel())
            finally:
                xsum.set_kernel_variant(0)
    a, b = res[0], res[v]
    print(f"variant {v}, n {n}: tx {b[2]} same={bool(torch.equal(a[0], b[0]))}; rx {b[3]} "
          f"same={bool(torch.equal(a[1], b[1]))} all_verified={bool((b[1] == 3).all())} (product: {a[2]}, {a[3]})")
    return torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


if __name__ == "__main__":
    main()
