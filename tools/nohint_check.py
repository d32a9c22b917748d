"""Bit-exactness of an A/B kernel variant against the product on bench.py's
tcp4_nohint (room) and tcp4_frames_only batches (64K TAS frames, out of place),
both through the A/B build.  python tools/nohint_check.py 43"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402


def main():
    v = int(sys.argv[1])
    wl = bench.Tcp4Workload(1, pktgen.SEED)
    ok = True
    with xsum.using_library(xsum.AB_LIB_PATH):
        for name, kw in (("room", dict(room=bench.STRIDE)), ("frames_only", {})):
            res = {}
            for var in (0, v):
                xsum.set_kernel_variant(var)
                try:
                    out = torch.full((2 * wl.n,), 0x5a5a, dtype=torch.int16, device="cuda")
                    xsum.tcp4_cksum_batch(wl.bufs[0], wl.n, stride=wl.stride, out=out, **kw)
                    torch.cuda.synchronize()
                    res[var] = (out.cpu(), xsum.last_kernel())
                finally:
                    xsum.set_kernel_variant(0)
            same = torch.equal(res[0][0], res[v][0])
            ok &= same
            print(f"variant {v} {name}: {res[v][1]} same={same} (product {res[0][1]})")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
