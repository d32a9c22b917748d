"""Probe: the data/ACK mix's access pattern (tasx_ab_tcp4_mix_pattern, A/B
build) over bench.py's flush_mix frames -- one frame per row (chain 0, the
product's loads), the dependent chain alone (1) and two frames per row (2,
one generation of resident rows) -- beside the product's flush_mix launch,
interleaved over --rounds.  One JSON line per case and round.

    python tools/mix_probe.py --rounds 3
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=200)
    a = ap.parse_args()
    xsum.lib()
    ab = xsum._load(xsum.AB_LIB_PATH)
    mw = bench.FlushMixWorkload(12, pktgen.SEED + 500)
    s = torch.cuda.current_stream().cuda_stream
    R = len(mw.bufs)
    outs = [torch.empty(mw.n, dtype=torch.int32, device="cuda") for _ in range(2)]

    def timed(fn):
        for k in range(20):
            fn(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for k in range(a.launches):
            fn(k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.launches

    def pat(chain):
        def f(k):
            rc = ab.tasx_ab_tcp4_mix_pattern(mw.bufs[k % R].data_ptr(), mw.stride, mw.n, mw.flen.data_ptr(),
                                             bench.IP_OFF, chain, outs[k % 2].data_ptr(), s)
            if rc:
                raise xsum.TasxError(rc, "tasx_ab_tcp4_mix_pattern")
        return f
    loop = mw.loop()

    def product():
        loop(0, 20)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        loop(0, a.launches)  # the K launches issued from C, as bench.py times them
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.launches
    for r in range(a.rounds):
        for name, fn in (("product", None), ("pattern", pat(0)), ("chain", pat(1)), ("pair_pattern", pat(2))):
            us = product() if fn is None else timed(fn)
            print(json.dumps({"case": name, "round": r, "us": round(us, 3)}), flush=True)


if __name__ == "__main__":
    main()
