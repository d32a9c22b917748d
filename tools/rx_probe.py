"""Probe: one RX pass (tasx_rx_batch_dev) against the two calls it replaces.

RX bursts of TAS frames in 2048 B mbufs (data segments and pure ACKs in random
order, the ACK fraction swept), flow keys from bench.py's TAS-sized flow table,
each frame's received length as its hint.  Times, per case, the product's
split grid (variant 0: lookup blocks ahead of the verify blocks), the A/B
variants --variants names (26: the lookup inside the verify rows, 27: the other
frames-per-lane choice, 32 / 35: lookup blocks on their verify blocks' XCD with
one / two frames per lane; needs TASX_LIB=tas_amd/_lib/libtasx_ab.so) and the
two kernels in turn, every
result checked against the first run's, interleaved over --rounds.  One JSON
line per case.  Launches come from C (tas_amd/benchsrc/bench_loop.c).

  TASX_LIB=tas_amd/_lib/libtasx_ab.so python tools/rx_probe.py --fracs 0,0.5,1 --rounds 2
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from tas_amd import benchloop, pktgen, xsum  # noqa: E402


def timed(loop, steps: int, R: int) -> float:
    loop(0, 2 * R)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    loop(0, steps)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rotate", type=int, default=8)
    ap.add_argument("--fracs", default="u,0,0.5,1")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="26,27", help="A/B variants timed beside the product (A/B build)")
    a = ap.parse_args()
    ab = xsum.library_path().name == "libtasx_ab.so"
    fw = bench.FlowLookupWorkload(1, pktgen.SEED + 3000)
    fracs = [x for x in a.fracs.split(",")]
    for fs in fracs:  # "u": all data, the received length as a uniform hint
        uniform = fs == "u"
        frac = 0.0 if uniform else float(fs)
        rp = bench.RxPassWorkload(fw, a.rotate, pktgen.SEED + 4000, ack_frac=frac)
        cases = [("product", benchloop.RX_FUSED, 0), ("separate", benchloop.RX_SEPARATE, 0)]
        if ab:
            cases += [(f"v{v}", benchloop.RX_FUSED, int(v)) for v in a.variants.split(",") if v]
        ref = None
        res = {k: [] for k, _, _ in cases}
        for _ in range(a.rounds):
            for name, which, var in cases:
                xsum.set_kernel_variant(var)
                try:
                    loop = rp.loop(which, uniform=uniform)
                    loop(0, 1)
                    torch.cuda.synchronize()
                    kern = xsum.last_kernel()
                    got = [t.cpu().numpy().copy() for t in (rp.flags[0], rp.fids[0], rp.hashes[0])]
                    if ref is None:
                        ref = got
                    ok = all(np.array_equal(x, y) for x, y in zip(got, ref))
                    res[name].append((timed(loop, a.steps, a.rotate), kern, ok))
                finally:
                    xsum.set_kernel_variant(0)
        for name, runs in res.items():
            print(json.dumps({"ack_frac": frac, "uniform_hint": uniform, "case": name, "kernel": runs[0][1],
                              "us": [round(r[0], 3) for r in runs], "same_results": all(r[2] for r in runs)}),
                  flush=True)
        del rp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
