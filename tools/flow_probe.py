"""A/B of the RX flow lookup kernel variants (tuning aid, not the product).

Builds bench.py's FlowLookupWorkload once and times each variant
(tasx_set_kernel_variant: 0/1 = bitwise CRC + byte loads, 2 = bitwise + chunk
loads, 3 = LDS slice-by-4 + byte loads, 4 = LDS + chunks, 5 = LDS
byte-position tables + byte loads, 6 / 7 = 2 / 4 frames per lane) in interleaved
rounds; every variant's flow ids must equal variant 1's.

    python tools/flow_probe.py [--rounds 5] [--steps 100]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--variants", default="1,2,3,4,5")
    ap.add_argument("--no-check", action="store_true", help="diagnostic builds (TASX_FLOW_NOCRC_DIAG)")
    a = ap.parse_args()
    wl = bench.FlowLookupWorkload(4, pktgen.SEED + 3000)
    variants = [int(v) for v in a.variants.split(",")]
    ref = None
    times = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            xsum.set_kernel_variant(v)
            launch = wl.loop()
            launch(0, 8)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(0, a.steps)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.steps * 1e3)
            got = wl.fids[0].cpu()
            if ref is None:
                ref = got
            assert a.no_check or torch.equal(got, ref), f"variant {v} differs"
    xsum.set_kernel_variant(0)
    for v in variants:
        us = statistics.median(times[v])
        print(json.dumps({"variant": v, "us": round(us, 2), "mlookups_s": round(wl.N / us, 1)}), flush=True)


if __name__ == "__main__":
    main()
