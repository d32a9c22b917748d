"""A/B of the RAW kernel variants on the 8M x 1500 B batch (BASELINE.json
config 4 at N=1, 12.6 GB) -- tuning aid, interleaved rounds in one process.

    python tools/ab_raw_big.py [--variants 2,6] [--rounds 3] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from tas_amd import xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="2,6")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--n", type=int, default=8 << 20)
    a = ap.parse_args()
    n, ln = a.n, 1500
    buf = torch.randint(0, 256, (n * ln,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    vs = [int(v) for v in a.variants.split(",")]
    ref = None
    res = {v: [] for v in vs}
    for r in range(a.rounds):
        for v in vs:
            xsum.set_kernel_variant(v)
            xsum.raw_cksum_batch(buf, n, stride=ln, len0=ln, out=out)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            if ref is None:
                ref = got.copy()
            assert np.array_equal(ref, got), f"variant {v} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                xsum.raw_cksum_batch(buf, n, stride=ln, len0=ln, out=out)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.steps * 1e3)
    xsum.set_kernel_variant(0)
    for v in vs:
        us = float(np.median(res[v]))
        print(json.dumps({"variant": v, "us": round(us, 1), "GBps": round(n * (ln + 2) / us / 1e3, 1),
                          "all_us": [round(x, 1) for x in res[v]]}), flush=True)


if __name__ == "__main__":
    main()
