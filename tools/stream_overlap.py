"""Probe: the headline batches issued round-robin over S streams (independent
batches, as S TAS fast-path contexts would submit them), to price the per-launch
ramp-up / drain that one stream serialises.  Whole-job rate = K batches / wall.

    python tools/stream_overlap.py [--streams 1,2,3,4] [--steps 400]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from tas_amd import benchloop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    wl = bench.Tcp4Workload(16, 0x5EED, host=False)
    streams = [torch.cuda.Stream() for _ in range(8)]
    res = {}
    for _ in range(a.rounds):
        for S in [int(s) for s in a.streams.split(",")]:
            run = wl.loop(benchloop.HINT, streams=streams[:S])  # batch k on stream k % S, from C
            run(0, 64)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(64, a.steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res.setdefault(S, []).append(dt / a.steps * 1e6)
    for S, v in res.items():
        us = min(v)
        print(json.dumps({"streams": S, "us_per_batch": round(us, 3),
                          "GBps_alg": round(wl.n * 1504 / us / 1e3, 1), "all": [round(x, 3) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
