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
from tas_amd import pktgen, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    wl = bench.Tcp4Workload(16, 0x5EED, host=False)
    fn = xsum.lib().tasx_tcp4_cksum_batch_dev_hint
    R = len(wl.bufs)
    streams = [torch.cuda.Stream() for _ in range(8)]
    res = {}
    for _ in range(a.rounds):
        for S in [int(s) for s in a.streams.split(",")]:
            ss = streams[:S]

            def launch(k):
                s = ss[k % S].cuda_stream
                rc = fn(wl.bufs[k % R].data_ptr(), None, wl.stride, None, wl.hint, wl.n, pktgen.ETH_LEN,
                        pktgen.ETH_LEN + pktgen.IP_LEN, wl.outs[k % R].data_ptr(), 0, s)
                assert rc == 0
            for k in range(64):
                launch(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                launch(k)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res.setdefault(S, []).append(dt / a.steps * 1e6)
    for S, v in res.items():
        us = min(v)
        print(json.dumps({"streams": S, "us_per_batch": round(us, 3),
                          "GBps_alg": round(wl.n * 1504 / us / 1e3, 1), "all": [round(x, 3) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
