"""Probe the fused TX segment build against copy baselines on the GPU.

Times (HIP events over K back-to-back launches, R rotating batches):
  * torch copy_ of the payload bytes (contiguous, same byte count);
  * torch strided copy into the frames' payload windows (frames[:, 66:1514]);
  * tasx_tx_segment_batch_dev with several flow / buffer layouts.
Prints one JSON line per case.  Usage: python tools/txseg_probe.py [--steps K]
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

from tas_amd import pktgen, xsum  # noqa: E402

N, STRIDE, PAY = 65536, 2048, pktgen.TCP_MSS


def timeit(fn, steps, rot):
    for k in range(3 * rot):
        fn(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(steps):
        fn(k)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3  # us


def rnd(nbytes, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rotate", type=int, default=8)
    ap.add_argument("--only-kernel", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--case", default="", help="only cases whose name contains this")
    ap.add_argument("--room", type=int, default=STRIDE, help="descriptor room (0: frame bytes only)")
    a = ap.parse_args()
    R = a.rotate
    frames = [torch.zeros(N * STRIDE, dtype=torch.uint8, device="cuda") for _ in range(R)]
    if not a.only_kernel:
        copies(a, R, frames)
    kernel_cases(a, R, frames)


def copies(a, R, frames):
    payload_bytes = N * PAY
    # contiguous copy of the payload byte count
    src = [rnd(payload_bytes, 1 + r) for r in range(R)]
    dst = [torch.empty_like(s) for s in src]
    us = timeit(lambda k: dst[k % R].copy_(src[k % R]), a.steps, R)
    print(json.dumps({"case": "torch_copy_contig", "us": round(us, 2),
                      "GBps_rw": round(2 * payload_bytes / us / 1e3, 1)}), flush=True)
    # strided copy into frame payload windows
    views = [f.view(N, STRIDE)[:, 66:66 + PAY] for f in frames]
    srcv = [s.view(N, PAY) for s in src]
    us = timeit(lambda k: views[k % R].copy_(srcv[k % R]), a.steps, R)
    print(json.dumps({"case": "torch_copy_into_frames", "us": round(us, 2),
                      "GBps_rw": round(2 * payload_bytes / us / 1e3, 1)}), flush=True)
    del src, dst, views, srcv
    torch.cuda.empty_cache()


def kernel_cases(a, R, frames):
    fn = xsum.lib().tasx_tx_segment_batch_dev
    stream = torch.cuda.current_stream().cuda_stream
    hdr = torch.from_numpy(pktgen.tcp4_frames(N, payload=PAY, stride=STRIDE, seed=5)).cuda()
    for f in frames:
        f.copy_(hdr)
    outs = [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(R)]
    cases = [
        ("flows8192_tx16k", dict(nflows=8192, tx_len=16384)),
        ("flows65536_tx2k", dict(nflows=65536, tx_len=2048)),       # one segment per flow, many wraps
        ("flows64_tx2m", dict(nflows=64, tx_len=2 << 20)),          # few flows, rare wraps
        ("flows8192_tx16k_odd", dict(nflows=8192, tx_len=16384, odd=True)),
    ]
    for name, kw in cases:
        if a.case not in name:
            continue
        _, _, segs, shm_len = pktgen.tx_segments(N, seed=9, make_shm=False, room=a.room, **kw)
        if "flows64" in name:  # sequential: flow-major order, consecutive segments read consecutive bytes
            order = np.argsort(np.arange(N) % 64, kind="stable")
            segs = segs.copy()
            segs[["tx_base", "tx_len", "pos", "payload"]] = segs[["tx_base", "tx_len", "pos", "payload"]][order]
        dsegs = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
        shms = [rnd(shm_len, 100 + r) for r in range(R)]
        args = [(s.data_ptr(), shm_len, f.data_ptr(), dsegs.data_ptr(), N, 14, 34, o.data_ptr(), stream)
                for s, f, o in zip(shms, frames, outs)]

        def launch(k):
            assert fn(*args[k % R]) == 0
        us = timeit(launch, a.steps, R)
        alg = N * (2 * PAY + 20 + 32 + 4)
        wraps = int(((segs["pos"].astype(np.int64) + segs["payload"]) > segs["tx_len"]).sum())
        print(json.dumps({"case": name + a.tag, "us": round(us, 2), "GBps_alg": round(alg / us / 1e3, 1),
                          "wraps": wraps, "shm_MB": round(shm_len / 1e6, 1)}), flush=True)
        del shms
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
