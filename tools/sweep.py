"""Kernel-variant sweep on the GPU box (tuning aid, not part of the product).

For each (mode, variant): K back-to-back launches over R rotating batches,
GPU time measured by one event pair around the K launches (us/launch, includes
the ~1 us launch boundaries) and by per-launch event pairs (median); results
are checked bit-exact against the oracle on the first batch.

    python tools/sweep.py [--steps 200] [--rotate 16] [--modes tcp4,raw,mixed,tso]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from oracle.oracle_lib import Oracle  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402


def make(mode: str, rotate: int):
    """Returns (device buffers, launch(k, outs), out factory, bytes/launch, oracle expected)."""
    orc = Oracle()
    L = xsum.lib()
    stream = torch.cuda.current_stream().cuda_stream
    if mode in ("tcp4h", "tcp4hs"):
        n, stride = 65536, 2048
        hint = 1514 if mode == "tcp4h" else stride
        host = pktgen.tcp4_frames(n, payload=1448, stride=stride)
        exp = orc.tcp4_batch(host.copy(), n, stride=stride)
        bufs = [torch.from_numpy(host).cuda()]
        bufs += [bufs[0].clone() for _ in range(rotate - 1)]
        outs = [torch.empty(2 * n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        args = [(b.data_ptr(), None, stride, None, hint, n, 14, 34, o.data_ptr(), 0, stream)
                for b, o in zip(bufs, outs)]
        fn = L.tasx_tcp4_cksum_batch_dev_hint
        nbytes = n * 1504
    elif mode == "rawl4":  # RAW over exactly the L4 bytes of the TAS frames (no header work)
        n, stride = 65536, 2048
        host = pktgen.tcp4_frames(n, payload=1448, stride=stride)
        exp = orc.raw_batch(host[34:], n, stride=stride, len0=1480)
        bufs = [torch.from_numpy(host).cuda()]
        bufs += [bufs[0].clone() for _ in range(rotate - 1)]
        outs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        args = [(b.data_ptr() + 34, None, stride, None, 1480, n, o.data_ptr(), stream) for b, o in zip(bufs, outs)]
        fn = L.tasx_raw_cksum_batch_dev
        nbytes = n * 1482
    elif mode == "tcp4":
        n, stride = 65536, 2048
        host = pktgen.tcp4_frames(n, payload=1448, stride=stride)
        exp = orc.tcp4_batch(host.copy(), n, stride=stride)
        bufs = [torch.from_numpy(host).cuda()]
        bufs += [bufs[0].clone() for _ in range(rotate - 1)]
        outs = [torch.empty(2 * n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        args = [(b.data_ptr(), None, stride, n, 14, 34, o.data_ptr(), 0, stream) for b, o in zip(bufs, outs)]
        fn = L.tasx_tcp4_cksum_batch_dev
        nbytes = n * 1504
    elif mode == "tso":
        n, stride = 16384, 65552
        host = pktgen.tcp4_frames(n, payload=0, stride=stride, ip_total_len=65535)
        exp = orc.tcp4_batch(host.copy(), n, stride=stride)
        rotate = min(rotate, 3)
        bufs = [torch.from_numpy(host).cuda()]
        bufs += [bufs[0].clone() for _ in range(rotate - 1)]
        outs = [torch.empty(2 * n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        args = [(b.data_ptr(), None, stride, n, 14, 34, o.data_ptr(), 0, stream) for b, o in zip(bufs, outs)]
        fn = L.tasx_tcp4_cksum_batch_dev
        nbytes = n * (65535 + 4)
    elif mode.startswith("raw") and mode != "raw_mixed":
        n, ln = 65536, 1500
        st = int(mode[3:]) if len(mode) > 3 else ln   # raw2048: 1500 B payloads at a 2048 B stride
        host = pktgen.random_bytes(pktgen.SEED, n * st)
        exp = orc.raw_batch(host, n, stride=st, len0=ln)
        bufs = [torch.from_numpy(host).cuda()]
        bufs += [bufs[0].clone() for _ in range(rotate - 1)]
        outs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        args = [(b.data_ptr(), None, st, None, ln, n, o.data_ptr(), stream) for b, o in zip(bufs, outs)]
        fn = L.tasx_raw_cksum_batch_dev
        nbytes = n * (ln + 2)
    elif mode == "mixed":
        n = 1 << 20
        lens = pktgen.mixed_lengths(n).astype(np.int64)
        slot = (lens + 15) // 16 * 16
        offs = np.zeros(n, np.int64)
        np.cumsum(slot[:-1], out=offs[1:])
        host = pktgen.random_bytes(7, int(offs[-1] + slot[-1]))
        exp = orc.raw_batch(host, n, offsets=offs, lengths=lens)
        rotate = 1  # 2.9 GB per batch: far beyond the Infinity Cache already
        bufs = [torch.from_numpy(host).cuda()]
        doff = torch.from_numpy(offs).cuda()
        dlen = torch.from_numpy(lens.astype(np.int32)).cuda()
        outs = [torch.empty(n, dtype=torch.int16, device="cuda")]
        args = [(bufs[0].data_ptr(), doff.data_ptr(), 0, dlen.data_ptr(), 0, n, outs[0].data_ptr(), stream)]
        fn = L.tasx_raw_cksum_batch_dev
        nbytes = int(lens.sum()) + 2 * n
        bufs += [doff, dlen]
    else:
        raise ValueError(mode)
    return fn, args, outs, nbytes, exp


def measure(fn, args, steps):
    R = len(args)
    for k in range(2 * R):
        assert fn(*args[k % R]) == 0, xsum.last_error()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for k in range(steps):
        fn(*args[k % R])
    b.record()
    torch.cuda.synchronize()
    wall_us = a.elapsed_time(b) * 1e3 / steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for k in range(steps):
        ev[k][0].record()
        fn(*args[k % R])
        ev[k][1].record()
    torch.cuda.synchronize()
    per = float(np.median([x.elapsed_time(y) for x, y in ev])) * 1e3
    return wall_us, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rotate", type=int, default=16)
    ap.add_argument("--modes", default="tcp4,raw")
    ap.add_argument("--variants", default="1,2,3")
    ap.add_argument("--rounds", type=int, default=3, help="interleaved rounds per config (median)")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    xsum.lib()
    rows = []
    for mode in args.modes.split(","):
        fn, fargs, outs, nbytes, exp = make(mode, args.rotate)
        configs = []
        for v in map(int, args.variants.split(",")):
            xsum.set_kernel_variant(v)
            outs[0].zero_()
            if fn(*fargs[0]) != 0:  # variant not available for this mode
                continue
            torch.cuda.synchronize()
            got = outs[0].cpu().numpy().view(np.uint16)
            configs.append((v, 0, bool(np.array_equal(got, exp))))
        # prewarm the clocks, then interleave rounds over all configs (rule 24)
        xsum.set_kernel_variant(configs[0][0])
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            for k in range(32):
                fn(*fargs[k % len(fargs)])
            torch.cuda.synchronize()
        steps = args.steps if mode not in ("mixed", "tso") else max(10, args.steps // 10)
        res = {c: [] for c in configs}
        for _ in range(args.rounds):
            for c in configs:
                xsum.set_kernel_variant(c[0])
                res[c].append(measure(fn, fargs, steps))
        for c in configs:
            wall = float(np.median([w for w, _ in res[c]]))
            per = float(np.median([e for _, e in res[c]]))
            row = dict(mode=mode, variant=c[0], ppg=c[1], exact=c[2], wall_us=round(wall, 2),
                       event_us=round(per, 2), gbs_wall=round(nbytes / wall / 1e3, 1),
                       gbs_event=round(nbytes / per / 1e3, 1),
                       wall_min=round(min(w for w, _ in res[c]), 2))
            rows.append(row)
            print(json.dumps(row), flush=True)
        del fn, fargs, outs
        torch.cuda.empty_cache()
    xsum.set_kernel_variant(0)


if __name__ == "__main__":
    main()
