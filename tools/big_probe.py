"""Config 4 at one GPU (8M x 1500 B RAW, 12.6 GB): the product kernel beside a
pure streaming read of the same buffer, at several batch sizes, on a torch
buffer and on a tasx_dev_alloc (hipMalloc) buffer -- why the product's share
of the trivial read falls as the batch grows.  Tuning aid.

    python tools/big_probe.py [--sizes 1024,8192] [--allocs torch,dev] [--rounds 3] [--steps 5]
    python tools/big_probe.py --pmc          # 8M, torch buffer, 3 launches per leg (under rocprofv3 --pmc)
    python tools/big_probe.py --sustain 40   # per-launch times of 40 back-to-back product launches

Legs: `prod` = libtasx.so's automatic RAW kernel (raw_sad_kernel<s32>); `vNN` =
libtasx_ab.so kernel variant NN; `xK` = libtasx_ab.so's automatic kernel with
every grid in XCD order xrun K (tasx_ab_set_xrun: 0 = grid order, K = runs of
2^(K-1) blocks); `readP` = tasx_ab_stream_read path P over the same bytes (0:
register loads in grid order, 2 + k: in XCD runs of 2^k blocks).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from tas_amd import xsum  # noqa: E402

LEN = 1500


def dev_buffer(nbytes: int, src: torch.Tensor) -> int:
    p = xsum.lib().tasx_dev_alloc(0, nbytes)
    if not p:
        raise RuntimeError("tasx_dev_alloc failed")
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(ctypes.c_void_p(p), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(nbytes), 3)
    if rc:
        raise RuntimeError(f"hipMemcpy D2D rc {rc}")
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,8192", help="packets, in units of 2^10")
    ap.add_argument("--allocs", default="torch,dev")
    ap.add_argument("--legs", default="prod,x1,x7,x8,x9,x10,x11,read0,read8,read10")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--pmc", action="store_true")
    ap.add_argument("--sustain", type=int, default=0)
    a = ap.parse_args()
    if a.pmc:
        a.sizes, a.allocs, a.rounds, a.steps = "8192", "torch", 1, 3
        a.legs = "x1,x9,read0,read10"
    prod = xsum.lib()
    ab = xsum._load(xsum.AB_LIB_PATH)
    s = torch.cuda.current_stream().cuda_stream
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    legs = a.legs.split(",")
    for m in [int(x) for x in a.sizes.split(",")]:
        n = m << 10
        nbytes = n * LEN
        src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        # batches below 2 GB rotate over copies (no step served by the 256 MiB MALL)
        rot = max(1, -(-(2 << 30) // nbytes))
        copies = [src.clone() for _ in range(rot - 1)]
        steps = max(a.steps, int(20e-3 / (nbytes / 7e12)))
        for alloc in a.allocs.split(","):
            if alloc == "dev" and rot > 1:
                continue
            bases = [src.data_ptr()] + [c.data_ptr() for c in copies] if alloc == "torch" else [dev_buffer(nbytes, src)]
            k = [0]

            def launch(leg):
                base = bases[k[0] % len(bases)]
                k[0] += 1
                if leg == "prod":
                    rc = prod.tasx_raw_cksum_batch_dev(base, None, LEN, None, LEN, n, out.data_ptr(), s)
                elif leg.startswith("v") or leg.startswith("x"):
                    rc = ab.tasx_raw_cksum_batch_dev(base, None, LEN, None, LEN, n, out.data_ptr(), s)
                else:
                    rc = ab.tasx_ab_stream_read(base, nbytes // 1024 * 1024, int(leg[4:]), sink.data_ptr(), s)
                if rc:
                    raise xsum.TasxError(rc, leg)

            def select(leg):
                # vNN: kernel variant NN; xK: the automatic kernel with XCD order xrun K
                xsum._check(ab.tasx_ab_set_xrun(int(leg[1:]) if leg.startswith("x") else -1), "xrun")
                if leg.startswith("v"):
                    xsum._check(ab.tasx_set_kernel_variant(int(leg[1:])), "variant")

            ref = None
            res = {leg: [] for leg in legs}
            names = {}
            if a.sustain:
                select("prod")
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.sustain)]
                launch("prod")
                torch.cuda.synchronize()
                for e0, e1 in ev:
                    e0.record()
                    launch("prod")
                    e1.record()
                torch.cuda.synchronize()
                ts = [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
                print(json.dumps({"n": n, "alloc": alloc, "sustain_us": [round(t, 1) for t in ts]}), flush=True)
                continue
            for r in range(a.rounds):
                for leg in legs:
                    select(leg)
                    k[0] = 0
                    launch(leg)
                    torch.cuda.synchronize()
                    if not leg.startswith("read"):
                        names[leg] = (prod if leg == "prod" else ab).tasx_last_kernel().decode()
                        got = out.cpu().numpy()
                        if ref is None:
                            ref = got.copy()
                        assert np.array_equal(ref, got), f"{leg} differs"
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(steps):
                        launch(leg)
                    e1.record()
                    torch.cuda.synchronize()
                    res[leg].append(e0.elapsed_time(e1) / steps * 1e3)
            ab.tasx_set_kernel_variant(0)
            ab.tasx_ab_set_xrun(-1)
            for leg in legs:
                us = float(np.median(res[leg]))
                alg = n * (LEN + 2) if not leg.startswith("read") else nbytes // 1024 * 1024
                print(json.dumps({"n": n, "alloc": alloc, "rot": rot, "steps": steps, "leg": leg, "kernel": names.get(leg, "stream_read"),
                                  "us": round(us, 1), "GBps": round(alg / us / 1e3, 1),
                                  "frac": round(alg / us / 1e3 / 8000, 4), "all_us": [round(x, 1) for x in res[leg]]}),
                      flush=True)
            if alloc == "dev":
                xsum.lib().tasx_dev_free(bases[0])
        del src, out, copies
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
