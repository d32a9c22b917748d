"""Probe: the TX segment build with one segment per wave (A/B
TASX_TXSEG_DEBUG=29) against the product row kernel, on bench.py's 64K-segment
workload with its ring wraps (~9 % of segments) and on the same segments laid
out without wraps.  Run with TASX_LIB=tas_amd/_lib/libtasx_ab.so; the variant
is switched per case through TASX_TXSEG_DEBUG (read by the A/B library at
each call).  Results are compared against the product's frames."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402


def timed(loop, steps=200, R=8):
    loop(0, 2 * R)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    loop(0, steps)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def main():
    tw = bench.TxSegWorkload(8, pktgen.SEED + 2000)
    segs_wrap = tw.segs_np.copy()
    nflows = 8192
    segs_nowrap = segs_wrap.copy()
    segs_nowrap["pos"] = (np.arange(tw.n) // nflows) * pktgen.TCP_MSS
    for name, sg in (("wraps", segs_wrap), ("no_wraps", segs_nowrap)):
        tw.segs = torch.from_numpy(sg.view(np.uint8).copy()).cuda()
        res = {}
        ref = None
        for rnd in range(2):
            for v in ("0", "29"):
                os.environ["TASX_TXSEG_DEBUG"] = v
                loop = tw.loop()
                loop(0, 1)
                torch.cuda.synchronize()
                got = tw.bufs[0].cpu().numpy().copy()
                if ref is None:
                    ref = got
                res.setdefault(v, []).append((round(timed(loop), 3), xsum.last_kernel(), bool(np.array_equal(got, ref))))
        print(json.dumps({"case": name, "wrapping_segments": int((sg["pos"].astype(np.int64) + sg["payload"] > sg["tx_len"]).sum()),
                          "results": res}), flush=True)


if __name__ == "__main__":
    main()
