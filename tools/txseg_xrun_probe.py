"""The device-resident TX segment build (64K segments, tx_segment_lds_kernel,
4,096 blocks: below the product's XCD-run threshold) in grid order against
XCD runs of 16 / 64 / 256 blocks (A/B build, tasx_ab_set_xrun), alternating
rounds, with each order's built frames and results against grid order's.
Run with TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so.  The record of profiles/r05
r05zg: the TX kernel's XCD-run option was removed after it (no gain)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402

L = xsum.lib()
assert xsum.library_path().name == "libtasx_ab.so"
tw = bench.TxSegWorkload(16, pktgen.SEED + 2000)
run = tw.loop()
bench.prewarm(run)
cur = torch.cuda.current_stream()


def timed(k=400):
    run(0, 10)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cur)
    run(10, k)
    e1.record(cur)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k


for r in range(3):
    row = {}
    for x in (0, 5, 7, 9):
        assert L.tasx_ab_set_xrun(x) == 0
        row[f"x{x}"] = round(timed(), 3)
        assert xsum.last_kernel() == "tx_segment_lds_kernel", xsum.last_kernel()
    print(json.dumps(row), flush=True)
res = {}
for x in (0, 7):
    L.tasx_ab_set_xrun(x)
    tw.bufs[0].copy_(tw.bufs[1])
    run(0, 1)
    torch.cuda.synchronize()
    res[x] = (tw.bufs[0].clone(), tw.outs[0].clone())
L.tasx_ab_set_xrun(-1)
print(json.dumps({"xrun7_frames_match": bool(torch.equal(res[0][0], res[7][0])),
                  "xrun7_results_match": bool(torch.equal(res[0][1], res[7][1]))}), flush=True)
