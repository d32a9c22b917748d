"""Config 5 (16,384 TSO segments): tcp4_tas_kernel with 16-lane rows (the
product) against 32-lane rows (A/B variant 5: half the concurrent 64 KB
streams per block) and one block per frame (A/B 51: one contiguous stream
per block), alternating rounds, with the read of the same bytes; each
variant's results against the product's, on config 5 and on the headline's
1500-byte frames.  Run with TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so.  The record of profiles/r05
r05zf: variant 51 was removed after it (kept as r05zf/tso_block_kernel.diff)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from tas_amd import benchloop, xsum  # noqa: E402

L = xsum.lib()
assert xsum.library_path().name == "libtasx_ab.so"
wl = bench.tso_workload(0)
run = wl.loop(benchloop.HINT)
bench.prewarm(run)
cur = torch.cuda.current_stream()


def timed(k=200):
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
    for v, name in ((0, "tcp4_tas_kernel"), (5, "tcp4_tas_kernel<g32>"), (51, "tcp4_tso_block_kernel")):
        assert L.tasx_set_kernel_variant(v) == 0
        row[f"v{v}"] = round(timed(), 3)
        assert xsum.last_kernel() == name, xsum.last_kernel()
    L.tasx_set_kernel_variant(0)
    row["read"] = round(bench.read_ceiling(wl, 1.0)["us"], 3)
    print(json.dumps(row), flush=True)
def same(wl, run, v):
    L.tasx_set_kernel_variant(0)
    run(0, 1)
    torch.cuda.synchronize()
    ref = wl.outs[0].clone()
    wl.outs[0].zero_()
    L.tasx_set_kernel_variant(v)
    run(0, 1)
    torch.cuda.synchronize()
    L.tasx_set_kernel_variant(0)
    return bool(torch.equal(ref, wl.outs[0]))


hw = bench.Tcp4Workload(1, 1234, host=False)
hrun = hw.loop(benchloop.DEV, flen0=0)   # frames only: the product's tcp4_tas_kernel path is variant 3
print(json.dumps({"g32_matches": same(wl, run, 5), "block_matches": same(wl, run, 51),
                  "block_matches_1500B": same(hw, hrun, 51)}), flush=True)
