"""Config 5 (16,384 TSO segments, 1.07 GB) with tcp4_tas_kernel's grid in
grid order against XCD runs (A/B build: tasx_ab_set_xrun K = runs of
2^(K-1) blocks; the product applies XCD runs from 16,384 blocks up, and this
grid has 1,024), beside the streaming read of the same bytes in the same
orders, alternating rounds.  Run with TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so.
    python tools/tso_xrun_probe.py [--rounds 3] [--launches 200]"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from tas_amd import benchloop, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=200)
    a = ap.parse_args()
    L = xsum.lib()
    assert xsum.library_path().name == "libtasx_ab.so", "run with TASX_LIB=.../libtasx_ab.so"
    wl = bench.tso_workload(0)
    run = wl.loop(benchloop.HINT)
    bench.prewarm(run)
    cur = torch.cuda.current_stream()

    def timed():
        run(0, 10)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        run(10, a.launches)
        e1.record(cur)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.launches

    for r in range(a.rounds):
        row = {"round": r}
        for x in (0, 5, 6, 7, 8, 9):
            assert L.tasx_ab_set_xrun(x) == 0
            row[f"x{x}"] = round(timed(), 3)
            assert xsum.last_kernel() == "tcp4_tas_kernel", xsum.last_kernel()
        L.tasx_ab_set_xrun(-1)
        row["read"] = round(bench.read_ceiling(wl, 1.0)["us"], 3)
        print(json.dumps(row), flush=True)
    # parity in XCD order: every segment's checksums against the default order
    L.tasx_ab_set_xrun(0)
    run(0, 1)
    torch.cuda.synchronize()
    ref = [o.clone() for o in wl.outs]
    L.tasx_ab_set_xrun(7)
    run(0, 1)
    torch.cuda.synchronize()
    print(json.dumps({"xrun7_matches_grid_order": bool(torch.equal(ref[0], wl.outs[0]))}), flush=True)


if __name__ == "__main__":
    main()
