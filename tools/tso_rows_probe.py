"""Config 5 (16,384 TSO segments, 1.07 GB): tcp4_tas_kernel with 6 (the
product), 12 and 24 loads per lane a round (A/B variants 49, 50: fewer bubbles
between a 64 KB row's rounds), alternating rounds, beside the streaming read;
each variant's results compared with the product's.  Run with
TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so.  The record of profiles/r05 r05w:
variants 49 / 50 were removed after it (no gain), so this no longer runs
as is.
    python tools/tso_rows_probe.py [--rounds 3] [--launches 200]"""
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

    names = {0: "tcp4_tas_kernel", 49: "tcp4_tas_kernel<12>", 50: "tcp4_tas_kernel<24>"}
    for r in range(a.rounds):
        row = {"round": r}
        for v, name in names.items():
            assert L.tasx_set_kernel_variant(v) == 0
            row[f"v{v}"] = round(timed(), 3)
            assert xsum.last_kernel() == name, xsum.last_kernel()
        L.tasx_set_kernel_variant(0)
        row["read"] = round(bench.read_ceiling(wl, 1.0)["us"], 3)
        print(json.dumps(row), flush=True)
    same = {}
    L.tasx_set_kernel_variant(0)
    run(0, 1)
    torch.cuda.synchronize()
    ref = wl.outs[0].clone()
    for v in (49, 50):
        wl.outs[0].zero_()
        L.tasx_set_kernel_variant(v)
        run(0, 1)
        torch.cuda.synchronize()
        same[f"v{v}_matches_product"] = bool(torch.equal(ref, wl.outs[0]))
    L.tasx_set_kernel_variant(0)
    print(json.dumps(same), flush=True)


if __name__ == "__main__":
    main()
