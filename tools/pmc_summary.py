"""Median counter values per rocprofv3 --pmc run directory, for the
dispatches whose kernel name contains a pattern: one JSON line per run
directory (the compact form kept under profiles/).

    python tools/pmc_summary.py gpurun_out/r03_rx tcp4_tas14_kernel
"""
from __future__ import annotations

import csv
import json
import statistics
import sys
from pathlib import Path


def summarize(root: Path, pattern: str):
    for d in sorted(p for p in root.iterdir() if p.is_dir()):
        vals: dict[str, list[float]] = {}
        kern = set()
        for f in d.rglob("*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if pattern in r.get("Kernel_Name", ""):
                        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                        kern.add(r["Kernel_Name"])
        if vals:
            yield {"run": d.name, "kernels": sorted(kern), "dispatches": max(len(v) for v in vals.values()),
                   "median": {k: statistics.median(v) for k, v in sorted(vals.items())}}


if __name__ == "__main__":
    for line in summarize(Path(sys.argv[1]), sys.argv[2]):
        print(json.dumps(line))
