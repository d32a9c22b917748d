"""Copy one gpu_round.sh pass (gpurun_out/TAG) into profiles/: the bench lines
as pretty JSON and the rocprofv3 kernel-stats summary; prints a summary.

    python tools/collect_round.py TAG [--prefix r01]
"""
from __future__ import annotations

import argparse
import json
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def last_json(log: Path) -> dict:
    for line in reversed(log.read_text().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise ValueError(f"no JSON line in {log}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--prefix", default="r01")
    a = ap.parse_args()
    src = ROOT / "gpurun_out" / a.tag
    dst = ROOT / "profiles"
    for name, out in (("bench", "bench"), ("bench_mixed", "bench_mixed"), ("bench_shard8m", "bench_shard8m"),
                      ("bench_tso", "bench_tso")):
        d = last_json(src / f"{name}.log")
        d["source"] = f"gpurun_out/{a.tag}/{name}.log (tools/gpu_round.sh {a.tag})"
        (dst / f"{a.prefix}_{out}.json").write_text(json.dumps(d, indent=4) + "\n")
        r = d["roofline"]
        print(f"{out:14s} {d['value']:9.2f} GiB/s  frac {r['frac']:.4f}  launch {r['launch_avg_us']:.2f} us")
    shutil.copy(src / "prof" / "run_kernel_stats.csv", dst / f"{a.prefix}_rocprof_kernel_stats.csv")
    shutil.copy(src / "prof" / "run_agent_info.csv", dst / f"{a.prefix}_rocprof_agent_info.csv")
    import csv
    for row in csv.DictReader(open(src / "prof" / "run_kernel_stats.csv")):
        if "tasx" in row["Name"] or "_kernel<" in row["Name"] and "at::" not in row["Name"]:
            print(f"  rocprof {row['Name'][:78]:78s} calls {row['Calls']:>6s} avg {float(row['AverageNs']) / 1e3:7.2f} us")


if __name__ == "__main__":
    main()
