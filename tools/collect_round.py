"""Copy one gpu_round.sh pass (gpurun_out/TAG) into profiles/DIR/TAG/: the
logs, the bench lines as pretty JSON and the rocprofv3 kernel-stats summary
(whichever of them the pass produced: PART=a has no rocprof run); prints a
summary.

    python tools/collect_round.py TAG [--dir r06]
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
    ap.add_argument("--dir", default="r06")
    a = ap.parse_args()
    src = ROOT / "gpurun_out" / a.tag
    dst = ROOT / "profiles" / a.dir / a.tag
    dst.mkdir(parents=True, exist_ok=True)
    for log in sorted(src.glob("*.log")):
        shutil.copy(log, dst / log.name)
    for name in ("bench", "bench_k20", "bench_mixed", "bench_shard8m", "bench_tso", "bench_n2"):
        if not (src / f"{name}.log").exists():
            continue
        d = last_json(src / f"{name}.log")
        d["source"] = f"gpurun_out/{a.tag}/{name}.log (tools/gpu_round.sh {a.tag})"
        (dst / f"{name}.json").write_text(json.dumps(d, indent=4) + "\n")
        r = d["roofline"]
        print(f"{name:14s} {d['value']:9.2f} GiB/s  frac {r['frac']:.4f}  launch {r['launch_avg_us']:.2f} us")
    stats = src / "prof" / "run_kernel_stats.csv"
    if not stats.exists():
        return
    shutil.copy(stats, dst / "rocprof_kernel_stats.csv")
    shutil.copy(src / "prof" / "run_agent_info.csv", dst / "rocprof_agent_info.csv")
    import csv
    for row in csv.DictReader(open(stats)):
        if "tasx" in row["Name"] or "_kernel<" in row["Name"] and "at::" not in row["Name"]:
            print(f"  rocprof {row['Name'][:78]:78s} calls {row['Calls']:>6s} avg {float(row['AverageNs']) / 1e3:7.2f} us")


if __name__ == "__main__":
    main()
