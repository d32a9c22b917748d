"""Split a rocprofv3 kernel trace of tools/price_leg.py into the server_cost
leg's states and report the headline and TX kernels' own durations in each
(median, and the median gap between consecutive launches), so the server's
cost to device-resident work can be told from host-side launch gaps.
States: before the first flush_server_kernel starts (stopped), while the
first one runs (idle), while the second one runs (busy: the 8 x 3 flush run
starts its own server), after it (stopped again).
Usage: python3 tools/price_trace.py gpurun_out/TAG/prof/price_kernel_trace.csv"""
import csv
import json
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    srv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                 if "flush_server_kernel" in r["Kernel_Name"])
    if len(srv) < 2:
        raise SystemExit(f"expected two server kernels, found {len(srv)}")

    def state(t):
        if t < srv[0][0]:
            return "stopped"
        if t <= srv[0][1]:
            return "idle"
        if srv[1][0] <= t <= srv[1][1]:
            return "busy_8x3"
        return "stopped_after" if t > srv[1][1] else "between"

    kinds = {"headline": "tcp4_tas14_kernel<6, 0, false, 1, false, 256, false, 0, 0>", "tx_segment": "tx_segment_lds_kernel"}
    out = {}
    for name, key in kinds.items():
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                    if key in r["Kernel_Name"])
        per = {}
        prev_end = None
        for s, e in ks:
            st = state(s)
            d = per.setdefault(st, {"dur": [], "gap": []})
            d["dur"].append((e - s) / 1e3)
            if prev_end is not None and state(prev_end) == st and s >= prev_end:
                d["gap"].append((s - prev_end) / 1e3)
            prev_end = e
        out[name] = {st: {"launches": len(d["dur"]), "median_us": round(statistics.median(d["dur"]), 3),
                          "median_gap_us": round(statistics.median(d["gap"]), 3) if d["gap"] else None}
                     for st, d in per.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
