"""Probe: where bench.py's fixed per-region host overhead goes (the gap between
ms_per_step and the event-timed launch average at small K).

Times, for K = 20 and 200 headline launches issued from C, the host span of the
timed region against the GPU event span, with HIP's default device scheduling
or hipDeviceScheduleSpin (set before the runtime initialises), and with the
region split into phases (event record, loop issue, synchronize).

  python tools/sync_overhead.py [--spin]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    if a.spin:
        hip = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln]
        L = ctypes.CDLL(hip[0]) if hip else ctypes.CDLL("libamdhip64.so")
        rc = L.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
        print(json.dumps({"hipSetDeviceFlags_spin_rc": rc}), flush=True)
    import bench
    from tas_amd import benchloop
    torch.cuda.set_device(0)
    wl = bench.Tcp4Workload(16, 1)
    run = wl.loop(benchloop.HINT)
    bench.prewarm(run)
    for K in (1, 20, 200):
        rows = []
        for r in range(a.reps):
            cur = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(cur)
            t1 = time.perf_counter()
            run(r * K, K)
            t2 = time.perf_counter()
            e1.record(cur)
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            rows.append(((t4 - t0) * 1e6, e0.elapsed_time(e1) * 1e3, (t1 - t0) * 1e6, (t2 - t1) * 1e6,
                         (t3 - t2) * 1e6, (t4 - t3) * 1e6))
        import numpy as np
        m = np.median(np.array(rows), axis=0)
        print(json.dumps({"spin": a.spin, "K": K, "host_us": round(m[0], 2), "event_us": round(m[1], 2),
                          "overhead_us": round(m[0] - m[1], 2), "record0_us": round(m[2], 2),
                          "issue_us": round(m[3], 2), "record1_us": round(m[4], 2), "sync_us": round(m[5], 2),
                          "event_per_launch_us": round(m[1] / K, 3), "host_per_launch_us": round(m[0] / K, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
