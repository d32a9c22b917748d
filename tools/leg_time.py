"""Time one bench.py leg with whatever library TASX_LIB selects (A/B variants
through their env knobs), the way bench.py times it: the same workload
objects, K launches issued from C, a HIP event pair around them.  One JSON line
per repetition.  Usage on the GPU box:

  TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so TASX_TXSEG_DEBUG=10 python tools/leg_time.py txseg --tag abl10
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from tas_amd import benchloop, pktgen, xsum  # noqa: E402


def make(leg: str, rotate: int = 16):
    if leg == "txseg":
        w = bench.TxSegWorkload(rotate, pktgen.SEED + 2000)
        return w.loop(), w.bytes_per_step
    if leg in ("txseg_randpos", "txseg_nowrap"):
        # the TX segment leg with other segment positions: randpos = every
        # segment at its own random position in its flow's buffer, no wraps
        # (tools/txseg_lds_probe.hip's pattern); nowrap = the bench's flows
        # (consecutive positions) shifted so that no payload wraps
        import numpy as np
        w = bench.TxSegWorkload(16, pktgen.SEED + 2000)
        segs = w.segs_np.copy()
        rng = np.random.default_rng(5)
        if leg == "txseg_randpos":
            segs["pos"] = rng.integers(16, 16384 - 1448 - 32, len(segs)).astype(np.uint32)
        else:
            segs["pos"] = (segs["pos"].astype(np.int64) % (16384 - 1448)).astype(np.uint32)
        w.segs = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
        return w.loop(), w.bytes_per_step
    if leg == "raw":  # bench.py's raw leg: 64K x 1500 B packed payloads
        w = bench.RawWorkload(rotate, pktgen.SEED + 1000)
        return w.loop(), w.bytes_per_step
    if leg in ("shard8m", "shard1m"):  # config 4 at N = 1 (12.6 GB) / its per-GPU shard at N = 8 (1.57 GB)
        w = bench.shard8m_workload(1 if leg == "shard8m" else 8, 0)
        return w.loop(), w.bytes_per_step
    if leg == "mixed":  # config 3: 1M RAW packets of {64,576,1500,9000} B
        w = bench.mixed_workload(1, 0)
        return w.loop(), w.bytes_per_step
    if leg == "tso":  # config 5: 16,384 TSO segments
        w = bench.tso_workload(0)
        return w.loop(bench.HINT), w.bytes_per_step
    if leg == "flow":  # bench.py's flow_lookup leg: 256K lookups in TAS-sized tables
        w = bench.FlowLookupWorkload(4, pktgen.SEED + 3000)
        return w.loop(), w.N * 64
    if leg in ("flow_small", "flow_tiny"):
        # the same 256K lookups in tables that fit every XCD's L2 (small: 8192
        # flows / 16K entries = 1 MiB + 128 KiB; tiny: 1024 / 2048 = 128 KiB +
        # 16 KiB): what the lookup would take with the table levels served by L2
        nf = 8192 if leg == "flow_small" else 1024
        cls = type("SmallFlow", (bench.FlowLookupWorkload,), {"NFLOWS": nf, "ENTRIES": 2 * nf})
        w = cls(4, pktgen.SEED + 3000)
        return w.loop(), w.N * 64
    if leg == "rx":
        w = bench.RxPassWorkload(bench.FlowLookupWorkload(1, pktgen.SEED + 3000), 12, pktgen.SEED + 4000)
        return w.loop(benchloop.RX_FUSED), w.bytes_per_step
    if leg == "rx_separate":
        w = bench.RxPassWorkload(bench.FlowLookupWorkload(1, pktgen.SEED + 3000), 12, pktgen.SEED + 4000)
        return w.loop(benchloop.RX_SEPARATE), w.bytes_per_step
    if leg == "rx_verify":
        w = bench.RxPassWorkload(bench.FlowLookupWorkload(1, pktgen.SEED + 3000), 12, pktgen.SEED + 4000)
        return benchloop.Loop("tcp4", [a.v for a in w.loop(benchloop.RX_FUSED).arr], [
            torch.cuda.current_stream().cuda_stream], bench.VERIFY, "verify"), w.bytes_per_step
    if leg == "flushmix":
        w = bench.FlushMixWorkload(12, pktgen.SEED + 500)
        return w.loop(), w.bytes_per_step
    if leg == "tcp4":
        w = bench.Tcp4Workload(16, pktgen.SEED)
        return w.loop(bench.HINT), w.bytes_per_step
    if leg == "tcp4_nohint":  # bench.py's tcp4_nohint leg: no hint, room = the mbuf data room
        w = bench.Tcp4Workload(16, pktgen.SEED)
        return w.loop(bench.ROOM, flen0=0, room=bench.STRIDE), w.bytes_per_step
    if leg == "tcp4_frames_only":  # bench.py's tcp4_frames_only leg
        w = bench.Tcp4Workload(16, pktgen.SEED)
        return w.loop(bench.DEV, flen0=0), w.bytes_per_step
    raise SystemExit(f"unknown leg {leg}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("leg")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default="")
    ap.add_argument("--rotate", type=int, default=16, help="txseg: rotating input sets")
    ap.add_argument("--variant", type=int, default=0, help="tasx_set_kernel_variant (A/B variants need TASX_LIB)")
    a = ap.parse_args()
    xsum.lib()
    run, nbytes = make(a.leg, a.rotate)
    xsum.set_kernel_variant(a.variant)
    bench.prewarm(run)
    for r in range(a.reps):
        run(0, 20)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(20, a.steps)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.steps
        print(json.dumps({"leg": a.leg, "tag": a.tag, "rep": r, "us": round(us, 3), "kernel": xsum.last_kernel(),
                          "frac": round(nbytes / us / 1e3 / bench.HBM_PEAK_GBS, 4),
                          "lib": Path(xsum.library_path()).name, "variant": a.variant,
                          "env": {k: v for k, v in os.environ.items() if k.startswith("TASX_")}}), flush=True)


if __name__ == "__main__":
    main()
