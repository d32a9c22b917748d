"""Probe: TCP4 batches that mix TAS data segments with pure ACKs.

A real tx_flush batch (fastemu.c:544-566) holds both: flow_tx_segment frames
(1514 B, ip.len 1500) and flow_tx_ack frames (66 B, ip.len 52, fast_flows.c:957-1030),
all in 2048 B mbuf rooms.  This times the TCP4 kernels on such batches (random
order, ACK fraction swept) with per-frame hints or none and a room or none,
checks every result against the oracle, and prints one JSON line per case.
Launches come from C (tas_amd/benchsrc/bench_loop.c), as in bench.py.

  TASX_LIB=tas_amd/_lib/libtasx_ab.so python tools/ackmix_probe.py --variants 9,10,11 --rooms 0,2048
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oracle.oracle_lib import Oracle  # noqa: E402  (checker only)
from tas_amd import benchloop, pktgen, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rotate", type=int, default=12)
    ap.add_argument("--fracs", default="0,0.25,0.5,0.75")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--hints", default="per,none")
    ap.add_argument("--rooms", default="0,2048")
    ap.add_argument("--rounds", type=int, default=1, help="repeat the sweep (interleaved A/B)")
    ap.add_argument("--verify", action="store_true", help="RX verification of checksummed frames instead of TX")
    ap.add_argument("--offsets", action="store_true", help="frames by an offsets array (i * 2048) instead of stride mode")
    a = ap.parse_args()
    n, stride = a.n, pktgen.MBUF_ROOM
    orc = Oracle()
    rng = np.random.default_rng(7)
    s = [torch.cuda.current_stream().cuda_stream]
    for frac in [float(x) for x in a.fracs.split(",")]:
        pay = np.where(rng.random(n) < frac, 0, pktgen.TCP_MSS).astype(np.int64)
        host = pktgen.tcp4_frames(n, payload=pay, stride=stride)
        exp = orc.tcp4_batch(host.copy(), n, stride=stride)
        tl = pay + 52
        if a.verify:  # received frames: checksummed in place, flags expected from the oracle
            orc.tcp4_batch(host, n, stride=stride, inplace=True)
            exp = orc.tcp4_verify_batch_bounded(host.copy(), n, (tl + pktgen.ETH_LEN).astype(np.uint32),
                                                stride=stride)
        flen = torch.from_numpy((tl + pktgen.ETH_LEN).astype(np.int32)).cuda()
        alg = int((tl + 4).sum())
        first = torch.from_numpy(host).cuda()
        bufs = [first] + [first.clone() for _ in range(a.rotate - 1)]
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride if a.offsets else None
        outs = [torch.empty(n if a.verify else 2 * n, dtype=torch.uint8 if a.verify else torch.int16,
                            device="cuda") for _ in bufs]
        for _ in range(a.rounds):
            for v in [int(x) for x in a.variants.split(",")]:
                xsum.set_kernel_variant(v)
                for hint in a.hints.split(","):
                    for room in [int(x) for x in a.rooms.split(",")]:
                        # verify without per-frame lengths: bounded by the room / stride
                        # slot, at least each honest frame, so the same flags are expected
                        fl = flen.data_ptr() if hint == "per" else None
                        args = [benchloop.Tcp4Args(b.data_ptr(), offs.data_ptr() if a.offsets else None,
                                                   0 if a.offsets else stride, fl, 0, room, n, pktgen.ETH_LEN,
                                                   pktgen.ETH_LEN + pktgen.IP_LEN, 0, o.data_ptr())
                                for b, o in zip(bufs, outs)]
                        run = benchloop.Loop("tcp4", args, s, benchloop.VERIFY if a.verify else benchloop.ROOM)
                        outs[0].zero_()
                        run(0, 1)
                        kern = xsum.last_kernel()
                        torch.cuda.synchronize()
                        got = outs[0].cpu().numpy()
                        ok = bool(np.array_equal(got if a.verify else got.view(np.uint16), exp))
                        run(1, 20)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        torch.cuda.synchronize()
                        e0.record()
                        run(21, a.steps)
                        e1.record()
                        torch.cuda.synchronize()
                        us = e0.elapsed_time(e1) * 1e3 / a.steps
                        print(json.dumps({"ack_frac": frac, "variant": v, "hint": hint, "room": room, "kernel": kern,
                                          "offsets": a.offsets, "verify": a.verify, "bit_exact": ok,
                                          "us": round(us, 3), "alg_bytes": alg, "GBps": round(alg / us / 1e3, 1),
                                          "frac_8TBps": round(alg / us / 8e6, 4)}), flush=True)
        del bufs, first, outs
    xsum.set_kernel_variant(0)


if __name__ == "__main__":
    main()
