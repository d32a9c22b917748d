"""Probe: TCP4 batches that mix TAS data segments with pure ACKs.

A real tx_flush batch (fastemu.c:544-566) holds both: flow_tx_segment frames
(1514 B, ip.len 1500) and flow_tx_ack frames (66 B, ip.len 52, fast_flows.c:957-1030),
all in 2048 B mbuf rooms.  This times the TCP4 kernels on such batches (random
order, ACK fraction swept) against the uniform data batch, checks every result
against the oracle, and prints one JSON line per case.

  python tools/ackmix_probe.py [--steps 200] [--variants 0,2,3]
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
from tas_amd import pktgen, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rotate", type=int, default=12)
    ap.add_argument("--fracs", default="0,0.25,0.5,0.75")
    ap.add_argument("--variants", default="0,3,8")
    ap.add_argument("--hints", default="per,none,max")
    ap.add_argument("--verify", action="store_true", help="RX verification of checksummed frames instead of TX")
    ap.add_argument("--offsets", action="store_true", help="frames by an offsets array (i * 2048) instead of stride mode")
    a = ap.parse_args()
    n, stride = a.n, pktgen.MBUF_ROOM
    orc = Oracle()
    rng = np.random.default_rng(7)
    for frac in [float(x) for x in a.fracs.split(",")]:
        pay = np.where(rng.random(n) < frac, 0, pktgen.TCP_MSS).astype(np.int64)
        host = pktgen.tcp4_frames(n, payload=pay, stride=stride)
        exp = orc.tcp4_batch(host.copy(), n, stride=stride)
        if a.verify:  # received frames: checksummed in place, flags expected from the oracle
            orc.tcp4_batch(host, n, stride=stride, inplace=True)
            exp = orc.tcp4_verify_batch(host.copy(), n, stride=stride)
        tl = pay + 52
        flen = torch.from_numpy((tl + pktgen.ETH_LEN).astype(np.int32)).cuda()
        alg = int((tl + 4).sum())
        first = torch.from_numpy(host).cuda()
        bufs = [first] + [first.clone() for _ in range(a.rotate - 1)]
        out = torch.empty(2 * n, dtype=torch.int16, device="cuda")
        for v in [int(x) for x in a.variants.split(",")]:
            xsum.set_kernel_variant(v)
            for hint in a.hints.split(","):
                fl = flen if hint == "per" else None
                fl0 = pktgen.ETH_LEN + 1500 if hint == "max" else 0  # uniform MTU hint (rooms are 2048 B)
                offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride if a.offsets else None
                out.zero_()
                if a.verify:
                    got = xsum.tcp4_verify_batch(bufs[0], n, stride=0 if a.offsets else stride, offsets=offs,
                                                 frame_len=fl if fl is not None else (fl0 or None))
                    torch.cuda.synchronize()
                    ok = np.array_equal(got.cpu().numpy(), exp)
                    out = torch.empty(n, dtype=torch.uint8, device="cuda")
                else:
                    xsum.tcp4_cksum_batch(bufs[0], n, stride=0 if a.offsets else stride, offsets=offs, out=out,
                                          frame_len=fl if fl is not None else (fl0 or None))
                    torch.cuda.synchronize()
                    ok = np.array_equal(out.cpu().numpy().view(np.uint16), exp)
                # direct C-ABI calls with prebuilt arguments (no wrapper overhead in the loop)
                fn = xsum.lib().tasx_tcp4_verify_batch_dev_hint if a.verify else xsum.lib().tasx_tcp4_cksum_batch_dev_hint
                s = torch.cuda.current_stream().cuda_stream
                args = [(b.data_ptr(), offs.data_ptr() if a.offsets else None, 0 if a.offsets else stride, fl.data_ptr() if fl is not None else None, fl0, n,
                         pktgen.ETH_LEN, pktgen.ETH_LEN + pktgen.IP_LEN, out.data_ptr(), *(() if a.verify else (0,)), s)
                        for b in bufs]
                for k in range(20):
                    assert fn(*args[k % a.rotate]) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for k in range(a.steps):
                    fn(*args[k % a.rotate])
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.steps
                print(json.dumps({"ack_frac": frac, "variant": v, "hint": hint, "offsets": a.offsets, "verify": a.verify, "bit_exact": ok,
                                  "us": round(us, 3), "alg_bytes": alg,
                                  "GBps": round(alg / us / 1e3, 1), "frac_8TBps": round(alg / us / 8e6, 4)}),
                      flush=True)
        del bufs, first
    xsum.set_kernel_variant(0)


if __name__ == "__main__":
    main()
