"""A/B: workgroups per ring (TASX_SRV_K, A/B build) for the flush server's
checksum and TX segment slots, from C (tasxb_fastpath_mt /
tasxb_txseg_server_mt).  One JSON line per shape.  Usage on the GPU box:

  TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so TASX_SRV_K=4 python tools/server_k_ab.py --tag k4
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from tas_amd import benchloop, xsum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--flushes", type=int, default=3000)
    a = ap.parse_args()
    xsum.lib()
    dev = torch.cuda.current_device()
    for th, q in ((1, 1), (8, 3), (8, 7)):
        r = benchloop.fastpath_mt(dev, 8, th, q, a.flushes, "server")
        r["frames_per_s"] = round(r["frames_per_s"])
        t = benchloop.txseg_server_mt(dev, 8, th, q, a.flushes)
        print(json.dumps({"tag": a.tag, "shape": f"{th}x{q}", "server": r, "txseg_server": t,
                          "k": os.environ.get("TASX_SRV_K", "product")}), flush=True)


if __name__ == "__main__":
    main()
