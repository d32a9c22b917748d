"""The flush server's timing split per batch (A/B build, TASX_SRV_DIAG=1):
checksum slots against TX segment slots at 1 x 1 and 8 x 3, from C
(tasxb_fastpath_mt / tasxb_txseg_server_mt print the sums on stderr).  Usage
on the GPU box:

  TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so TASX_SRV_DIAG=1 python tools/server_diag.py
"""
import json, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from tas_amd import benchloop, xsum
xsum.lib()
dev = torch.cuda.current_device()
for th, q in ((1, 1), (8, 3)):
    r = benchloop.fastpath_mt(dev, 8, th, q, 3000, "server")
    print(json.dumps({"shape": f"{th}x{q}", "server": r}), flush=True)
    t = benchloop.txseg_server_mt(dev, 8, th, q, 3000)
    print(json.dumps({"shape": f"{th}x{q}", "txseg_server": t}), flush=True)
