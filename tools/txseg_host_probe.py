"""TX segment build by data placement (not a product file): tas_shm and the
frames and the 32-byte descriptors each in HBM or in pinned host memory
mapped for the GPU, 64K TAS segments as bench.py's tx_segment leg; ms per
batch over 20 launches after 0.2 s of warm-up launches.  Shows which PCIe
traffic bounds the host-resident build."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402  (helpers only; bench's main is not run)
from tas_amd import pktgen, xsum  # noqa: E402

n, stride = bench.N_FRAMES, bench.STRIDE
_, _, segs, shm_len = pktgen.tx_segments(n, seed=pktgen.SEED + 2000, nflows=8192, tx_len=16384, make_shm=False,
                                         room=stride)
shm_d = bench.device_random(shm_len, pktgen.SEED + 7)
fr_d = bench.device_tcp4_frames(n, stride, bench.IP_TOTAL, pktgen.SEED)
segs_d = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
hs = xsum.PinnedBuffer(shm_len)
hs.array[:] = shm_d.cpu().numpy()
hf = xsum.PinnedBuffer(n * stride)
hf.array[:] = fr_d.cpu().numpy()
hd = xsum.PinnedBuffer(segs.nbytes)
hd.array[:] = segs.view(np.uint8)
out = torch.empty(n, dtype=torch.int32, device="cuda")
ref = None
for shm_where, fr_where, sg_where in [(a, b, c) for c in ("hbm", "host") for a in ("hbm", "host")
                                      for b in ("hbm", "host")]:
    if True:
        shm = shm_d if shm_where == "hbm" else hs.dev_addr
        fr = fr_d if fr_where == "hbm" else hf.dev_addr
        sg = segs_d if sg_where == "hbm" else hd.dev_addr

        def run():
            xsum.tx_segment_batch(shm, fr, sg, n, shm_len=shm_len, out=out)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.2:
            run()
            torch.cuda.synchronize()
        res = out.cpu().numpy().copy()
        if ref is None:
            ref = res
        t0 = time.perf_counter()
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        print(json.dumps({"shm": shm_where, "frames": fr_where, "segs": sg_where, "ms_per_64k": round(ms, 4),
                          "Msegs_per_s": round(n / ms / 1e3, 2),
                          "pcie_read_GBps": round(n * (1448 + 66 + 32) / ms / 1e6, 1) if shm_where == "host" else 0,
                          "pcie_write_GBps": round(n * 1514 / ms / 1e6, 1) if fr_where == "host" else 0,
                          "same_results": bool((res == ref).all())}), flush=True)
hs.free()
hf.free()
hd.free()
