"""Wave-timeline diagnostic for the TCP4 TAS-layout kernel (variant 4: the
production tcp4_tas_kernel plus s_memrealtime stamps, 100 MHz).  Tuning aid only.

Per wave: t0 entry, t1 total_length known (header chunks landed), t2 data
accumulated, t3 stored.  Prints the dispatch ramp, phase latencies under load
and the number of waves alive over time.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from tas_amd import pktgen, xsum  # noqa: E402


def run(hint: int, rotate: int = 16):
    n, stride = 65536, 2048
    host = pktgen.tcp4_frames(n, payload=1448, stride=stride)
    bufs = [torch.from_numpy(host).cuda()]
    bufs += [bufs[0].clone() for _ in range(rotate - 1)]
    out = torch.empty(2 * n, dtype=torch.int16, device="cuda")
    waves = (n + 15) // 16 * 4
    diag = torch.zeros(waves * 4, dtype=torch.int64, device="cuda")
    L = xsum.lib()
    L.tasx_set_diag_buffer(diag.data_ptr())
    xsum.set_kernel_variant(4)
    st = torch.cuda.current_stream().cuda_stream
    for k in range(3 * rotate):
        assert L.tasx_tcp4_cksum_batch_dev_hint(bufs[k % rotate].data_ptr(), None, stride, None, hint, n, 14, 34,
                                                out.data_ptr(), 0, st) == 0
    torch.cuda.synchronize()
    d = diag.cpu().numpy().reshape(-1, 4).astype(np.int64)
    xsum.set_kernel_variant(0)
    L.tasx_set_diag_buffer(None)
    d = d[(d > 0).all(axis=1)]
    t = (d - d[:, 0].min()) * 10 / 1000.0  # us
    print(f"hint={hint}: {len(t)} waves, kernel span {t[:, 3].max():.2f} us")
    q = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100))
    print("  start     p0/10/50/90/100:", q(t[:, 0]))
    print("  hdr lat   (t1-t0)        :", q(t[:, 1] - t[:, 0]))
    print("  data lat  (t2-t1)        :", q(t[:, 2] - t[:, 1]))
    print("  reduce    (t3-t2)        :", q(t[:, 3] - t[:, 2]))
    print("  life      (t3-t0)        :", q(t[:, 3] - t[:, 0]))
    print("  end                      :", q(t[:, 3]))
    grid = np.arange(0, t[:, 3].max() + 0.5, 0.5)
    alive = [int(((t[:, 0] <= g) & (t[:, 3] > g)).sum()) for g in grid]
    print("  alive waves every 0.5us:", alive)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    xsum.lib()
    run(0)
    run(1514)
