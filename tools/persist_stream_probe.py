"""Do other streams keep running beside the resident flush kernel?  Starts
the kernel (one flush), then times a small torch op on a side stream and on
the default stream (diagnostic tool).  Measured stream kinds for the kernel
(profiles/r01_flush_latency.jsonl): high-priority non-blocking (adopted) and
plain non-blocking 0.04-0.1 ms on the default stream; a CU-masked stream
(blocking by construction) 99.6 ms, i.e. the kernel's whole lifetime."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tas_amd import pktgen, xsum  # noqa: E402

torch.ones(1, device="cuda").sum().item()
side = torch.cuda.Stream()
pin = xsum.PinnedBuffer(8 * 2048)
xsum.ctx_init(1, 0, 1 << 20)
xsum.register_frames(1, pin.addr, pin.nbytes)
xsum.set_persistent(1, True, cap=8)
frames = pktgen.tcp4_frames(8, payload=1448, stride=2048, seed=1)
res = {}
for trial in range(3):
    xsum.set_persistent(1, False)
    xsum.set_persistent(1, True, cap=8)
    pin.array[:] = frames
    for i in range(8):
        xsum.tcp_checksums(1, pin.addr + i * 2048)
    xsum.tx_flush(1)
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        torch.ones(1 << 20, device="cuda").sum().item()
    t1 = time.perf_counter()
    torch.ones(1 << 20, device="cuda").sum().item()
    t2 = time.perf_counter()
    res[f"side_ms_{trial}"] = round((t1 - t0) * 1e3, 2)
    res[f"default_ms_{trial}"] = round((t2 - t1) * 1e3, 2)
xsum.ctx_destroy(1)
pin.free()
print(res, flush=True)
