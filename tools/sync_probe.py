"""Probe: the host cost of torch.cuda.synchronize() on an idle device, by the
number of streams that exist, against hipDeviceSynchronize / hipStreamSynchronize
called directly, and after libtasx is loaded.  Medians of 200 calls, microseconds."""
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def med(fn, n=200):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(ts), 2)


hip = ctypes.CDLL("libamdhip64.so")
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
out = {"torch_sync_idle": med(torch.cuda.synchronize),
       "hipDeviceSynchronize": med(lambda: hip.hipDeviceSynchronize()),
       "hipStreamSynchronize_null": med(lambda: hip.hipStreamSynchronize(None))}
x = torch.empty(1 << 20, device="cuda")
def after_kernel():
    x.add_(1)
    torch.cuda.synchronize()
out["torch_add_then_sync"] = med(after_kernel)
from tas_amd import xsum  # noqa: E402
xsum.lib()
out["torch_sync_after_libtasx"] = med(torch.cuda.synchronize)
ss = [torch.cuda.Stream() for _ in range(4)]
for s in ss:
    with torch.cuda.stream(s):
        x.add_(1)
torch.cuda.synchronize()
out["torch_sync_4_streams"] = med(torch.cuda.synchronize)
ss += [torch.cuda.Stream() for _ in range(12)]
for s in ss:
    with torch.cuda.stream(s):
        x.add_(1)
torch.cuda.synchronize()
out["torch_sync_16_streams"] = med(torch.cuda.synchronize)
out["torch_add_then_sync_16_streams"] = med(after_kernel)
print(json.dumps(out))
