"""Does a free wait for the running flush server's kernel?  (VERDICT r04,
weak item 6: "while it runs, any hipFree in the process blocks until the
stop".)  One process; for each form of free: start the server, have a
watchdog thread stop it HOLD seconds later, and time the free on the main
thread.  A free that returns well before HOLD did not wait for the kernel; one
that returns at HOLD waited until the stop.  (The stop word is stored before
the watchdog makes any HIP call, so a free that waits cannot deadlock it.)

    python tools/free_probe.py             # the runtime's frees, torch's native allocator
    PYTORCH_CUDA_ALLOC_CONF=backend:cudaMallocAsync python tools/free_probe.py torch
    TASX_FREE_PAUSED=1 python tools/free_probe.py   # each free between tasx_server_pause / _resume (ABI 9)
"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tas_amd import xsum  # noqa: E402

HOLD = 1.0
MB = 1 << 20


def _hip():
    return ctypes.CDLL("libamdhip64.so", mode=os.RTLD_NOLOAD)


def case(name, prep, free):
    obj = prep()
    torch.cuda.synchronize()
    xsum.server_start(0)
    time.sleep(0.05)
    out = {}

    def dog():
        time.sleep(HOLD)
        out["stop_at_s"] = round(time.perf_counter() - t0, 4)
        try:
            xsum.server_stop(0)
            out["stop"] = "ok"
        except xsum.TasxError as e:
            out["stop"] = str(e)

    th = threading.Thread(target=dog)
    paused = os.environ.get("TASX_FREE_PAUSED") == "1"
    t0 = time.perf_counter()
    th.start()
    if paused:
        xsum.server_pause(0)
        out["pause_s"] = round(time.perf_counter() - t0, 6)
    tf = time.perf_counter()
    rc = free(obj)
    out["free_only_s"] = round(time.perf_counter() - tf, 6)
    if paused:
        tr = time.perf_counter()
        xsum.server_resume(0)
        out["resume_s"] = round(time.perf_counter() - tr, 6)
    dt = time.perf_counter() - t0
    th.join()
    print(json.dumps({"case": name, "rc": rc, "free_s": round(dt, 4), "waited_for_stop": dt > 0.9 * HOLD, **out}),
          flush=True)


def main():
    torch.cuda.set_device(0)
    xsum.lib()
    hip = _hip()
    vp = ctypes.c_void_p
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    hip.hipFree.argtypes = [vp]
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [vp]
    hip.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [vp]
    hip.hipMallocAsync.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, vp]
    hip.hipFreeAsync.argtypes = [vp, vp]
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    only = sys.argv[1:]
    print(json.dumps({"allocator_backend": torch.cuda.get_allocator_backend()}), flush=True)

    def want(n):
        return not only or n in only

    if want("torch"):
        def prep_t():
            x = torch.empty(256 * MB, dtype=torch.uint8, device="cuda")
            x.fill_(1)
            return [x]

        def free_t(box):
            box.clear()
            torch.cuda.synchronize()  # the tensor's stream work is done before the server starts anyway
            torch.cuda.empty_cache()
            return 0
        case("torch_empty_cache", prep_t, free_t)
    if want("hipFree"):
        def prep_d():
            p = vp()
            assert hip.hipMalloc(ctypes.byref(p), 64 * MB) == 0
            return p
        case("hipFree", prep_d, lambda p: hip.hipFree(p))
    if want("hipHostFree"):
        def prep_h():
            p = vp()
            assert hip.hipHostMalloc(ctypes.byref(p), 64 * MB, 0) == 0
            return p
        case("hipHostFree", prep_h, lambda p: hip.hipHostFree(p))
    if want("hipHostUnregister"):
        keep = []

        def prep_r():
            a = np.zeros(64 * MB, np.uint8)
            keep.append(a)
            assert hip.hipHostRegister(vp(a.ctypes.data), a.nbytes, 0) == 0
            return vp(a.ctypes.data)
        case("hipHostUnregister", prep_r, lambda p: hip.hipHostUnregister(p))
    if want("hipFreeAsync"):
        st = vp()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0

        def prep_a():
            p = vp()
            assert hip.hipMallocAsync(ctypes.byref(p), 64 * MB, st) == 0
            return p
        case("hipFreeAsync", prep_a, lambda p: hip.hipFreeAsync(p, st))


if __name__ == "__main__":
    main()
