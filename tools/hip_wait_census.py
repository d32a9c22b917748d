"""Which HIP calls wait for the running flush server, and for how long?
(INTEGRATION.md section 4f lists the result.)

One process: the server started, one context flushing 32-frame batches
through it from a second thread the whole time; each call form below is timed
on the main thread.  A watchdog thread pauses the server if a call has not
returned after HOLD seconds (so that a call that waits for the server's stop
ends instead of hanging) and the record says so.  Since round 6 the server runs
in 5 ms epochs: a call that waits for all of the device's work waits for the
queued epochs only.  Round 5's numbers for the frees (no epochs) are
profiles/r05/INDEX.md r05free: every free returned at the stop.

    python tools/hip_wait_census.py > census.jsonl
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
from tas_amd import pktgen, xsum  # noqa: E402

HOLD = 3.0
MB = 1 << 20


def _hip():
    h = ctypes.CDLL("libamdhip64.so", mode=os.RTLD_NOLOAD)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    sig = {
        "hipMalloc": [ctypes.POINTER(vp), sz], "hipFree": [vp],
        "hipHostMalloc": [ctypes.POINTER(vp), sz, ctypes.c_uint], "hipHostFree": [vp],
        "hipHostRegister": [vp, sz, ctypes.c_uint], "hipHostUnregister": [vp],
        "hipMallocAsync": [ctypes.POINTER(vp), sz, vp], "hipFreeAsync": [vp, vp],
        "hipStreamCreateWithFlags": [ctypes.POINTER(vp), ctypes.c_uint], "hipStreamDestroy": [vp],
        "hipStreamSynchronize": [vp], "hipDeviceSynchronize": [],
        "hipMemcpy": [vp, vp, sz, ctypes.c_int], "hipMemset": [vp, ctypes.c_int, sz],
        "hipMemsetAsync": [vp, ctypes.c_int, sz, vp],
        "hipEventCreate": [ctypes.POINTER(vp)], "hipEventDestroy": [vp], "hipEventRecord": [vp, vp],
        "hipEventSynchronize": [vp],
    }
    for k, a in sig.items():
        getattr(h, k).argtypes = a
        getattr(h, k).restype = ctypes.c_int
    return h


def main():
    torch.cuda.set_device(0)
    xsum.lib()
    hip = _hip()
    vp = ctypes.c_void_p
    n, nb = 32, 64
    frames = pktgen.tcp4_frames(nb * n, payload=pktgen.TCP_MSS, stride=2048, seed=5)
    pin = xsum.PinnedBuffer(frames.size)
    pin.array[:] = frames
    dbuf = vp()
    assert hip.hipMalloc(ctypes.byref(dbuf), 16 * MB) == 0
    host = np.zeros(16 * MB, np.uint8)
    nbst = vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(nbst), 1) == 0
    torch.cuda.synchronize()
    xsum.server_start(0)
    xsum.ctx_init(3, 0, 1 << 20)
    xsum.register_frames(3, pin.addr, pin.nbytes)
    xsum.use_server(3)
    stop = threading.Event()
    flushed = [0]

    def flusher():
        while not stop.is_set():
            for b in range(nb):
                for i in range(n):
                    xsum.tcp_checksums(3, pin.addr + (b * n + i) * 2048)
                xsum.tx_flush(3)
                flushed[0] += 1
    ft = threading.Thread(target=flusher)
    ft.start()

    def case(name, prep, call):
        obj = prep()
        state = {"paused": False}
        done = threading.Event()

        def dog():
            if not done.wait(HOLD):
                state["paused"] = True
                xsum.server_pause(0)
        th = threading.Thread(target=dog)
        th.start()
        f0 = flushed[0]
        t = time.perf_counter()
        rc = call(obj)
        dt = time.perf_counter() - t
        done.set()
        th.join()
        if state["paused"]:
            xsum.server_resume(0)
        print(json.dumps({"call": name, "rc": rc if isinstance(rc, int) else 0, "seconds": round(dt, 5),
                          "waited_until_pause": state["paused"], "flushes_meanwhile": flushed[0] - f0}),
              flush=True)

    none = lambda: None  # noqa: E731

    def dmalloc():
        p = vp()
        assert hip.hipMalloc(ctypes.byref(p), 64 * MB) == 0
        return p

    def hmalloc():
        p = vp()
        assert hip.hipHostMalloc(ctypes.byref(p), 64 * MB, 0) == 0
        return p

    keep = []

    def hreg():
        a = np.zeros(64 * MB, np.uint8)
        keep.append(a)
        assert hip.hipHostRegister(vp(a.ctypes.data), a.nbytes, 0) == 0
        return vp(a.ctypes.data)

    def tseg():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        x = torch.empty(64 * MB, dtype=torch.uint8, device="cuda")
        x.fill_(1)
        return [x]

    def tfree(box):
        box.clear()
        torch.cuda.empty_cache()

    def ev_null():
        e = vp()
        hip.hipEventCreate(ctypes.byref(e))
        hip.hipEventRecord(e, None)
        return e

    t16 = torch.zeros(16 * MB, dtype=torch.uint8, device="cuda")
    cases = [
        ("torch.cuda.synchronize (hipDeviceSynchronize)", none, lambda _: torch.cuda.synchronize()),
        ("hipDeviceSynchronize", none, lambda _: hip.hipDeviceSynchronize()),
        ("torch current (null) stream synchronize", none, lambda _: torch.cuda.current_stream().synchronize()),
        ("hipStreamSynchronize(null)", none, lambda _: hip.hipStreamSynchronize(None)),
        ("hipStreamSynchronize(non-blocking stream)", none, lambda _: hip.hipStreamSynchronize(nbst)),
        ("hipEventSynchronize(event on the null stream)", ev_null, lambda e: hip.hipEventSynchronize(e)),
        ("tensor.cpu() (D2H to pageable memory, 16 MiB)", none, lambda _: t16.cpu()),
        ("torch.from_numpy().cuda() (H2D from pageable memory, 16 MiB)", none,
         lambda _: torch.from_numpy(host).cuda()),
        ("hipMemcpy D2H (pageable, 16 MiB)", none, lambda _: hip.hipMemcpy(vp(host.ctypes.data), dbuf, 16 * MB, 2)),
        ("hipMemcpy H2D (pageable, 16 MiB)", none, lambda _: hip.hipMemcpy(dbuf, vp(host.ctypes.data), 16 * MB, 1)),
        ("hipMemset (16 MiB)", none, lambda _: hip.hipMemset(dbuf, 0, 16 * MB)),
        ("hipMemsetAsync(non-blocking stream) + its stream synchronize", none,
         lambda _: hip.hipMemsetAsync(dbuf, 0, 16 * MB, nbst) or hip.hipStreamSynchronize(nbst)),
        ("hipMalloc (64 MiB)", none, lambda _: keep.append(dmalloc()) or 0),
        ("hipFree (64 MiB)", dmalloc, lambda p: hip.hipFree(p)),
        ("hipHostMalloc (64 MiB)", none, lambda _: (keep.append(hmalloc()) or 0)),
        ("hipHostFree (64 MiB)", hmalloc, lambda p: hip.hipHostFree(p)),
        ("hipHostRegister (64 MiB)", none, lambda _: (hreg() and 0)),
        ("hipHostUnregister (64 MiB)", hreg, lambda p: hip.hipHostUnregister(p)),
        ("torch.cuda.empty_cache (a 64 MiB segment)", tseg, tfree),
        ("hipStreamCreate + hipStreamDestroy", none,
         lambda _: (lambda s: hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) or hip.hipStreamDestroy(s))(vp())),
        ("hipEventCreate + hipEventDestroy", none,
         lambda _: (lambda e: hip.hipEventCreate(ctypes.byref(e)) or hip.hipEventDestroy(e))(vp())),
    ]
    for name, prep, call in cases:
        case(name, prep, call)
    # HIP maps streams onto at most GPU_MAX_HW_QUEUES (4) hardware queues; a
    # stream that shares the server's queue waits behind the server's queued
    # launches (round 5: one long kernel, so such a stream waited until the
    # stop: profiles/r05 r05q / r05r).  Eight fresh streams, a small kernel
    # and that stream's synchronize on each.
    keep_streams = []
    waits = []
    fired = []
    dog = threading.Timer(3 * HOLD, lambda: (fired.append(1), xsum.server_pause(0)))
    dog.start()
    for _ in range(8):
        st = torch.cuda.Stream()
        keep_streams.append(st)
        with torch.cuda.stream(st):
            x = torch.ones(1024, device="cuda")
            x.add_(1)
        t = time.perf_counter()
        st.synchronize()
        waits.append(round(time.perf_counter() - t, 5))
        keep.append(x)
    dog.cancel()
    dog.join()
    if fired:
        xsum.server_resume(0)
    print(json.dumps({"call": "a small kernel + hipStreamSynchronize on each of 8 fresh streams",
                      "seconds_per_stream": waits, "waited_until_pause": bool(fired)}), flush=True)
    stop.set()
    ft.join()
    ep = xsum.server_epochs(0)
    xsum.use_server(3, False)
    xsum.server_stop(0)
    xsum.ctx_destroy(3)
    print(json.dumps({"epochs": ep[0], "slow_waits": ep[1], "max_wait_ms": ep[2], "flushes": flushed[0]}), flush=True)


if __name__ == "__main__":
    main()
