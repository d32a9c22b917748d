"""ctypes side of libtasx_bench.so (tas_amd/benchsrc/bench_loop.c): bench.py's
timed steps are K calls of one libtasx entry point made from C, one call per
step over R rotating batches, so no Python runs between the launches of a
timed region.  Measurement plumbing only; the product API is tas_amd.xsum."""
from __future__ import annotations

import ctypes

from . import xsum
from .build import LIB_BENCH, LIB_BENCH_AB

_vp, _u32, _u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64

# tasxb_tcp4_loop entry points
DEV, HINT, ROOM, VERIFY = 0, 1, 2, 3


class Tcp4Args(ctypes.Structure):
    _fields_ = [("base", _vp), ("off", _vp), ("stride", _u64), ("flen", _vp), ("flen0", _u32),
                ("room", _u32), ("n", _u32), ("ip_off", _u32), ("l4_off", _u32), ("flags", _u32),
                ("out", _vp)]


class RawArgs(ctypes.Structure):
    _fields_ = [("base", _vp), ("off", _vp), ("stride", _u64), ("len", _vp), ("len0", _u32), ("n", _u32),
                ("out", _vp)]


class TxSegArgs(ctypes.Structure):
    _fields_ = [("shm", _vp), ("shm_len", _u64), ("frames", _vp), ("segs", _vp), ("n", _u32),
                ("ip_off", _u32), ("l4_off", _u32), ("out", _vp)]


class FlowArgs(ctypes.Structure):
    _fields_ = [("base", _vp), ("off", _vp), ("stride", _u64), ("n", _u32), ("ip_off", _u32), ("l4_off", _u32),
                ("flowht", _vp), ("ht_entries", _u32), ("flowst", _vp), ("fs_num", _u32), ("fs_stride", _u32),
                ("fs_key_off", _u32), ("hash_out", _vp), ("fid_out", _vp)]


class RxArgs(ctypes.Structure):
    _fields_ = [("v", Tcp4Args), ("f", FlowArgs)]


# tasxb_rx_loop entry points
RX_FUSED, RX_SEPARATE = 0, 1

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        # the loops call the library xsum uses (libtasx.so, or the A/B build under
        # TASX_LIB): loaded first, it is the instance the loop library binds to by soname
        path = LIB_BENCH_AB if xsum.library_path().name == "libtasx_ab.so" else LIB_BENCH
        xsum.lib()
        if not path.exists():
            raise RuntimeError(f"{path} not built; run python -c 'import __graft_entry__ as g; g.build()'")
        L = ctypes.CDLL(str(path))
        pp = ctypes.POINTER(_vp)
        L.tasxb_tcp4_loop.argtypes = [ctypes.c_int, ctypes.POINTER(Tcp4Args), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, pp, ctypes.c_int]
        L.tasxb_raw_loop.argtypes = [ctypes.POINTER(RawArgs), ctypes.c_int, ctypes.c_int, ctypes.c_int, pp,
                                     ctypes.c_int]
        L.tasxb_txseg_loop.argtypes = [ctypes.POINTER(TxSegArgs), ctypes.c_int, ctypes.c_int, ctypes.c_int, pp,
                                       ctypes.c_int]
        L.tasxb_flow_loop.argtypes = [ctypes.POINTER(FlowArgs), ctypes.c_int, ctypes.c_int, ctypes.c_int, pp,
                                      ctypes.c_int]
        L.tasxb_rx_loop.argtypes = [ctypes.c_int, ctypes.POINTER(RxArgs), ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, pp, ctypes.c_int]
        L.tasxb_flush_loop.argtypes = [ctypes.c_uint, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_double)]
        L.tasxb_fastpath_mt.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_double), _vp, ctypes.c_size_t]
        L.tasxb_txseg_server_mt.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_double)]
        L.tasxb_txseg_server_mt.restype = ctypes.c_int
        for f in (L.tasxb_tcp4_loop, L.tasxb_raw_loop, L.tasxb_txseg_loop, L.tasxb_flow_loop, L.tasxb_rx_loop,
                  L.tasxb_flush_loop, L.tasxb_fastpath_mt):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


class Loop:
    """run(first, K): K steps, batch (first + k) % R on stream (first + k) % S."""

    def __init__(self, kind: str, args: list, streams: list[int], which: int = 0, what: str = ""):
        cls = {"tcp4": Tcp4Args, "raw": RawArgs, "txseg": TxSegArgs, "flow": FlowArgs, "rx": RxArgs}[kind]
        self.arr = (cls * len(args))(*args)
        self.streams = (_vp * len(streams))(*streams)
        self.R, self.S, self.which, self.kind = len(args), len(streams), which, kind
        self.what = what or kind
        L = lib()
        self.fn = {"tcp4": L.tasxb_tcp4_loop, "raw": L.tasxb_raw_loop, "txseg": L.tasxb_txseg_loop,
                   "flow": L.tasxb_flow_loop, "rx": L.tasxb_rx_loop}[kind]

    def __call__(self, first: int, K: int) -> None:
        if K <= 0:
            return
        if self.kind in ("tcp4", "rx"):
            rc = self.fn(self.which, self.arr, self.R, first, K, self.streams, self.S)
        else:
            rc = self.fn(self.arr, self.R, first, K, self.streams, self.S)
        if rc:
            raise xsum.TasxError(rc, self.what)


def flush_loop(ctx: int, base: int, stride: int, n: int, iters: int):
    """`iters` synchronous tx_flush rounds of n deferred frames from C
    (tasxb_flush_loop): the fast-path core's microseconds per flush."""
    import numpy as np
    us = np.zeros(iters, np.float64)
    rc = lib().tasxb_flush_loop(ctx, base, stride, n, iters, us.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc:
        raise xsum.TasxError(rc, "tasxb_flush_loop")
    return us


MT_MODES = {"per_context": 0, "feeder": 1, "server": 2}


def fastpath_mt(device: int, ctx0: int, threads: int, inflight: int, flushes: int, mode: str,
                keep: "np.ndarray | None" = None) -> dict:
    """`threads` fast-path threads at TAS's batch size, each on its own context
    (ctx0 + k), 32-frame tx_flush batches with up to `inflight` out
    (tasxb_fastpath_mt): frames/s, median latencies, median core time per
    flush.  keep: a uint8 array that receives thread 0's mempool afterwards."""
    import numpy as np
    out = np.zeros(4, np.float64)
    rc = lib().tasxb_fastpath_mt(device, ctx0, threads, inflight, flushes, MT_MODES[mode],
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                 None if keep is None else keep.ctypes.data, 0 if keep is None else keep.nbytes)
    if rc:
        raise xsum.TasxError(rc, "tasxb_fastpath_mt")
    return {"frames_per_s": float(out[0]), "latency_us": round(float(out[1]), 2),
            "latency_from_submit_us": round(float(out[2]), 2), "core_us_per_flush": round(float(out[3]), 3)}


def txseg_server_mt(device: int, ctx0: int, threads: int, inflight: int, flushes: int) -> dict:
    """The fused TX segment build through the flush server from `threads`
    fast-path threads, 32 segments (1448-B payloads) per flush
    (tasxb_txseg_server_mt): segments/s, median latency and core time."""
    import numpy as np
    out = np.zeros(4, np.float64)
    rc = lib().tasxb_txseg_server_mt(device, ctx0, threads, inflight, flushes,
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc:
        raise xsum.TasxError(rc, "tasxb_txseg_server_mt")
    return {"segments_per_s": round(float(out[0])), "latency_us": round(float(out[1]), 2),
            "core_us_per_flush": round(float(out[3]), 3)}
