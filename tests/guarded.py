"""Device buffers with unmapped guard pages on both sides (test infrastructure).

A `Guarded` buffer reserves a virtual range of (guard + mapped + guard) bytes
with HIP's virtual memory API (hipMemAddressReserve / hipMemCreate /
hipMemMap / hipMemSetAccess) and maps only the middle.  The data is placed
flush against the end of the mapping (`at="end"`) or its start (`at="start"`),
so a kernel that reads or writes even one byte past the data's last (first)
page faults instead of touching a neighbour: tests/test_guard_pages.py runs
the product kernels over such buffers to show that their accesses stay inside
the bounds include/tasx_xsum.h promises (round 6, VERDICT r05 item 1: a GPU
fault that could not be attributed from its record).  Nothing here is used by
the product.
"""
from __future__ import annotations

import ctypes

import numpy as np

_HIP = None


class _Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class _Flags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class _Prop(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", _Loc),
                ("win32HandleMetaData", ctypes.c_void_p), ("allocFlags", _Flags)]


class _Access(ctypes.Structure):
    _fields_ = [("location", _Loc), ("flags", ctypes.c_int)]


def hip():
    global _HIP
    if _HIP is None:
        import torch  # noqa: F401  (loads the HIP runtime torch uses: one runtime per process)
        h = ctypes.CDLL("libamdhip64.so")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        for name, args in {
            "hipMemGetAllocationGranularity": [ctypes.POINTER(sz), ctypes.POINTER(_Prop), ctypes.c_int],
            "hipMemAddressReserve": [ctypes.POINTER(vp), sz, sz, vp, ctypes.c_ulonglong],
            "hipMemCreate": [ctypes.POINTER(vp), sz, ctypes.POINTER(_Prop), ctypes.c_ulonglong],
            "hipMemMap": [vp, sz, sz, vp, ctypes.c_ulonglong],
            "hipMemSetAccess": [vp, sz, ctypes.POINTER(_Access), sz],
            "hipMemUnmap": [vp, sz],
            "hipMemRelease": [vp],
            "hipMemAddressFree": [vp, sz],
            "hipDeviceSynchronize": [],
        }.items():
            f = getattr(h, name)
            f.argtypes, f.restype = args, ctypes.c_int
        _HIP = h
    return _HIP


class _Cai:
    """A device range as __cuda_array_interface__ (torch.as_tensor wraps it
    without a copy)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


def _view(ptr: int, nbytes: int, device: int):
    import torch
    return torch.as_tensor(_Cai(ptr, nbytes), device=f"cuda:{device}")


_PARKED = []  # (va, total, map_base, mapped, handle) of every freed buffer: see Guarded.free


def _ok(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


class Guarded:
    """`nbytes` of device memory with an unmapped guard range on both sides."""

    def __init__(self, nbytes: int, at: str = "end", device: int = 0):
        assert at in ("start", "end") and nbytes > 0
        h = hip()
        # Uncached physical memory (hipMemAllocationTypeUncached): the XCDs'
        # L2s do not keep lines of it, so what one kernel (or copy) wrote is
        # what the next one reads on every XCD.  Cached VMM memory (type
        # Pinned) was not kept coherent across XCDs between kernels here: data
        # moved in by a copy read back wrong on another XCD (r06a, r06b, r06i
        # in profiles/r06/INDEX.md), a harness problem, not the kernels'.
        prop = _Prop(type=0x40000000, requestedHandleType=0, location=_Loc(1, device))
        g = ctypes.c_size_t(0)
        _ok(h.hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(prop), 0), "granularity")
        self.gran = g.value
        self.mapped = (nbytes + self.gran - 1) // self.gran * self.gran
        self.total = self.mapped + 2 * self.gran
        va = ctypes.c_void_p(0)
        _ok(h.hipMemAddressReserve(ctypes.byref(va), self.total, self.gran, None, 0), "hipMemAddressReserve")
        self.va = va.value
        self.handle = ctypes.c_void_p(0)
        _ok(h.hipMemCreate(ctypes.byref(self.handle), self.mapped, ctypes.byref(prop), 0), "hipMemCreate (uncached)")
        self.map_base = self.va + self.gran
        _ok(h.hipMemMap(self.map_base, self.mapped, 0, self.handle, 0), "hipMemMap")
        acc = _Access(location=_Loc(1, device), flags=3)
        _ok(h.hipMemSetAccess(self.map_base, self.mapped, ctypes.byref(acc), 1), "hipMemSetAccess")
        self.nbytes = nbytes
        # the data: flush against the mapping's end or its start
        self.addr = self.map_base + (self.mapped - nbytes if at == "end" else 0)
        # Data moves in and out by device kernels through torch views of the
        # mapping
        self._all = _view(self.map_base, self.mapped, device)
        self._all.zero_()
        self.data = self._all[self.addr - self.map_base:self.addr - self.map_base + nbytes]

    def upload(self, a: np.ndarray, offset: int = 0) -> None:
        import torch
        a = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        assert offset + a.nbytes <= self.nbytes
        # (the host-to-device copy of a whole buffer whose size is a multiple
        # of 16; the odd-sized part moves device to device)
        h = np.zeros((a.nbytes + 15) // 16 * 16, np.uint8)
        h[:a.nbytes] = a
        self.data[offset:offset + a.nbytes].copy_(torch.from_numpy(h).cuda()[:a.nbytes])
        torch.cuda.synchronize()
        # the data as the kernels will see it (a mismatch later is theirs)
        assert np.array_equal(self.download()[offset:offset + a.nbytes], a), "upload into the guarded mapping"

    def download(self) -> np.ndarray:
        import torch
        torch.cuda.synchronize()
        pad = torch.zeros((self.nbytes + 15) // 16 * 16, dtype=torch.uint8, device=self.data.device)
        pad[:self.nbytes].copy_(self.data)
        out = pad.cpu().numpy()[:self.nbytes]
        torch.cuda.synchronize()
        return out

    def free(self) -> None:
        # The mapping is kept (parked until the process exits), never unmapped
        # and reserved again: a range unmapped and handed to the next buffer
        # at the same virtual address was read stale by a later kernel on
        # this stack (r06j: 9 of 70 sums wrong with every upload verified), so
        # every guarded buffer of a session lives at an address of its own.
        if self.va:
            self.data = self._all = None
            _PARKED.append((self.va, self.total, self.map_base, self.mapped, self.handle))
            self.va = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()
