"""The fused TX segment build from host memory, by the kind of host pages it
reads and writes (round 6): TAS's `tas_shm` is hugepage-backed by default
(`fp_hugepages = 1`, /root/reference/tas/config.c:591; tas/shm.c:51-64) and
DPDK's mbuf pools live in hugepages, while the bench's `e2e.tx_segment_host`
leg uses hipHostMalloc memory.  For each kind -- hipHostMalloc, plain 4 KiB
pages pinned by hipHostRegister, transparent huge pages (madvise
MADV_HUGEPAGE on a 2 MiB-aligned anonymous mapping) pinned by hipHostRegister
-- it times the bench's 64K-segment build (same segments and frames; by HIP
events and by the host's clock) and the
plain streaming copy of the same bytes between two buffers of that kind, and
checks the frames built against the hipHostMalloc run's.

    python tools/host_pages_probe.py [--reps 20]   # one JSON line per kind
"""
from __future__ import annotations

import argparse
import ctypes
import json
import mmap
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from tas_amd import pktgen, xsum  # noqa: E402

HUGE = 2 << 20


def thp_mode() -> str:
    try:
        return Path("/sys/kernel/mm/transparent_hugepage/enabled").read_text().strip()
    except OSError:
        return "unknown"


def anon_huge_kib() -> int:
    for line in Path("/proc/self/smaps_rollup").read_text().splitlines():
        if line.startswith("AnonHugePages:"):
            return int(line.split()[1])
    return -1


class HostBuf:
    """`nbytes` of host memory of one kind, with its device address."""

    def __init__(self, nbytes: int, kind: str):
        self.kind, self.nbytes, self._pb, self._mm = kind, nbytes, None, None
        if kind == "hostmalloc":
            self._pb = xsum.PinnedBuffer(nbytes)
            self.array, self.addr, self.dev_addr = self._pb.array, self._pb.addr, self._pb.dev_addr
            return
        size = (nbytes + HUGE - 1) // HUGE * HUGE
        self._mm = mmap.mmap(-1, size + HUGE, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        base = ctypes.addressof(ctypes.c_char.from_buffer(self._mm))
        off = (-base) % HUGE
        if kind == "thp":
            self._mm.madvise(mmap.MADV_HUGEPAGE, off, size)
        else:
            self._mm.madvise(mmap.MADV_NOHUGEPAGE)
        self.array = np.frombuffer(self._mm, dtype=np.uint8, count=nbytes, offset=off)
        self.array[:] = 0  # fault every page in (huge ones where THP allows)
        self.addr = base + off
        rc = xsum.lib().tasx_host_register(ctypes.c_void_p(self.addr), ctypes.c_size_t(size))
        if rc:
            raise xsum.TasxError(rc, "tasx_host_register")
        self.dev_addr = xsum.lib().tasx_host_device_pointer(ctypes.c_void_p(self.addr))
        if not self.dev_addr:
            raise xsum.TasxError(-5, "tasx_host_device_pointer")

    def free(self):
        if self._pb is not None:
            self._pb.free()
        elif self._mm is not None:
            torch.cuda.synchronize()
            xsum.lib().tasx_host_unregister(ctypes.c_void_p(self.addr))
            self.array = None
            self._mm.close()
        self._pb = self._mm = None


def events_us(fn, reps: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--kinds", default="hostmalloc,pages4k,thp")
    a = ap.parse_args()
    n, stride = bench.N_FRAMES, bench.STRIDE
    _, _, segs, shm_len = pktgen.tx_segments(n, seed=pktgen.SEED + 2000, nflows=8192, tx_len=16384,
                                             make_shm=False, room=stride)
    shm0 = bench.device_random(shm_len, pktgen.SEED + 7).cpu().numpy()
    fr0 = bench.device_tcp4_frames(n, stride, bench.IP_TOTAL, pktgen.SEED).cpu().numpy()
    ab = xsum._load(xsum.AB_LIB_PATH)
    st = torch.cuda.current_stream().cuda_stream
    ref = None
    print(json.dumps({"thp": thp_mode(), "anon_huge_kib_before": anon_huge_kib()}), flush=True)
    for kind in a.kinds.split(","):
        bufs = []
        try:
            hs = HostBuf(shm_len, kind)
            bufs.append(hs)
            hf = HostBuf(n * stride, kind)
            bufs.append(hf)
            hd = HostBuf(segs.nbytes, kind)
            bufs.append(hd)
            hs.array[:] = shm0
            hf.array[:] = fr0
            hd.array[:] = segs.view(np.uint8)
            out = torch.empty(n, dtype=torch.int32, device="cuda")

            def build():
                xsum.tx_segment_batch(hs.dev_addr, hf.dev_addr, hd.dev_addr, n, shm_len=shm_len, out=out)
            build()
            torch.cuda.synchronize()
            got = hf.array.copy()
            same = None if ref is None else bool(np.array_equal(got, ref))
            ref = got if ref is None else ref
            us = events_us(build, a.reps)
            # the same launches by the host's clock (what e2e.tx_segment_host
            # reports), then by the host's clock with the device synchronized
            # through the stream only
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                build()
            torch.cuda.synchronize()
            wall_us = (time.perf_counter() - t0) * 1e6 / a.reps
            t0 = time.perf_counter()
            for _ in range(a.reps):
                build()
            torch.cuda.current_stream().synchronize()
            wall_stream_us = (time.perf_counter() - t0) * 1e6 / a.reps
            h2d = n * (pktgen.TCP_MSS + pktgen.HDRS_LEN + 32)
            cb = h2d // 16 * 16
            c1 = HostBuf(cb, kind)
            bufs.append(c1)
            c2 = HostBuf(cb, kind)
            bufs.append(c2)
            c1.array[:] = 1

            def copy():
                rc = ab.tasx_ab_stream_copy(c1.dev_addr, c2.dev_addr, cb, st)
                if rc:
                    raise xsum.TasxError(rc, "tasx_ab_stream_copy")
            cus = events_us(copy, a.reps)
            print(json.dumps({"kind": kind, "anon_huge_kib": anon_huge_kib(), "build_us": round(us, 1),
                              "build_wall_us": round(wall_us, 1), "build_wall_stream_us": round(wall_stream_us, 1),
                              "segments_per_s": round(n / us * 1e6), "copy_us": round(cus, 1),
                              "copy_GBps_each_way": round(cb / cus / 1e3, 1),
                              "build_frac_of_copy": round(cus / us, 3), "frames_match_hostmalloc": same,
                              "kernel": xsum.last_kernel()}), flush=True)
        finally:
            for b in bufs:
                b.free()


if __name__ == "__main__":
    main()
