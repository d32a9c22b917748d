"""TEST INFRASTRUCTURE ONLY -- ctypes view of oracle/build/liboracle.so (the C
restatement in oracle/tasx_oracle.c).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker or the
reported CPU baseline; never by the product (tas_amd/).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"

_u8p = ctypes.c_void_p


def build(out_dir: Path | None = None, march: str | None = None) -> Path:
    cmd = ["make", "-s", "-C", str(HERE)]
    if out_dir is not None:
        cmd.append(f"OUT={out_dir}")
    if march is not None:
        cmd.append(f"MARCH={march}")
    subprocess.run(cmd, check=True)
    return (out_dir or (HERE / "build")) / "liboracle.so"


class Oracle:
    def __init__(self, path: Path | None = None):
        path = Path(path or LIB)
        if not path.exists():
            build()
        L = ctypes.CDLL(str(path))
        sig = {
            "oracle_raw_cksum": (ctypes.c_uint16, [_u8p, ctypes.c_size_t]),
            "oracle_raw_cksum_acc": (ctypes.c_uint32, [_u8p, ctypes.c_size_t, ctypes.c_uint32]),
            "oracle_raw_cksum_reduce": (ctypes.c_uint16, [ctypes.c_uint32]),
            "oracle_ipv4_cksum": (ctypes.c_uint16, [_u8p]),
            "oracle_ipv4_phdr_cksum": (ctypes.c_uint16, [_u8p, ctypes.c_uint64]),
            "oracle_ipv4_udptcp_cksum": (ctypes.c_uint16, [_u8p, _u8p]),
            "oracle_tcp_checksums": (None, [_u8p, _u8p]),
            "oracle_ip_phdr_xsum": (ctypes.c_uint16, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint16]),
            "oracle_raw_batch": (None, [_u8p, _u8p, _u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t, _u8p]),
            "oracle_tcp4_batch": (None, [_u8p, _u8p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_int]),
            "oracle_ipv4_hdr_verify": (ctypes.c_int, [_u8p]),
            "oracle_ipv4_udptcp_cksum_verify": (ctypes.c_int, [_u8p, _u8p]),
            "oracle_tcp4_verify_batch": (None, [_u8p, _u8p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                                                ctypes.c_uint32, _u8p]),
            "oracle_tcp4_verify_batch_bounded": (None, [_u8p, _u8p, ctypes.c_uint64, ctypes.c_size_t,
                                                        ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32,
                                                        _u8p]),
            "oracle_tx_segment_batch": (None, [_u8p, ctypes.c_uint64, _u8p, _u8p, ctypes.c_size_t,
                                               ctypes.c_uint32, ctypes.c_uint32, _u8p]),
            "oracle_bench_tx_segment": (ctypes.c_double, [_u8p, ctypes.c_uint64, _u8p, _u8p, ctypes.c_size_t,
                                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                                          ctypes.c_int]),
            "oracle_crc32c_u32": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
            "oracle_crc32c_u64": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32]),
            "oracle_flow_hash": (ctypes.c_uint32, [_u8p, _u8p]),
            "oracle_flow_lookup_batch": (None, [_u8p, _u8p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                                                ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.c_uint32, _u8p, _u8p]),
            "oracle_bench_flow_lookup": (ctypes.c_double, [_u8p, _u8p, ctypes.c_uint64, ctypes.c_size_t,
                                                           ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32,
                                                           _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                           _u8p, ctypes.c_int, ctypes.c_int]),
            "oracle_bench": (ctypes.c_double, [ctypes.c_int, _u8p, _u8p, _u8p, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_int, ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        self.L = L
        self.path = path

    # -- per-call helpers on bytes-like objects --------------------------------
    @staticmethod
    def _buf(b):
        if isinstance(b, np.ndarray):
            assert b.flags.c_contiguous
            return b, b.ctypes.data
        arr = (ctypes.c_uint8 * len(b)).from_buffer(b) if isinstance(b, bytearray) else \
            (ctypes.c_uint8 * len(b)).from_buffer_copy(b)
        return arr, ctypes.addressof(arr)

    def raw_cksum(self, b) -> int:
        keep, p = self._buf(b)
        return self.L.oracle_raw_cksum(p, len(b))

    def ipv4_cksum(self, ip) -> int:
        keep, p = self._buf(ip)
        return self.L.oracle_ipv4_cksum(p)

    def ipv4_phdr_cksum(self, ip, ol_flags: int = 0) -> int:
        keep, p = self._buf(ip)
        return self.L.oracle_ipv4_phdr_cksum(p, ol_flags)

    def ipv4_udptcp_cksum(self, ip, l4) -> int:
        k1, p1 = self._buf(ip)
        k2, p2 = self._buf(l4)
        return self.L.oracle_ipv4_udptcp_cksum(p1, p2)

    def tcp_checksums(self, frame: bytearray, ip_off: int = 14, l4_off: int = 34) -> tuple[int, int]:
        keep, p = self._buf(frame)
        self.L.oracle_tcp_checksums(p + ip_off, p + l4_off)
        return (int.from_bytes(frame[ip_off + 10: ip_off + 12], "little"),
                int.from_bytes(frame[l4_off + 16: l4_off + 18], "little"))

    def ip_phdr_xsum(self, src_be: int, dst_be: int, proto: int, l3_paylen: int) -> int:
        return self.L.oracle_ip_phdr_xsum(src_be, dst_be, proto, l3_paylen)

    # -- batches over numpy buffers -------------------------------------------
    def raw_batch(self, buf: np.ndarray, n: int, offsets=None, lengths=None, stride: int = 0,
                  len0: int = 0) -> np.ndarray:
        out = np.empty(n, np.uint16)
        o = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        ln = None if lengths is None else np.ascontiguousarray(lengths, np.uint32)
        self.L.oracle_raw_batch(buf.ctypes.data, None if o is None else o.ctypes.data,
                                None if ln is None else ln.ctypes.data, stride, len0, n,
                                out.ctypes.data)
        return out

    def tcp4_batch(self, buf: np.ndarray, n: int, offsets=None, stride: int = 0, ip_off: int = 14,
                   l4_off: int = 34, inplace: bool = False) -> np.ndarray:
        out = np.empty(2 * n, np.uint16)
        o = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        self.L.oracle_tcp4_batch(buf.ctypes.data, None if o is None else o.ctypes.data, stride, n,
                                 ip_off, l4_off, out.ctypes.data, 1 if inplace else 0)
        return out

    def tcp4_verify_batch(self, buf: np.ndarray, n: int, offsets=None, stride: int = 0, ip_off: int = 14,
                          l4_off: int = 34) -> np.ndarray:
        out = np.empty(n, np.uint8)
        o = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        self.L.oracle_tcp4_verify_batch(buf.ctypes.data, None if o is None else o.ctypes.data, stride, n,
                                        ip_off, l4_off, out.ctypes.data)
        return out

    def tcp4_verify_batch_bounded(self, buf: np.ndarray, n: int, bounds, offsets=None, stride: int = 0,
                                  ip_off: int = 14, l4_off: int = 34) -> np.ndarray:
        """RX verification with per-frame read bounds (an int for all frames, or
        an array; bytes from the frame start, 0 = none)."""
        out = np.empty(n, np.uint8)
        o = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        if isinstance(bounds, (int, np.integer)):
            b, b0 = None, int(bounds)
        else:
            b, b0 = np.ascontiguousarray(bounds, np.uint32), 0
        self.L.oracle_tcp4_verify_batch_bounded(buf.ctypes.data, None if o is None else o.ctypes.data, stride, n,
                                                ip_off, l4_off, None if b is None else b.ctypes.data, b0,
                                                out.ctypes.data)
        return out

    def tx_segment_batch(self, shm: np.ndarray, shm_len: int, frames: np.ndarray, segs: np.ndarray,
                         ip_off: int = 14, l4_off: int = 34) -> np.ndarray:
        """In place on `frames`; returns ip.chksum | tcp.chksum << 16 (0 = rejected)."""
        assert frames.flags.c_contiguous and segs.flags.c_contiguous and segs.dtype.itemsize == 32
        out = np.zeros(len(segs), np.uint32)
        self.L.oracle_tx_segment_batch(shm.ctypes.data, shm_len, frames.ctypes.data, segs.ctypes.data,
                                       len(segs), ip_off, l4_off, out.ctypes.data)
        return out

    def bench_tx_segment(self, shm: np.ndarray, shm_len: int, frames: np.ndarray, segs: np.ndarray,
                         ip_off: int = 14, l4_off: int = 34, threads: int = 1, reps: int = 5) -> float:
        return self.L.oracle_bench_tx_segment(shm.ctypes.data, shm_len, frames.ctypes.data, segs.ctypes.data,
                                              len(segs), ip_off, l4_off, threads, reps)

    def flow_lookup_batch(self, buf: np.ndarray, n: int, flowht: np.ndarray, flowst: np.ndarray, *,
                          fs_num: int, offsets=None, stride: int = 0, ip_off: int = 14, l4_off: int = 34,
                          fs_stride: int = 128, fs_key_off: int = 32):
        """Returns (hashes u32, flow ids u32; 0xffffffff = no flow)."""
        ht = np.ascontiguousarray(flowht, np.uint32)
        fs = np.ascontiguousarray(flowst, np.uint8)
        h = np.empty(n, np.uint32)
        fid = np.empty(n, np.uint32)
        o = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        self.L.oracle_flow_lookup_batch(buf.ctypes.data, None if o is None else o.ctypes.data, stride, n, ip_off,
                                        l4_off, ht.ctypes.data, ht.size // 2, fs.ctypes.data, fs_num, fs_stride,
                                        fs_key_off, h.ctypes.data, fid.ctypes.data)
        return h, fid

    def bench_flow_lookup(self, buf: np.ndarray, n: int, flowht: np.ndarray, flowst: np.ndarray, *, fs_num: int,
                          stride: int, ip_off: int = 14, l4_off: int = 34, fs_stride: int = 128,
                          fs_key_off: int = 32, threads: int = 1, reps: int = 5) -> float:
        ht = np.ascontiguousarray(flowht, np.uint32)
        fs = np.ascontiguousarray(flowst, np.uint8)
        fid = np.empty(n, np.uint32)
        return self.L.oracle_bench_flow_lookup(buf.ctypes.data, None, stride, n, ip_off, l4_off, ht.ctypes.data,
                                               ht.size // 2, fs.ctypes.data, fs_num, fs_stride, fs_key_off,
                                               fid.ctypes.data, threads, reps)

    def bench(self, mode: int, buf: np.ndarray, n: int, *, offsets=None, lengths=None, stride=0,
              len0=0, ip_off=14, l4_off=34, threads=1, reps=5) -> float:
        out = np.empty(max(n, 1), np.uint16)
        o = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        ln = None if lengths is None else np.ascontiguousarray(lengths, np.uint32)
        return self.L.oracle_bench(mode, buf.ctypes.data, None if o is None else o.ctypes.data,
                                   None if ln is None else ln.ctypes.data, stride, len0, n,
                                   ip_off, l4_off, out.ctypes.data, threads, reps)
