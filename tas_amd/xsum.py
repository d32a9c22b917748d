"""Python host mirror of the checksum path's interface, over libtasx's C ABI.

Names follow the reference (/root/reference):

* ``tcp_checksums(ctx_id, frame)`` -- tcp_checksums() flag-off branch,
  tas/fast/fast_flows.c:1058-1069: records the frame; ``tx_flush(ctx_id)``
  (tas/fast/fastemu.c:544-566) checksums every recorded frame on the GPU and
  stores ip.chksum / tcp.chksum into it.
* ``fast_flows_kernelxsums(ctx_id, frame)`` -- tas/fast/fast_flows.c:1071-1076.
* ``raw_cksum_batch`` / ``tcp4_cksum_batch`` -- device-resident batches of
  rte_raw_cksum / (rte_ipv4_cksum, rte_ipv4_udptcp_cksum), the DPDK 19.11 calls
  the reference makes per frame.

PyTorch is plumbing here (device memory, streams); the checksum work is the HIP
kernels in libtasx.so.  There is no CPU fallback: if the library cannot be
loaded or a call fails, a ``TasxError`` is raised.
"""
from __future__ import annotations

import ctypes
import errno
import os
from pathlib import Path

import torch  # noqa: F401  -- must be imported first: libtasx then binds torch's HIP runtime

_LIB_DIR = Path(__file__).resolve().parent / "_lib"
# TASX_LIB: another in-tree build of the library (e.g. the comparison build
# tas_amd/_lib/libtasx_ab.so)
_LIB_PATH = Path(os.environ.get("TASX_LIB") or _LIB_DIR / "libtasx.so")
AB_LIB_PATH = _LIB_DIR / "libtasx_ab.so"
_lib = None
_loaded: dict = {}

TASX_F_INPLACE = 0x1
TASX_F_ZEROCOPY = 0x2  # host batches over offsets: the GPU reads the packets in place
TXSEG_SCRATCH = 0x80000000  # tasx_tx_seg.room flag: bytes past the frame are scratch
TAS_IP_OFF = 14
TAS_L4_OFF = 34
RAW_MAX_LEN = 131073
MAX_CTX = 16
CTX_SELF = 0xFFFFFFFF  # TASX_CTX_SELF: the calling thread's context (tasx_set_thread_ctx)

_c_int, _c_u16, _c_u32, _c_u64 = ctypes.c_int, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64
_vp, _sz, _uns = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint

# name -> (restype, argtypes); mirrors include/tasx_xsum.h
SIGNATURES = {
    "tasx_abi_version": (_c_int, []),
    "tasx_last_error": (ctypes.c_char_p, []),
    "tasx_device_count": (_c_int, []),
    "tasx_raw_cksum_batch_dev": (_c_int, [_vp, _vp, _c_u64, _vp, _c_u32, _c_u32, _vp, _vp]),
    "tasx_tcp4_cksum_batch_dev": (_c_int, [_vp, _vp, _c_u64, _c_u32, _c_u32, _c_u32, _vp, _c_u32, _vp]),
    "tasx_tcp4_cksum_batch_dev_hint": (_c_int, [_vp, _vp, _c_u64, _vp, _c_u32, _c_u32, _c_u32, _c_u32, _vp,
                                                _c_u32, _vp]),
    "tasx_tcp4_cksum_batch_dev_room": (_c_int, [_vp, _vp, _c_u64, _vp, _c_u32, _c_u32, _c_u32, _c_u32, _c_u32,
                                                _vp, _c_u32, _vp]),
    "tasx_tcp4_verify_batch_dev": (_c_int, [_vp, _vp, _c_u64, _c_u32, _c_u32, _c_u32, _vp, _vp]),
    "tasx_tcp4_verify_batch_dev_room": (_c_int, [_vp, _vp, _c_u64, _vp, _c_u32, _c_u32, _c_u32, _c_u32, _c_u32,
                                                 _vp, _vp]),
    "tasx_tcp4_verify_batch_dev_hint": (_c_int, [_vp, _vp, _c_u64, _vp, _c_u32, _c_u32, _c_u32, _c_u32, _vp,
                                                 _vp]),
    "tasx_flow_lookup_batch_dev": (_c_int, [_vp, _vp, _c_u64, _c_u32, _c_u32, _c_u32, _vp, _c_u32, _vp, _c_u32,
                                            _c_u32, _c_u32, _vp, _vp, _vp]),
    "tasx_rx_batch_dev": (_c_int, [_vp, _vp, _c_u64, _vp, _c_u32, _c_u32, _c_u32, _c_u32, _c_u32, _vp, _vp, _c_u32,
                                   _vp, _c_u32, _c_u32, _c_u32, _vp, _vp, _vp]),
    "tasx_tx_segment_batch_dev": (_c_int, [_vp, _c_u64, _vp, _vp, _c_u32, _c_u32, _c_u32, _vp, _vp]),
    "tasx_ctx_init": (_c_int, [_uns, _c_int, _sz]),
    "tasx_ctx_destroy": (_c_int, [_uns]),
    "tasx_tcp4_cksum_batch_host": (_c_int, [_uns, _vp, _c_u64, _c_u32, _c_u32, _c_u32, _vp, _c_u32]),
    "tasx_raw_cksum_batch_host": (_c_int, [_uns, _vp, _c_u64, _c_u32, _c_u32, _vp]),
    "tasx_tcp4_cksum_batch_host_offs": (_c_int, [_uns, _vp, _vp, _vp, _c_u32, _c_u32, _c_u32, _vp, _c_u32]),
    "tasx_raw_cksum_batch_host_offs": (_c_int, [_uns, _vp, _vp, _vp, _c_u32, _c_u32, _vp, _c_u32]),
    "tasx_set_thread_ctx": (_c_int, [_uns]),
    "tasx_thread_ctx": (_c_int, []),
    "tasx_tcp_checksums": (_c_int, [_uns, _vp, _vp, _c_u32, _c_u32, _c_u16]),
    "tasx_fast_flows_kernelxsums": (_c_int, [_uns, _vp, _vp]),
    "tasx_defer_tcp4": (_c_int, [_uns, _vp, _c_u16, _c_u16]),
    "tasx_pending": (_c_int, [_uns]),
    "tasx_flush": (_c_int, [_uns]),
    "tasx_flush_submit": (_c_int, [_uns, ctypes.POINTER(_c_u32)]),
    "tasx_flush_poll": (_c_int, [_uns, _c_u32]),
    "tasx_flush_wait": (_c_int, [_uns, _c_u32]),
    "tasx_ctx_register_frames": (_c_int, [_uns, _vp, _sz]),
    "tasx_ctx_stats": (_c_int, [_uns, ctypes.POINTER(_c_u32), ctypes.POINTER(_c_u32)]),
    "tasx_tcp4_offload_batch_dev": (_c_int, [_vp, _vp, _c_u64, _c_u32, _c_u32, _c_u32, _vp, _c_u32, _vp]),
    "tasx_feeder_start": (_c_int, [_c_int]),
    "tasx_feeder_stop": (_c_int, [_c_int]),
    "tasx_feeder_stats": (_c_int, [_c_int, ctypes.POINTER(_c_u64), ctypes.POINTER(_c_u64)]),
    "tasx_ctx_use_feeder": (_c_int, [_uns, _c_int]),
    "tasx_ctx_feeder_flushes": (_c_int, [_uns, ctypes.POINTER(_c_u32)]),
    "tasx_server_start": (_c_int, [_c_int]),
    "tasx_ctx_register_shm": (_c_int, [_uns, _vp, _sz]),
    "tasx_server_tx_segments": (_c_int, [_uns, _vp, _c_u32, ctypes.POINTER(ctypes.c_uint32)]),
    "tasx_server_stop": (_c_int, [_c_int]),
    "tasx_server_stats": (_c_int, [_c_int, ctypes.POINTER(_c_u64), ctypes.POINTER(_c_u64)]),
    "tasx_server_epochs": (_c_int, [_c_int, ctypes.POINTER(_c_u64), ctypes.POINTER(_c_u32), ctypes.POINTER(_c_u32)]),
    "tasx_ctx_use_server": (_c_int, [_uns, _c_int]),
    "tasx_ctx_server_flushes": (_c_int, [_uns, ctypes.POINTER(_c_u32)]),
    "tasx_take_unfinished": (_c_int, [_uns, _vp, _c_u32]),
    "tasx_take_unfinished_segs": (_c_int, [_uns, _vp, _c_u32]),
    "tasx_server_abort": (_c_int, [_c_int]),
    "tasx_server_pause": (_c_int, [_c_int]),
    "tasx_server_resume": (_c_int, [_c_int]),
    "tasx_set_kernel_variant": (_c_int, [_c_int]),
    "tasx_last_kernel": (ctypes.c_char_p, []),
    "tasx_host_alloc": (_vp, [_sz]),
    "tasx_host_free": (_c_int, [_vp]),
    "tasx_host_register": (_c_int, [_vp, _sz]),
    "tasx_host_device_pointer": (_vp, [_vp]),
    "tasx_host_unregister": (_c_int, [_vp]),
    "tasx_dev_alloc": (_vp, [_c_int, _sz]),
    "tasx_dev_free": (_c_int, [_vp]),
    "tasx_memcpy_h2d": (_c_int, [_vp, _vp, _sz]),
    "tasx_memcpy_d2h": (_c_int, [_vp, _vp, _sz]),
    "tasx_stream_sync": (_c_int, [_vp]),
}


# the comparison build only (include/tasx_ab.h)
AB_SIGNATURES = {
    "tasx_ab_flow_pattern": (_c_int, [_vp, _c_u64, _c_u32, _c_u32, _vp, _c_u32, _vp, _c_u32, _c_u32, _c_u32, _vp,
                                      _vp]),
    "tasx_ab_tcp4_pattern": (_c_int, [_vp, _c_u64, _c_u32, _c_u32, _c_u32, _vp, _vp]),
    "tasx_ab_tcp4_mix_pattern": (_c_int, [_vp, _c_u64, _c_u32, _vp, _c_u32, _c_int, _vp, _vp]),
    "tasx_ab_stream_copy": (_c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "tasx_ab_stream_read": (_c_int, [_vp, ctypes.c_size_t, _c_int, _vp, _vp]),
    "tasx_ab_tx_segment_form": (_c_int, [_c_int, _vp, _c_u64, _vp, _vp, _c_u32, _c_u32, _c_u32, _vp, _vp]),
    "tasx_ab_ctx_set_tickets": (_c_int, [_uns, _c_u32]),
}


class TasxError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        name = errno.errorcode.get(-code, str(code))
        super().__init__(f"{what}: {name} ({last_error()})")


def library_path() -> Path:
    return _LIB_PATH


def _load(path: Path) -> ctypes.CDLL:
    path = Path(path)
    if path in _loaded:
        return _loaded[path]
    if not path.exists():
        raise RuntimeError(
            f"{path.name} not built ({path}); run python -c 'import __graft_entry__ as g; g.build()'")
    L = ctypes.CDLL(str(path), mode=os.RTLD_NOW | ctypes.RTLD_LOCAL)
    for name, (res, args) in {**SIGNATURES, **AB_SIGNATURES}.items():
        fn = getattr(L, name, None)
        if fn is None:
            if name in SIGNATURES:
                raise RuntimeError(f"{path} does not export {name}")
            continue
        fn.restype = res
        fn.argtypes = args
    _loaded[path] = L
    return L


def lib() -> ctypes.CDLL:
    """Load libtasx.so (built in-tree by tas_amd.build / __graft_entry__.build)."""
    global _lib
    if _lib is None:
        _lib = _load(_LIB_PATH)
    return _lib


class using_library:
    """Route this module's calls through another build of the library for the
    duration of a with-block (``with xsum.using_library(xsum.AB_LIB_PATH):
    ...``: the comparison build behaves as the product).  Both builds are
    linked -Bsymbolic and loaded RTLD_LOCAL, so they coexist in one process."""

    def __init__(self, path):
        self.path = Path(path)

    def __enter__(self):
        global _lib
        lib()
        self.prev = _lib
        _lib = _load(self.path)
        return _lib

    def __exit__(self, *exc):
        global _lib
        _lib = self.prev
        return False


def last_kernel() -> str:
    """Name of the kernel this thread's last batch call launched."""
    s = lib().tasx_last_kernel()
    return s.decode() if s else ""


def last_error() -> str:
    if _lib is None:
        return ""
    s = _lib.tasx_last_error()
    return s.decode() if s else ""


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise TasxError(rc, what)
    return rc


def _ptr(t) -> int | None:
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


# ---------------------------------------------------------------------------
# device-resident batches

def raw_cksum_batch(buf: torch.Tensor, n: int, *, offsets: torch.Tensor | None = None,
                    lengths: torch.Tensor | None = None, stride: int = 0, len0: int = 0,
                    out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """out[i] = rte_raw_cksum(buf + off_i, len_i) on the GPU; int16 tensor holding
    the uint16 results (view as uint16 on the host)."""
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=buf.device)
    if offsets is not None:
        assert offsets.dtype in (torch.int64,) and offsets.numel() >= n
    if lengths is not None:
        assert lengths.dtype == torch.int32 and lengths.numel() >= n
    assert out.numel() >= n and out.element_size() == 2
    _check(lib().tasx_raw_cksum_batch_dev(_ptr(buf), _ptr(offsets), stride, _ptr(lengths), len0,
                                          n, _ptr(out), _stream(stream)), "tasx_raw_cksum_batch_dev")
    return out


def tcp4_cksum_batch(frames: torch.Tensor, n: int, *, offsets: torch.Tensor | None = None,
                     stride: int = 0, ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF,
                     out: torch.Tensor | None = None, inplace: bool = False,
                     want_out: bool = True, frame_len: torch.Tensor | int | None = None,
                     room: int = 0, stream=None) -> torch.Tensor | None:
    """tcp_checksums() flag-off branch for n frames on the GPU.  Returns an int16
    tensor of 2n values: [ip.chksum, tcp.chksum] per frame (uint16 bit patterns).
    frame_len: optional frame-length hints (int32 tensor, or one int for all
    frames) -- prefetch only, results never depend on it.  room: bytes from
    each frame's start that may be read (the mbuf data room; 0 = unknown)."""
    if out is None and want_out:
        out = torch.empty(2 * n, dtype=torch.int16, device=frames.device)
    if offsets is not None:
        assert offsets.dtype == torch.int64 and offsets.numel() >= n
    flags = TASX_F_INPLACE if inplace else 0
    if frame_len is None and not room:
        _check(lib().tasx_tcp4_cksum_batch_dev(_ptr(frames), _ptr(offsets), stride, n, ip_off, l4_off,
                                               _ptr(out), flags, _stream(stream)),
               "tasx_tcp4_cksum_batch_dev")
    else:
        flen, flen0 = _hints(frame_len, n)
        if room:
            _check(lib().tasx_tcp4_cksum_batch_dev_room(_ptr(frames), _ptr(offsets), stride, _ptr(flen), flen0,
                                                        room, n, ip_off, l4_off, _ptr(out), flags,
                                                        _stream(stream)), "tasx_tcp4_cksum_batch_dev_room")
        else:
            _check(lib().tasx_tcp4_cksum_batch_dev_hint(_ptr(frames), _ptr(offsets), stride, _ptr(flen), flen0,
                                                        n, ip_off, l4_off, _ptr(out), flags, _stream(stream)),
                   "tasx_tcp4_cksum_batch_dev_hint")
    return out


def _hints(frame_len, n):
    if frame_len is None:
        return None, 0
    if isinstance(frame_len, int):
        return None, frame_len
    assert frame_len.dtype == torch.int32 and frame_len.numel() >= n
    return frame_len, 0


RX_IP_OK, RX_L4_OK, RX_IHL_NOT5 = 0x1, 0x2, 0x4


def tcp4_verify_batch(frames: torch.Tensor, n: int, *, offsets: torch.Tensor | None = None,
                      stride: int = 0, ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF,
                      out: torch.Tensor | None = None, frame_len: torch.Tensor | int | None = None,
                      room: int = 0, stream=None) -> torch.Tensor:
    """Receive-side checksum verification of n frames: uint8 flags per frame
    (RX_IP_OK | RX_L4_OK | RX_IHL_NOT5).  frame_len: optional received frame
    lengths (int32 tensor, or one int for all frames): the read bound and a
    prefetch hint.  room: the read bound of frames without a length."""
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=frames.device)
    if offsets is not None:
        assert offsets.dtype == torch.int64 and offsets.numel() >= n
    if frame_len is None and not room:
        _check(lib().tasx_tcp4_verify_batch_dev(_ptr(frames), _ptr(offsets), stride, n, ip_off, l4_off,
                                                _ptr(out), _stream(stream)), "tasx_tcp4_verify_batch_dev")
    else:
        flen, flen0 = _hints(frame_len, n)
        _check(lib().tasx_tcp4_verify_batch_dev_room(_ptr(frames), _ptr(offsets), stride, _ptr(flen), flen0,
                                                     room, n, ip_off, l4_off, _ptr(out), _stream(stream)),
               "tasx_tcp4_verify_batch_dev_room")
    return out


FLOW_NONE = 0xFFFFFFFF


def flow_lookup_batch(frames: torch.Tensor, n: int, flowht: torch.Tensor, flowst: torch.Tensor, fs_num: int, *,
                      offsets: torch.Tensor | None = None, stride: int = 0, ip_off: int = TAS_IP_OFF,
                      l4_off: int = TAS_L4_OFF, fs_stride: int = 128, fs_key_off: int = 32,
                      want_hash: bool = True, ht_entries: int | None = None, stream=None):
    """RX flow lookup (fast_flows_packet_fss, tas/fast/fast_flows.c:1084-1163):
    returns (hashes int32 or None, flow ids int32; FLOW_NONE = no flow).
    frames / flowht / flowst may be device addresses (ints); an int flowht
    needs ht_entries."""
    dev = frames.device if isinstance(frames, torch.Tensor) else "cuda"
    fid = torch.empty(n, dtype=torch.int32, device=dev)
    h = torch.empty(n, dtype=torch.int32, device=dev) if want_hash else None
    ent = ht_entries if ht_entries is not None else flowht.numel() * flowht.element_size() // 8
    _check(lib().tasx_flow_lookup_batch_dev(_ptr(frames), _ptr(offsets), stride, n, ip_off, l4_off, _ptr(flowht),
                                            ent, _ptr(flowst), fs_num, fs_stride, fs_key_off, _ptr(h), _ptr(fid),
                                            _stream(stream)), "tasx_flow_lookup_batch_dev")
    return h, fid


def rx_batch(frames: torch.Tensor, n: int, flowht: torch.Tensor, flowst: torch.Tensor, fs_num: int, *,
             offsets: torch.Tensor | None = None, stride: int = 0, ip_off: int = TAS_IP_OFF,
             l4_off: int = TAS_L4_OFF, frame_len: torch.Tensor | int | None = None, room: int = 0,
             fs_stride: int = 128, fs_key_off: int = 32, want_hash: bool = True, flags=None, fid=None, h=None,
             ht_entries: int | None = None, stream=None):
    """One RX pass: tcp4_verify_batch and flow_lookup_batch of the same frames
    (tasx_rx_batch_dev).  Returns (flags uint8, hashes int32 or None, flow
    ids int32)."""
    dev = frames.device if isinstance(frames, torch.Tensor) else "cuda"
    flags = torch.empty(n, dtype=torch.uint8, device=dev) if flags is None else flags
    fid = torch.empty(n, dtype=torch.int32, device=dev) if fid is None else fid
    if h is None and want_hash:
        h = torch.empty(n, dtype=torch.int32, device=dev)
    if offsets is not None:
        assert offsets.dtype == torch.int64 and offsets.numel() >= n
    flen, flen0 = _hints(frame_len, n) if frame_len is not None else (None, 0)
    ent = ht_entries if ht_entries is not None else flowht.numel() * flowht.element_size() // 8
    _check(lib().tasx_rx_batch_dev(_ptr(frames), _ptr(offsets), stride, _ptr(flen), flen0, room, n, ip_off, l4_off,
                                   _ptr(flags), _ptr(flowht), ent, _ptr(flowst), fs_num, fs_stride, fs_key_off,
                                   _ptr(h), _ptr(fid), _stream(stream)), "tasx_rx_batch_dev")
    return flags, h, fid


def tx_segment_batch(shm, frames, segs, n: int, *, shm_len: int | None = None,
                     ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF,
                     out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Fused TX segment build: flow_tx_read() of each segment's payload from the
    shared-memory TX buffers into its frame, then tcp_checksums() in place
    (tas/fast/fast_flows.c:930-936).  `segs` holds n 32-byte tasx_tx_seg
    descriptors (pktgen.TX_SEG_DTYPE bytes, 16-byte aligned on the device).
    shm, frames and segs are device tensors or device addresses (ints: e.g. a
    PinnedBuffer's dev_addr, the tas_shm region or mbuf pool mapped for the
    GPU); an int shm needs shm_len.  Returns int32 ip.chksum | tcp.chksum << 16
    per segment (0 = rejected)."""
    if isinstance(segs, torch.Tensor):
        assert segs.numel() * segs.element_size() >= 32 * n
    if shm_len is None:
        shm_len = shm.numel() * shm.element_size()
    if out is None:
        out = torch.empty(n, dtype=torch.int32,
                          device=frames.device if isinstance(frames, torch.Tensor) else "cuda")
    _check(lib().tasx_tx_segment_batch_dev(_ptr(shm), shm_len, _ptr(frames),
                                           _ptr(segs), n, ip_off, l4_off, _ptr(out), _stream(stream)),
           "tasx_tx_segment_batch_dev")
    return out


# ---------------------------------------------------------------------------
# contexts, deferred surface, end-to-end host batches

def ctx_init(ctx_id: int, device: int = 0, max_batch_bytes: int = 0) -> None:
    _check(lib().tasx_ctx_init(ctx_id, device, max_batch_bytes), "tasx_ctx_init")


def set_thread_ctx(ctx_id: int) -> None:
    """Bind ctx_id to the calling thread (calls may then pass CTX_SELF)."""
    _check(lib().tasx_set_thread_ctx(ctx_id), "tasx_set_thread_ctx")


def ctx_destroy(ctx_id: int) -> None:
    _check(lib().tasx_ctx_destroy(ctx_id), "tasx_ctx_destroy")


def tcp_checksums(ctx_id: int, frame_addr: int, nbh: int | None = None, ip_s: int = 0,
                  ip_d: int = 0, l3_paylen: int = 0) -> None:
    _check(lib().tasx_tcp_checksums(ctx_id, nbh, frame_addr, ip_s, ip_d, l3_paylen),
           "tasx_tcp_checksums")


def fast_flows_kernelxsums(ctx_id: int, frame_addr: int, nbh: int | None = None) -> None:
    _check(lib().tasx_fast_flows_kernelxsums(ctx_id, nbh, frame_addr), "tasx_fast_flows_kernelxsums")


def defer_tcp4(ctx_id: int, frame_addr: int, ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF) -> None:
    _check(lib().tasx_defer_tcp4(ctx_id, frame_addr, ip_off, l4_off), "tasx_defer_tcp4")


def pending(ctx_id: int) -> int:
    return _check(lib().tasx_pending(ctx_id), "tasx_pending")


def tx_flush(ctx_id: int) -> None:
    _check(lib().tasx_flush(ctx_id), "tasx_flush")


def flush_submit(ctx_id: int) -> int:
    """Launch every recorded frame's checksums; returns the flush ticket."""
    t = ctypes.c_uint32()
    _check(lib().tasx_flush_submit(ctx_id, ctypes.byref(t)), "tasx_flush_submit")
    return t.value


def flush_poll(ctx_id: int, ticket: int) -> bool:
    """True once flush `ticket` (and every earlier one) has stored its results."""
    return bool(_check(lib().tasx_flush_poll(ctx_id, ticket), "tasx_flush_poll"))


def flush_wait(ctx_id: int, ticket: int) -> None:
    _check(lib().tasx_flush_wait(ctx_id, ticket), "tasx_flush_wait")


def register_frames(ctx_id: int, base_addr: int, nbytes: int) -> None:
    """Zero-copy region for the context's frames (tasx_ctx_register_frames)."""
    _check(lib().tasx_ctx_register_frames(ctx_id, base_addr, nbytes), "tasx_ctx_register_frames")


def ctx_stats(ctx_id: int) -> tuple[int, int]:
    z, st = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().tasx_ctx_stats(ctx_id, ctypes.byref(z), ctypes.byref(st)), "tasx_ctx_stats")
    return z.value, st.value


def tcp4_offload_batch(frames: torch.Tensor, n: int, *, offsets: torch.Tensor | None = None, stride: int = 0,
                       ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF, inplace: bool = False,
                       want_out: bool = True, stream=None) -> torch.Tensor | None:
    """The offload branch of tcp_checksums (tasx_tcp4_offload_batch_dev):
    uint16 network_ip_phdr_xsum per frame, and/or stored in place with
    ip.chksum zeroed."""
    out = torch.empty(n, dtype=torch.int16, device=frames.device) if want_out else None
    if offsets is not None:
        assert offsets.dtype == torch.int64 and offsets.numel() >= n
    _check(lib().tasx_tcp4_offload_batch_dev(frames.data_ptr(), None if offsets is None else offsets.data_ptr(),
                                             stride, n, ip_off, l4_off, None if out is None else out.data_ptr(),
                                             TASX_F_INPLACE if inplace else 0, _stream(stream)),
           "tasx_tcp4_offload_batch_dev")
    return out


def feeder_start(device: int = 0) -> None:
    """The shared feeder thread for `device` (tasx_feeder_start)."""
    _check(lib().tasx_feeder_start(device), "tasx_feeder_start")


def feeder_stop(device: int = 0) -> None:
    _check(lib().tasx_feeder_stop(device), "tasx_feeder_stop")


def feeder_stats(device: int = 0) -> tuple[int, int]:
    sw, fr = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().tasx_feeder_stats(device, ctypes.byref(sw), ctypes.byref(fr)), "tasx_feeder_stats")
    return sw.value, fr.value


def use_feeder(ctx_id: int, on: bool = True) -> None:
    """Attach the context to (or detach it from) its GPU's feeder."""
    _check(lib().tasx_ctx_use_feeder(ctx_id, 1 if on else 0), "tasx_ctx_use_feeder")


def feeder_flushes(ctx_id: int) -> int:
    n = ctypes.c_uint32()
    _check(lib().tasx_ctx_feeder_flushes(ctx_id, ctypes.byref(n)), "tasx_ctx_feeder_flushes")
    return n.value


def server_start(device: int = 0) -> None:
    """The persistent flush-server kernel for `device` (tasx_server_start)."""
    _check(lib().tasx_server_start(device), "tasx_server_start")


def server_stop(device: int = 0) -> None:
    _check(lib().tasx_server_stop(device), "tasx_server_stop")


def server_stats(device: int = 0) -> tuple[int, int]:
    b, fr = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().tasx_server_stats(device, ctypes.byref(b), ctypes.byref(fr)), "tasx_server_stats")
    return b.value, fr.value


def server_epochs(device: int = 0) -> tuple[int, int, int]:
    """(epochs completed, the epoch thread's waits over 50 ms, the longest in ms)."""
    e, n, m = _c_u64(), _c_u32(), _c_u32()
    _check(lib().tasx_server_epochs(device, ctypes.byref(e), ctypes.byref(n), ctypes.byref(m)), "tasx_server_epochs")
    return e.value, n.value, m.value


def register_shm(ctx_id: int, base_addr: int, nbytes: int) -> None:
    """The app's shared-memory region, TX payload sources for
    server_tx_segments (tasx_ctx_register_shm)."""
    _check(lib().tasx_ctx_register_shm(ctx_id, base_addr, nbytes), "tasx_ctx_register_shm")


def server_tx_segments(ctx_id: int, segs) -> int:
    """Hand TX segments (pktgen.TX_SEG_DTYPE records: frame_off from the frame
    region's start, tx_base from the shm region's start) to the flush server
    (tasx_server_tx_segments); returns the ticket of the last one."""
    import numpy as np
    a = np.ascontiguousarray(segs)
    assert a.dtype.itemsize == 32
    t = ctypes.c_uint32()
    _check(lib().tasx_server_tx_segments(ctx_id, a.ctypes.data, len(a), ctypes.byref(t)), "tasx_server_tx_segments")
    return t.value


def use_server(ctx_id: int, on: bool = True) -> None:
    """Attach the context to (or detach it from) its GPU's flush server."""
    _check(lib().tasx_ctx_use_server(ctx_id, 1 if on else 0), "tasx_ctx_use_server")


def take_unfinished(ctx_id: int, chunk: int = 64) -> list[tuple[int, int]]:
    """Error recovery (ABI 8): every frame the GPU did not finish, as (ip, l4)
    host addresses, taken back from the context (tasx_take_unfinished; the
    first call settles it).  The caller finishes them on the CPU."""
    refs = (ctypes.c_void_p * (2 * chunk))()
    got: list[tuple[int, int]] = []
    while True:
        k = _check(lib().tasx_take_unfinished(ctx_id, refs, chunk), "tasx_take_unfinished")
        got += [(refs[2 * i] or 0, refs[2 * i + 1] or 0) for i in range(k)]
        if k < chunk:
            return got


def take_unfinished_segs(ctx_id: int, chunk: int = 64):
    """The TX segments (pktgen.TX_SEG_DTYPE records, as submitted) the flush
    server did not build (tasx_take_unfinished_segs; after take_unfinished)."""
    import numpy as np
    from . import pktgen
    out = []
    buf = np.zeros(chunk, pktgen.TX_SEG_DTYPE)
    while True:
        k = _check(lib().tasx_take_unfinished_segs(ctx_id, buf.ctypes.data, chunk), "tasx_take_unfinished_segs")
        out.append(buf[:k].copy())
        if k < chunk:
            return np.concatenate(out)


def server_abort(device: int = 0) -> None:
    """Stop the flush server's kernel with contexts still attached (ABI 8)."""
    _check(lib().tasx_server_abort(device), "tasx_server_abort")


def server_pause(device: int = 0) -> None:
    """Let HIP frees through without stopping the flush server (ABI 9): its
    kernel leaves at its rings' positions; contexts stay attached."""
    _check(lib().tasx_server_pause(device), "tasx_server_pause")


def server_resume(device: int = 0) -> None:
    """Launch a paused flush server's kernel again at its rings' positions."""
    _check(lib().tasx_server_resume(device), "tasx_server_resume")


def server_flushes(ctx_id: int) -> int:
    n = ctypes.c_uint32()
    _check(lib().tasx_ctx_server_flushes(ctx_id, ctypes.byref(n)), "tasx_ctx_server_flushes")
    return n.value


def tcp4_cksum_batch_host(ctx_id: int, base_addr: int, stride: int, n: int, out_addr: int | None,
                          ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF,
                          inplace: bool = False) -> None:
    flags = TASX_F_INPLACE if inplace else 0
    _check(lib().tasx_tcp4_cksum_batch_host(ctx_id, base_addr, stride, n, ip_off, l4_off,
                                            out_addr, flags), "tasx_tcp4_cksum_batch_host")


def raw_cksum_batch_host(ctx_id: int, base_addr: int, stride: int, len0: int, n: int,
                         out_addr: int) -> None:
    _check(lib().tasx_raw_cksum_batch_host(ctx_id, base_addr, stride, len0, n, out_addr),
           "tasx_raw_cksum_batch_host")


def _np_ptr(a, dtype):
    """Host address of a contiguous numpy array of `dtype` (None passes through)."""
    import numpy as np
    if a is None:
        return None
    assert isinstance(a, np.ndarray) and a.dtype == dtype and a.flags["C_CONTIGUOUS"], (a.dtype, dtype)
    return a.ctypes.data


def tcp4_cksum_batch_host_offs(ctx_id: int, base_addr: int | None, offsets, n: int, out=None, *,
                               frame_len=None, ip_off: int = TAS_IP_OFF, l4_off: int = TAS_L4_OFF,
                               inplace: bool = False, zerocopy: bool = False):
    """tcp_checksums() of n frames in host memory at base_addr + offsets[i]
    (numpy uint64; base_addr None: offsets are addresses), end to end
    (tasx_tcp4_cksum_batch_host_offs).  out: numpy uint16 array of 2n, or None
    to allocate (skipped with inplace and out=False).  frame_len: numpy uint32
    frame lengths (the mbuf data_len), optional.  zerocopy: the GPU reads the
    frames in place (base_addr pinned or registered)."""
    import numpy as np
    if out is None:
        out = np.empty(2 * n, dtype=np.uint16)
    elif out is False:
        out = None
    assert offsets.size >= n and (frame_len is None or frame_len.size >= n)
    assert out is None or out.size >= 2 * n
    flags = (TASX_F_INPLACE if inplace else 0) | (TASX_F_ZEROCOPY if zerocopy else 0)
    _check(lib().tasx_tcp4_cksum_batch_host_offs(ctx_id, base_addr, _np_ptr(offsets, np.uint64),
                                                 _np_ptr(frame_len, np.uint32), n, ip_off, l4_off,
                                                 _np_ptr(out, np.uint16), flags),
           "tasx_tcp4_cksum_batch_host_offs")
    return out


def raw_cksum_batch_host_offs(ctx_id: int, base_addr: int | None, offsets, n: int, *, lengths=None,
                              len0: int = 0, out=None, zerocopy: bool = False):
    """rte_raw_cksum of n packets in host memory at base_addr + offsets[i]
    (lengths[i], numpy uint32, or len0 for all), end to end
    (tasx_raw_cksum_batch_host_offs).  Returns numpy uint16."""
    import numpy as np
    if out is None:
        out = np.empty(n, dtype=np.uint16)
    assert offsets.size >= n and out.size >= n and (lengths is None or lengths.size >= n)
    _check(lib().tasx_raw_cksum_batch_host_offs(ctx_id, base_addr, _np_ptr(offsets, np.uint64),
                                                _np_ptr(lengths, np.uint32), len0, n, _np_ptr(out, np.uint16),
                                                TASX_F_ZEROCOPY if zerocopy else 0),
           "tasx_raw_cksum_batch_host_offs")
    return out


def set_kernel_variant(variant: int = 0) -> None:
    """Select the kernel variant (0 = automatic; see include/tasx_xsum.h)."""
    _check(lib().tasx_set_kernel_variant(variant), "tasx_set_kernel_variant")


class PinnedBuffer:
    """Pinned host memory from tasx_host_alloc, exposed as a numpy array."""

    def __init__(self, nbytes: int):
        import numpy as np
        self.nbytes = nbytes
        self.addr = lib().tasx_host_alloc(nbytes)
        if not self.addr:
            raise TasxError(-errno.ENOMEM, "tasx_host_alloc")
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.addr))
        self.dev_addr = lib().tasx_host_device_pointer(self.addr)
        if not self.dev_addr:
            raise TasxError(-errno.EIO, "tasx_host_device_pointer")

    def free(self) -> None:
        # refused (-EBUSY) while a flush server runs (HIP frees wait for its
        # kernel): the buffer stays, and a later free() releases it
        if self.addr and lib().tasx_host_free(self.addr) == 0:
            self.addr = 0
            self.array = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
