"""libtasx C-ABI checks that need no GPU: the library builds and loads, exports
every entry point include/tasx_xsum.h declares (and the Python mirror binds
them all), carries no CPU checksum code, and rejects bad arguments before any
device work."""
import ctypes
import errno
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = ROOT / "include" / "tasx_xsum.h"
AB_HEADER = ROOT / "include" / "tasx_ab.h"


def header_functions(header=HEADER):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \t\*]*?\b(tasx_\w+)\s*\(", text, flags=re.M)))


@pytest.fixture(scope="module")
def libpath():
    from tas_amd import build
    return build.build()


@pytest.fixture(scope="module")
def L(libpath):
    from tas_amd import xsum
    return xsum.lib()


def test_header_parses():
    fns = header_functions()
    assert "tasx_tcp_checksums" in fns and "tasx_flush" in fns
    assert len(fns) >= 20


def test_exports_every_declared_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", str(libpath)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (tasx_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_python_mirror_binds_every_symbol(L):
    from tas_amd import xsum
    assert sorted(xsum.SIGNATURES) == header_functions()
    for name in header_functions():
        assert getattr(L, name) is not None


def test_no_cpu_checksum_in_product(libpath):
    """The product library must not contain or link the oracle (no CPU fallback)."""
    syms = subprocess.run(["nm", "-D", str(libpath)], capture_output=True, text=True, check=True).stdout
    assert "oracle" not in syms
    dyn = subprocess.run(["readelf", "-d", str(libpath)], capture_output=True, text=True, check=True).stdout
    assert "liboracle" not in dyn
    assert "libamdhip64" in dyn


def test_gfx950_code_object(libpath):
    data = libpath.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # the .hip_fatbin code object
    secs = subprocess.run(["readelf", "-S", str(libpath)], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in secs


def test_abi_version_and_errors_without_gpu(L):
    assert L.tasx_abi_version() == 10
    # argument errors are reported before any HIP call
    rc = L.tasx_raw_cksum_batch_dev(None, None, 0, None, 10, 5, None, None)
    assert rc == -errno.EINVAL
    rc = L.tasx_raw_cksum_batch_dev(ctypes.c_void_p(16), None, 0, None, 200000, 5,
                                    ctypes.c_void_p(16), None)
    assert rc == -errno.EINVAL  # len0 > TASX_RAW_MAX_LEN
    rc = L.tasx_tcp4_cksum_batch_dev(ctypes.c_void_p(16), None, 2048, 4, 14, 34,
                                     ctypes.c_void_p(18), 0, None)
    assert rc == -errno.EINVAL  # misaligned out
    rc = L.tasx_tcp4_cksum_batch_dev(ctypes.c_void_p(16), None, 2048, 4, 14, 34, None, 0, None)
    assert rc == -errno.EINVAL  # no out and not in place
    assert b"tcp4" in L.tasx_last_error()
    # n == 0 is a no-op
    assert L.tasx_raw_cksum_batch_dev(None, None, 0, None, 0, 0, None, None) == 0
    # contexts: not initialised / out of range
    assert L.tasx_defer_tcp4(3, ctypes.c_void_p(64), 14, 34) == -errno.EINVAL
    assert L.tasx_flush(3) == -errno.EINVAL
    assert L.tasx_pending(99) == -errno.EINVAL
    assert L.tasx_ctx_destroy(0) == -errno.EINVAL
    # host batches over offsets: the context is checked first, n == 0 is a no-op
    assert L.tasx_tcp4_cksum_batch_host_offs(5, None, None, None, 4, 14, 34, None, 0) == -errno.EINVAL
    assert L.tasx_raw_cksum_batch_host_offs(5, None, None, None, 0, 4, None, 0) == -errno.EINVAL
    assert b"not initialised" in L.tasx_last_error()
    # flush server (ABI 6): nothing running, no context
    assert L.tasx_server_stop(0) == -errno.EINVAL
    assert L.tasx_server_stats(0, None, None) == -errno.EINVAL
    assert L.tasx_server_epochs(0, None, None, None) == -errno.EINVAL   # ABI 10
    assert L.tasx_server_stop(-1) == -errno.ENODEV
    assert L.tasx_ctx_use_server(3, 1) == -errno.EINVAL
    assert L.tasx_ctx_server_flushes(3, None) == -errno.EINVAL
    assert L.tasx_ctx_register_shm(3, None, 0) == -errno.EINVAL
    assert L.tasx_server_tx_segments(3, None, 0, None) == -errno.EINVAL
    # ABI 8 error recovery: argument errors before any HIP call
    assert L.tasx_take_unfinished(3, None, 0) == -errno.EINVAL
    assert L.tasx_take_unfinished_segs(3, None, 0) == -errno.EINVAL
    assert L.tasx_server_abort(0) == -errno.EINVAL
    assert L.tasx_server_abort(-1) == -errno.ENODEV
    # ABI 9: pause / resume of a server that does not run
    assert L.tasx_server_pause(0) == -errno.EINVAL
    assert L.tasx_server_resume(0) == -errno.EINVAL
    assert L.tasx_server_pause(-1) == -errno.ENODEV
    assert L.tasx_server_resume(1 << 20) == -errno.ENODEV
    if L.tasx_device_count() <= 0:  # no GPU in this container: start fails, nothing launched
        assert L.tasx_server_start(0) in (-errno.EIO, -errno.ENODEV)


def test_python_wrapper_raises(L):
    from tas_amd import xsum
    with pytest.raises(xsum.TasxError):
        xsum.defer_tcp4(2, 4096)
    with pytest.raises(xsum.TasxError):
        xsum.tx_flush(2)


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True,
                         text=True, check=True).stdout
    return set(re.findall(r"\bT (\w+)", out))


def test_product_exports_only_the_header(libpath):
    """libtasx.so exports exactly tasx_xsum.h: no internal launchers, no A/B
    entry points, no kernel stubs."""
    assert _exports(libpath) == set(header_functions())


def test_ab_build_exports_the_ab_header(libpath):
    from tas_amd import build
    ab = _exports(build.LIB_AB)
    assert set(header_functions()) <= ab
    assert set(header_functions(AB_HEADER)) <= ab
    assert not set(header_functions(AB_HEADER)) & _exports(libpath)


def test_product_rejects_ab_variants(L):
    for v in (1, 4, 5, 8, 9, 10, 11, 12, -1):
        assert L.tasx_set_kernel_variant(v) == -errno.EINVAL, v
    for v in (0, 2, 3, 6, 7):
        assert L.tasx_set_kernel_variant(v) == 0
    assert L.tasx_set_kernel_variant(0) == 0
    assert L.tasx_last_kernel() == b""


def test_room_contract_errors(L):
    # a room must hold the headers and stay inside a stride-mode frame's slot
    rc = L.tasx_tcp4_cksum_batch_dev_room(ctypes.c_void_p(4096), None, 2048, None, 0, 40, 4, 14, 34,
                                          ctypes.c_void_p(4096), 0, None)
    assert rc == -errno.EINVAL and b"room" in L.tasx_last_error()
    rc = L.tasx_tcp4_cksum_batch_dev_room(ctypes.c_void_p(4096), None, 2048, None, 0, 4096, 4, 14, 34,
                                          ctypes.c_void_p(4096), 0, None)
    assert rc == -errno.EINVAL and b"stride" in L.tasx_last_error()
    rc = L.tasx_tcp4_verify_batch_dev_room(ctypes.c_void_p(4096), None, 2048, None, 0, 4096, 4, 14, 34,
                                           ctypes.c_void_p(4096), None)
    assert rc == -errno.EINVAL


def test_both_builds_coexist_in_one_process(L):
    """The comparison build loads next to the product (-Bsymbolic, RTLD_LOCAL):
    each keeps its own error state, and only it has the comparison entry points."""
    from tas_amd import xsum
    assert L.tasx_set_kernel_variant(-1) == -errno.EINVAL
    with xsum.using_library(xsum.AB_LIB_PATH) as ab:
        assert ab.tasx_set_kernel_variant(5) == -errno.EINVAL
        assert b"variant 5" in ab.tasx_last_error()
        assert ab.tasx_set_kernel_variant(0) == 0
        assert ab.tasx_ab_stream_read(None, 1024, 0, None, None) == -errno.EINVAL
    assert b"variant -1" in L.tasx_last_error()
    assert not hasattr(L, "tasx_ab_stream_read")


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: a missing build is an error naming the build step, not
    a silent switch to another path."""
    from tas_amd import xsum
    with pytest.raises(RuntimeError, match="not built"):
        xsum._load(tmp_path / "libtasx.so")
