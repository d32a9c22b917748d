"""tas_amd -- MI355X-native software TCP/IP checksum path for TAS.

The product is libtasx.so (tas_amd/csrc: HIP kernels for gfx950 + C host layer,
C ABI in include/tasx_xsum.h).  ``tas_amd.xsum`` is the Python mirror of the
reference's per-frame interface, used by the tests and by bench.py.
"""

__all__ = ["xsum", "build"]
