"""Build libtasx.so in-tree (tas_amd/_lib/) for gfx950.

hipcc compiles the HIP kernels for --offload-arch=gfx950 only; gcc compiles the
C host layer (gnu99, the reference's dialect) against the HIP runtime's C API.
The result links libamdhip64 by soname, so inside a process that already
imported torch it binds to the HIP runtime torch loaded (one runtime per
process).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "tas_amd" / "csrc"
OUT_DIR = ROOT / "tas_amd" / "_lib"
LIB = OUT_DIR / "libtasx.so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = "gfx950"

HIP_SRCS = ["xsum_kernels.hip", "txseg_kernels.hip", "flow_kernels.hip"]
C_SRCS = ["tasx_host.c"]


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = list(CSRC.glob("*")) + [ROOT / "include" / "tasx_xsum.h", Path(__file__)]
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, extra_hip_flags: list[str] | None = None) -> Path:
    if not force and not _stale():
        return LIB
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    objs = []
    hipcc = str(ROCM / "bin" / "hipcc")
    for s in HIP_SRCS:
        o = OUT_DIR / (Path(s).stem + ".o")
        _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
              "-Wall", "-Werror", "-Wno-unused-function",
              "-I", str(ROOT / "include"), *(extra_hip_flags or []),
              "-c", str(CSRC / s), "-o", str(o)])
        objs.append(o)
    for s in C_SRCS:
        o = OUT_DIR / (Path(s).stem + ".o")
        _run(["gcc", "-std=gnu99", "-O2", "-fPIC", "-Wall", "-Werror",
              "-D__HIP_PLATFORM_AMD__", "-I", str(ROCM / "include"),
              "-I", str(ROOT / "include"), "-c", str(CSRC / s), "-o", str(o)])
        objs.append(o)
    tmp = LIB.with_suffix(".so.tmp")
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp),
          *map(str, objs), f"-Wl,-rpath,{ROCM / 'lib'}", "-Wl,--no-undefined",
          "-Wl,-soname,libtasx.so"])
    tmp.replace(LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB)
