"""Build libtasx.so (and the A/B build libtasx_ab.so) in-tree (tas_amd/_lib/) for gfx950.

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
# the comparison build: the product's own objects plus tas_amd/csrc/ab/ (the
# ceiling kernels bench.py prices the product against, the round-2 TX kernel
# the tests run beside the product, one test hook: include/tasx_ab.h); the
# product sources know nothing of it
LIB_AB = OUT_DIR / "libtasx_ab.so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = "gfx950"

HIP_SRCS = ["xsum_kernels.hip", "txseg_kernels.hip", "flow_kernels.hip", "server_kernels.hip"]
C_SRCS = ["tasx_host.c"]
AB_HIP_SRCS = ["ab/ab_xsum.hip", "ab/ab_txseg.hip", "ab/ab_flow.hip"]
AB_C_SRCS = ["ab/ab_host.c"]


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def _stale(lib: Path) -> bool:
    if not lib.exists():
        return True
    t = lib.stat().st_mtime
    deps = (list(CSRC.glob("*")) + list((CSRC / "ab").glob("*")) + list((ROOT / "include").glob("*.h")) +
            [Path(__file__)])
    return any(d.stat().st_mtime > t for d in deps)


def _objects(hip_srcs: list[str], c_srcs: list[str], extra_hip_flags: list[str] | None) -> list[Path]:
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    objs = []
    hipcc = str(ROCM / "bin" / "hipcc")
    for s in hip_srcs:
        o = OUT_DIR / (Path(s).stem + ".o")
        _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
              "-Wall", "-Werror", "-Wno-unused-function",
              "-I", str(ROOT / "include"), *(extra_hip_flags or []),
              "-c", str(CSRC / s), "-o", str(o)])
        objs.append(o)
    for s in c_srcs:
        o = OUT_DIR / (Path(s).stem + ".o")
        _run(["gcc", "-std=gnu99", "-O2", "-fPIC", "-Wall", "-Werror",
              "-D__HIP_PLATFORM_AMD__", "-I", str(ROCM / "include"),
              "-I", str(ROOT / "include"), "-c", str(CSRC / s), "-o", str(o)])
        objs.append(o)
    return objs


def _link(lib: Path, objs: list[Path]) -> Path:
    hipcc = str(ROCM / "bin" / "hipcc")
    tmp = lib.with_suffix(".so.tmp")
    # -Bsymbolic: each library's internal calls bind to its own definitions, so
    # the product and the A/B build can be loaded into one process side by side
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp),
          *map(str, objs), f"-Wl,-rpath,{ROCM / 'lib'}", "-Wl,--no-undefined", "-Wl,-Bsymbolic",
          f"-Wl,-soname,{lib.name}"])
    tmp.replace(lib)
    return lib


# bench.py's launch loops (measurement plumbing over libtasx's public C ABI)
LIB_BENCH = OUT_DIR / "libtasx_bench.so"
LIB_BENCH_AB = OUT_DIR / "libtasx_bench_ab.so"  # the same loops over the A/B build
BENCH_SRC = ROOT / "tas_amd" / "benchsrc" / "bench_loop.c"


def build(force: bool = False, extra_hip_flags: list[str] | None = None, ab: bool = True) -> Path:
    """Build libtasx.so (and, with ab=True, libtasx_ab.so; and the bench loop
    library) when stale; returns the product library's path."""
    prod_objs = None
    if force or _stale(LIB):
        prod_objs = _objects(HIP_SRCS, C_SRCS, extra_hip_flags)
        _link(LIB, prod_objs)
    if ab and (force or _stale(LIB_AB)):
        if prod_objs is None:
            prod_objs = [OUT_DIR / (Path(s).stem + ".o") for s in HIP_SRCS + C_SRCS]
            if not all(o.exists() for o in prod_objs):
                prod_objs = _objects(HIP_SRCS, C_SRCS, extra_hip_flags)
        # the A/B library: the product's own objects, plus its variants and knobs
        _link(LIB_AB, prod_objs + _objects(AB_HIP_SRCS, AB_C_SRCS, extra_hip_flags))
    for out, dep, name in ((LIB_BENCH, LIB, "tasx"), (LIB_BENCH_AB, LIB_AB, "tasx_ab")):
        if not dep.exists():
            continue
        if force or not out.exists() or out.stat().st_mtime < max(
                BENCH_SRC.stat().st_mtime, dep.stat().st_mtime, (ROOT / "include" / "tasx_xsum.h").stat().st_mtime):
            _run(["gcc", "-std=gnu99", "-O2", "-fPIC", "-Wall", "-Werror", "-shared", "-pthread", "-I",
                  str(ROOT / "include"), "-o", str(out), str(BENCH_SRC), "-L", str(OUT_DIR), f"-l{name}",
                  "-Wl,-rpath,$ORIGIN", "-Wl,--no-undefined"])
    return LIB


# C boundary test (tests/c/boundary_test.c): compiled against the reference's own
# wire headers, so it is built only where /root/reference exists (this build
# container); the binary travels with the tree to the GPU box
REF_INCLUDE = Path("/root/reference/include")
C_TEST_SRC = ROOT / "tests" / "c" / "boundary_test.c"
C_TEST_BIN = ROOT / "tests" / "c" / "bin" / "boundary_test"


def build_c_tests(force: bool = False) -> Path | None:
    if not (REF_INCLUDE / "packet_defs.h").exists():
        return C_TEST_BIN if C_TEST_BIN.exists() else None
    deps = [C_TEST_SRC, C_TEST_SRC.with_name("tas_glue.h"), C_TEST_SRC.with_name("rte_standin.h"),
            ROOT / "include" / "tasx_xsum.h", LIB]
    if force or not C_TEST_BIN.exists() or C_TEST_BIN.stat().st_mtime < max(d.stat().st_mtime for d in deps):
        C_TEST_BIN.parent.mkdir(parents=True, exist_ok=True)
        _run(["gcc", "-std=gnu99", "-O2", "-Wall", "-I", str(REF_INCLUDE), "-I", str(ROOT / "include"),
              "-o", str(C_TEST_BIN), str(C_TEST_SRC), "-L", str(OUT_DIR), "-ltasx",
              "-Wl,-rpath,$ORIGIN/../../../tas_amd/_lib", "-Wl,--no-undefined"])
    return C_TEST_BIN


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB)
