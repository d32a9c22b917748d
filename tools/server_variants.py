"""Build the flush server's comparison forms (round 6, profiles/r06/INDEX.md
r06d, r06e): the product's sources copied to a scratch directory, one change
each in server_device.h / tasx_host.c, linked with the product's other objects
into tools/bin/exp_<name>/libtasx.so (soname libtasx.so, so bench.py's loop
library binds to it under TASX_LIB).  None of these is a product form:

  prod    the product as it is (two workgroups per ring taking turns at
          reading frames: the ring's read token)
  k1      one workgroup per ring
  notok   two workgroups per ring reading frames at once (round 4-5)
  rows8   a batch's frames summed 8 (rows16: 16) at a time
  sysld   system-scope frame loads and no acquire for checksum slots
  noacq   no acquire for checksum slots (serves stale lines: pricing only)

    python tools/server_variants.py          # then: bash tools/server_variants_price.sh TAG
"""
import os, shutil, subprocess, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMP = "/tmp/tasx_server_variants"
def run(c): subprocess.run(c, check=True)
VARS = {
  "prod": {},
  "rows8": {"rows": 8},
  "rows16": {"rows": 16},
  "k1": {"k": 1},
  "notok": {"notok": 1},
  "sysld": {"sys": 1},
  "noacq": {"noacq": 1},
}
os.makedirs(f"{TMP}/t", exist_ok=True)
if not os.path.exists(f"{TMP}/include"):  # tasx_kernels.h includes ../../include/tasx_xsum.h
    os.symlink(f"{R}/include", f"{TMP}/include")
for name, v in VARS.items():
    d = f"{TMP}/t/{name}"
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(f"{R}/tas_amd/csrc", d)
    s = open(f"{d}/server_device.h").read()
    if "rows" in v:
        n = v["rows"]
        a = "    } else if (row < s_n) {\n      const uint64_t base = s_base;"
        assert a in s
        s = s.replace(a, f"    }} else if (row < {n}u) {{\n     for (uint32_t jr = row; jr < s_n; jr += {n}u) {{\n      const uint64_t base = s_base;")
        a = "      const uint32_t fo = s_off[row], tl = s_tl[row];"
        s = s.replace(a, "      const uint32_t fo = s_off[jr], tl = s_tl[jr];")
        a = "      if (gl == 15 && !ok)\n        atomicOr(&s_bad, 1u);\n    }\n    if (K > 1u) {"
        assert a in s
        s = s.replace(a, "      if (gl == 15 && !ok)\n        atomicOr(&s_bad, 1u);\n     }\n    }\n    if (K > 1u) {")
    if "notok" in v:
        a = "      if (st == 1 && K > 1u) {\n        for (uint32_t sp = 1;; ++sp) {"
        assert a in s
        s = s.replace(a, "      if (st == 1 && K > 1u && false) {\n        for (uint32_t sp = 1;; ++sp) {")
    if "sys" in v:
        a = "      ok = ok && srv_row(rs, fo, tl, gl);"
        assert a in s
        s = s.replace(a, "      ok = ok && srv_row<kSys>(rs, fo, tl, gl);")
    if "sys" in v or "noacq" in v:
        a = "      if (st == 1)\n        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"\");"
        assert a in s
        s = s.replace(a, "      if (st == 1 && s_seg)\n        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"\");")
    open(f"{d}/server_device.h", "w").write(s)
    h = open(f"{d}/tasx_host.c").read()
    if "k" in v:
        h = h.replace("#define SRV_K 2u", f"#define SRV_K {v['k']}u"); assert f"SRV_K {v['k']}u" in h
    open(f"{d}/tasx_host.c", "w").write(h)
    o = f"{R}/tools/bin/exp_{name}"
    os.makedirs(o, exist_ok=True)
    objs = []
    for src in ["xsum_kernels.hip", "txseg_kernels.hip", "flow_kernels.hip", "server_kernels.hip"]:
        ob = f"{TMP}/{name}_{src}.o"
        if src != "server_kernels.hip":
            ob = f"{R}/tas_amd/_lib/{src.replace('.hip','.o')}"
        else:
            run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-I", d, "-I", f"{R}/include", "-c", f"{d}/{src}", "-o", ob])
        objs.append(ob)
    hob = f"{TMP}/{name}_host.o"
    run(["gcc", "-std=gnu99", "-O2", "-fPIC", "-Wall", "-Werror", "-pthread", "-I", f"{R}/include", "-I", d, "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-c", f"{d}/tasx_host.c", "-o", hob])
    objs.append(hob)
    run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{o}/libtasx.so", *objs, "-Wl,-rpath,/opt/rocm/lib", "-Wl,--no-undefined", "-Wl,-Bsymbolic", "-Wl,-soname,libtasx.so"])
    print("built", name)
