#!/usr/bin/env python3
"""Build K3 diagnostic variants of libswitchml_hip.so into tools/ab/ (sources
copied and patched there; tools/ab/ is git-ignored).  Variants:
  k3_base   the product source
  k3_const  K3 with a constant exponent instead of reading the global
            exponent plane (DIAGNOSTIC ONLY: wrong payload) — is the exponent
            read the whole K1-K3 gap?
Timed by tools/ab_k3b.py on the GPU."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "p4app-switchml_amd")
AB = os.path.join(ROOT, "tools", "ab")

ORIG = """    if (base + kTileElems <= a.nblocks * P && slice_exps_scalar_ok<P>(a.gexp)) {
#pragma unroll
        for (int u = 0; u < kU; u++) e[u] = (int)(int8_t)slice_exponent_byte<P>(a.gexp, base, u, lane);
    } else {"""
CONST = """    if (base + kTileElems <= a.nblocks * P && slice_exps_scalar_ok<P>(a.gexp)) {
#pragma unroll
        for (int u = 0; u < kU; u++) e[u] = 2;
    } else {"""


def build(name, patch=None):
    d = os.path.join(AB, name)
    if os.path.isdir(d):
        shutil.rmtree(d)
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(d, "csrc"))
    if patch:
        f = os.path.join(d, "csrc", "sml_quantizer.hip")
        s = open(f).read()
        assert s.count(patch[0]) == 1
        open(f, "w").write(s.replace(patch[0], patch[1]))
    objs = []
    for k in ("sml_quantizer", "sml_frames", "sml_switch"):
        o = os.path.join(d, k + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-I" + os.path.join(ROOT, "include"), "-fno-gpu-rdc", "-c", "-o", o,
                        os.path.join(d, "csrc", k + ".hip")], check=True)
        objs.append(o)
    out = os.path.join(AB, name + ".so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-fno-gpu-rdc", "-o", out] + objs,
                   check=True)
    shutil.rmtree(d)
    print(out)


if __name__ == "__main__":
    os.makedirs(AB, exist_ok=True)
    which = sys.argv[1:] or ["k3_base", "k3_const"]
    if "k3_base" in which:
        build("k3_base")
    if "k3_const" in which:
        build("k3_const", (ORIG, CONST))
    for name in which:
        if name not in ("k3_base", "k3_const"):
            build(name)     # any other name: the current product source
