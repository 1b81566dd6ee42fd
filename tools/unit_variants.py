#!/usr/bin/env python3
"""Tuning variants of ONE translation unit: recompile csrc/<unit> with extra
defines and link it with the product build's other objects (seconds, not a
full rebuild) into varlib/<name>.so (git-ignored, travels to the GPU box); bench with TBG_LIB=varlib/<name>.so.

  python tools/unit_variants.py k_miller_hex.hip NAME -DKNOB=V ...
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from charon_amd import _native
    unit, name = sys.argv[1], sys.argv[2]
    defs = [a for a in sys.argv[3:] if a.startswith("-D")]
    base = os.path.join(_native.PKG, "build_obj", "libtbls_gpu")
    os.makedirs(os.path.join(ROOT, "varlib", "obj"), exist_ok=True)
    obj = os.path.join(ROOT, "varlib", "obj", name + "_" + unit.replace(".hip", ".o"))
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed", "-Wno-unused-result",
             "-Wno-unused-value"] + defs
    subprocess.check_call([_native._hipcc()] + flags + ["-c", os.path.join(_native.CSRC, unit), "-o", obj])
    _native.check_return_address(obj)
    objs = [o for o in sorted(glob.glob(os.path.join(base, "*.o"))) if os.path.basename(o) != unit.replace(".hip", ".o")]
    out = os.path.join(ROOT, "varlib", name + ".so")
    subprocess.check_call([_native._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + [obj, "-o", out])
    print(out)


if __name__ == "__main__":
    main()
