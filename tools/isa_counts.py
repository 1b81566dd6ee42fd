#!/usr/bin/env python3
"""Static instruction mix of the engine's kernels (no GPU): compiles the
named csrc units for gfx950 to assembly and counts, per kernel, the VALU
instructions, the v_mad_u64_u32 among them, and the largest other classes.
The kernels are issue-bound, so fewer non-multiply
instructions per product is the lever this tracks.

  python tools/isa_counts.py k_miller_hex.hip k_decode.hip ... [--defines X=1 ...]
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "charon_amd", "csrc")


def kernels(asm):
    out = {}
    for m in re.finditer(r"^(_Z[^\s:]+):[^\n]*\n(.*?)^\.Lfunc_end", asm, re.M | re.S):
        name, body = m.group(1), m.group(2)
        ops = collections.Counter(l.split()[0] for l in body.splitlines() if re.match(r"\s+[vsgbd][a-z_0-9]+", l))
        out[name] = ops
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return dict(zip(names, r.stdout.splitlines()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("units", nargs="+")
    ap.add_argument("--defines", nargs="*", default=[])
    ap.add_argument("--out", default="/tmp/isa")
    ap.add_argument("--reuse", action="store_true", help="count existing .s files in --out")
    ap.add_argument("--min-valu", type=int, default=500, help="skip functions with fewer VALU instructions")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for u in a.units:
        s = os.path.join(a.out, os.path.basename(u).replace(".hip", ".s"))
        src = u if os.path.exists(u) else os.path.join(CSRC, u)
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
               "-Wno-pass-failed", "-I", CSRC, src, "-o", s] + ["-D" + d for d in a.defines]
        if not a.reuse or not os.path.exists(s):
            subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
        ks = kernels(open(s).read())
        print(f"-- {u}")
        dm = demangle(list(ks))
        for k, ops in ks.items():
            valu = sum(v for o, v in ops.items() if o.startswith("v_"))
            mad = ops.get("v_mad_u64_u32", 0)
            if valu < a.min_valu:
                continue
            top = ", ".join(f"{o[2:]} {v}" for o, v in ops.most_common(9) if o.startswith("v_") and o != "v_mad_u64_u32")
            print(f"{dm[k].split('(')[0]:45s} valu {valu:6d} mad {mad:6d} ({mad / max(1, valu):.3f})  "
                  f"scratch {ops.get('scratch_load_dword', 0) + ops.get('scratch_load_dwordx2', 0) + ops.get('scratch_load_dwordx4', 0):4d}  {top}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
