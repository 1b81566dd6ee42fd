#!/usr/bin/env python3
"""Register / scratch / LDS footprint of every kernel of a build, from the
gfx950 code objects' metadata notes (.vgpr_count, .agpr_count, scratch =
.private_segment_fixed_size, .group_segment_fixed_size) -- the occupancy
side of the roofline (waves per SIMD = 512 / (VGPR + AGPR) rounded down).

  python tools/kernel_resources.py [charon_amd/build_obj/libtbls_gpu] [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def code_object(obj, td):
    fat, co = os.path.join(td, "fat"), os.path.join(td, "co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "s.o")],
                          stderr=subprocess.DEVNULL)
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", f"--input={fat}", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    return co


def kernels(co):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    out = []
    for blk in notes.split("  - .agpr_count:")[1:]:
        blk = ".agpr_count:" + blk
        def g(k, default=0):
            m = re.search(r"\." + k + r":\s+(\S+)", blk)
            return m.group(1) if m else default
        out.append({"name": g("name", "?"), "vgpr": int(g("vgpr_count")), "agpr": int(g("agpr_count")),
                    "sgpr": int(g("sgpr_count")), "scratch": int(g("private_segment_fixed_size")),
                    "lds": int(g("group_segment_fixed_size")), "spill_v": int(g("vgpr_spill_count")),
                    "wg": int(g("max_flat_workgroup_size"))})
    return out


def main(objdir="charon_amd/build_obj/libtbls_gpu", filt=""):
    rows = []
    for f in sorted(os.listdir(objdir)):
        if not f.endswith(".o"):
            continue
        with tempfile.TemporaryDirectory() as td:
            try:
                co = code_object(os.path.join(objdir, f), td)
            except subprocess.CalledProcessError:
                continue
            rows += [(f, k) for k in kernels(co)]
    print(f"{'kernel':60s} {'vgpr':>5s} {'agpr':>5s} {'waves':>5s} {'scratch':>7s} {'spill':>5s} {'lds':>6s} {'wg':>5s}")
    for f, k in rows:
        if filt not in k["name"]:
            continue
        regs = k["vgpr"]  # the unified count (arch VGPRs + AGPRs) on gfx950
        waves = min(8, 512 // max(8, -(-regs // 8) * 8))
        print(f"{k['name'][:60]:60s} {k['vgpr']:5d} {k['agpr']:5d} {waves:5d} {k['scratch']:7d} {k['spill_v']:5d} "
              f"{k['lds']:6d} {k['wg']:5d}")


if __name__ == "__main__":
    main(*sys.argv[1:])
