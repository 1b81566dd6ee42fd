"""Build and load libtbls_gpu.so (the HIP engine behind include/tbls_gpu.h).

The library is built in-tree (``charon_amd/libtbls_gpu.so``) so it travels
with the repository snapshot to the GPU box.  There is no CPU fallback: if
the library or a gfx950 device is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_PATH = os.path.join(PKG, "libtbls_gpu.so")
HEADER = os.path.join(ROOT, "include", "tbls_gpu.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "tbls_ssz.h")]


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build libtbls_gpu.so")


def _clangxx():
    c = "/opt/rocm/llvm/bin/clang++"
    if not os.path.exists(c):
        raise RuntimeError("ROCm clang++ not found: cannot build the host units of libtbls_gpu.so")
    return c


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                  if f.endswith((".h", ".hip", ".cpp"))) + HEADERS


# What the last build() call did (reported by __graft_entry__.build): "reused"
# (the in-tree library was newer than every source), "compiled" (units
# recompiled with hipcc, then linked) or "relinked" (objects up to date).
LAST_BUILD = {"mode": None}


def is_stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    # (this file holds the compile flags)
    return any(os.path.getmtime(s) > t for s in list(sources()) + [os.path.abspath(__file__)])


# Per-translation-unit compiler flags on top of the common ones.  The
# machine scheduler's max-ILP strategy for the decode and Miller units
# (k_decode_sigs -3 %, k_miller_hex<L0> -2 % with unchanged occupancy;
# driver shape +1.6 %, profiles/r06/ilp/), then also the H(m)-lines,
# cofactor and aggregation units (+0.75 %, ilp/units_more/).  Library-wide it raised small
# kernels' VGPRs (k_sgb_sort 66 -> 119: 7 -> 4 waves) and the SSWU spills,
# and lost at 20 steps although every big kernel ran faster alone.
_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
UNIT_FLAGS: dict = {u: _ILP for u in ("k_decode.hip", "k_miller_hex.hip", "k_verify.hip", "k_hash_clear.hip",
                                       "k_aggregate.hip")}


def build(force: bool = False, verbose: bool = False, jobs: int = 0, defines=(), out: str | None = None,
          extra_flags=(), link_flags=(), unit_flags=None) -> str:
    """Compile the engine for gfx950: every csrc/*.hip translation unit in
    parallel (hipcc -c), then link libtbls_gpu.so.  `defines` / `out` build a
    tuning variant elsewhere (tools/ab_variants.py)."""
    target = out or LIB_PATH
    if not force and out is None and not is_stale():
        LAST_BUILD.update(mode="reused", target=target, units_compiled=0, units_total=0)
        return LIB_PATH
    from concurrent.futures import ThreadPoolExecutor
    hipcc = _hipcc()
    # .hip: device + host code (hipcc); .cpp: host-only code (ROCm clang++, no offload)
    units = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    # one object directory per output (variants never share the product's objects)
    tag = os.path.basename(target).replace(".so", "")
    if os.path.abspath(target) != LIB_PATH:
        tag = os.path.basename(os.path.dirname(os.path.abspath(target))) + "_" + tag
    objdir = os.path.join(PKG, "build_obj", tag)
    os.makedirs(objdir, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed", "-Wno-unused-result", "-Wno-unused-value"]
    flags += ["-D" + d for d in defines] + list(extra_flags)

    unit_flags = UNIT_FLAGS if unit_flags is None else unit_flags
    stamp_text = " ".join(flags) + "".join(f" [{u}: {' '.join(f)}]" for u, f in sorted(unit_flags.items()))
    headers = [s for s in sources() if s.endswith(".h")]
    stamp = os.path.join(objdir, "flags.txt")
    same_flags = os.path.exists(stamp) and open(stamp).read() == stamp_text

    host_flags = ["-O3", "-std=c++17", "-fPIC"] + ["-D" + d for d in defines] + \
        [f for f in extra_flags if f != "-Xarch_host"]

    compiled = []

    def compile_unit(u):
        obj = os.path.join(objdir, os.path.splitext(u)[0] + ".o")
        if same_flags and not force and os.path.exists(obj):
            t = os.path.getmtime(obj)
            if all(os.path.getmtime(d) < t for d in headers + [os.path.join(CSRC, u)]):
                return obj  # up to date (incremental rebuild)
        compiled.append(u)
        if u.endswith(".cpp"):
            cmd = [_clangxx()] + host_flags + ["-c", os.path.join(CSRC, u), "-o", obj]
        else:
            cmd = [hipcc] + flags + list(unit_flags.get(u, ())) + ["-c", os.path.join(CSRC, u), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        return obj

    jobs = jobs or min(len(units), max(1, (os.cpu_count() or 4)), 8)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_unit, units))
    for obj in objs:
        check_return_address(obj)
    with open(stamp, "w") as f:
        f.write(stamp_text)
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC"] + list(link_flags) + objs + ["-o", target + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(target + ".tmp", target)
    LAST_BUILD.update(mode="compiled" if compiled else "relinked", target=target, units_compiled=len(compiled),
                      units_total=len(units))
    return target


def check_return_address(obj: str) -> None:
    """Refuse a code object in which a callable function clobbers its return
    address.  When a loop body in an out-of-line device function exceeds the
    16-bit branch range, this compiler expands the long branch as
    `s_getpc_b64 s[30:31]` ... `s_setpc_b64 s[30:31]` -- s[30:31] holds the
    function's return address, so the return jumps into the function again
    and the kernel never finishes (observed on gfx950).  Kernels use a free
    SGPR pair and are not affected."""
    llvm = "/opt/rocm/llvm/bin"
    for tool in ("llvm-objdump", "llvm-objcopy", "clang-offload-bundler"):
        if not os.path.exists(os.path.join(llvm, tool)):
            # fail closed: this guard stands between a known GPU hang and the box
            raise RuntimeError(f"{llvm}/{tool} is missing: cannot run the return-address check on {obj}")
    import re
    import tempfile
    heads = subprocess.run([os.path.join(llvm, "llvm-objdump"), "-h", obj], capture_output=True, text=True).stdout
    if ".hip_fatbin" not in heads:
        return  # host-only translation unit
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fatbin"), os.path.join(td, "co")
        subprocess.check_call([os.path.join(llvm, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj,
                               os.path.join(td, "stripped.o")])
        subprocess.check_call([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", f"--input={fat}", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        asm = subprocess.run([os.path.join(llvm, "llvm-objdump"), "-d", co], capture_output=True, text=True,
                             check=True).stdout
        syms = subprocess.run([os.path.join(llvm, "llvm-objdump"), "-t", co], capture_output=True, text=True,
                              check=True).stdout
    # kernels (a .kd descriptor each) may use s[30:31] as a free pair; every
    # other function holds its return address there
    kernels = set(re.findall(r"\s(\S+)\.kd\s*$", syms, flags=re.M))
    bad = []
    for m in re.finditer(r"^[0-9a-f]+ <([^>]+)>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", asm, flags=re.M | re.S):
        if m.group(1) not in kernels and re.search(r"s_getpc_b64\s+s\[30:31\]", m.group(2)):
            bad.append(m.group(1))
    if bad:
        raise RuntimeError(f"{obj}: long branch(es) through s[30:31] in out-of-line function(s) {bad} "
                           "(return-address clobber; would hang on the GPU) -- keep that loop body smaller")


class TbgBatch(ctypes.Structure):
    _fields_ = [
        ("op", ctypes.c_uint32),
        ("n_duties", ctypes.c_uint32),
        ("n_partials", ctypes.c_uint32),
        ("n_msgs", ctypes.c_uint32),
        ("msgs", ctypes.c_void_p),
        ("msg_off", ctypes.c_void_p),
        ("duty_msg", ctypes.c_void_p),
        ("duty_first", ctypes.c_void_p),
        ("duty_threshold", ctypes.c_void_p),
        ("sigs", ctypes.c_void_p),
        ("identifiers", ctypes.c_void_p),
        ("pubkey_ids", ctypes.c_void_p),
    ]


class TbgKernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 64), ("ms", ctypes.c_float)]


class TbgConfig(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("max_partials", ctypes.c_uint32),
        ("max_duties", ctypes.c_uint32),
        ("max_msg_bytes", ctypes.c_uint32),
        ("slots", ctypes.c_uint32),
        ("verify_mode", ctypes.c_uint32),
        ("rlc_group", ctypes.c_uint32),
        ("rlc_seed", ctypes.c_uint64),
        ("rlc_chunk", ctypes.c_uint32),
        ("streams_per_slot", ctypes.c_uint32),
        ("rlc_batch", ctypes.c_uint32),
        ("gident", ctypes.c_uint32),
        ("fb_window", ctypes.c_uint32),
        ("subgroup_batch", ctypes.c_uint32),
        ("express_partials", ctypes.c_uint32),
    ]


# exported symbols and their signatures (checked by tests/test_cabi.py)
SIGNATURES = {
    "tbg_init": (ctypes.c_int, [ctypes.POINTER(TbgConfig), ctypes.POINTER(ctypes.c_void_p)]),
    "tbg_destroy": (None, [ctypes.c_void_p]),
    "tbg_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "tbg_device_count": (ctypes.c_int, []),
    "tbg_device_cu_count": (ctypes.c_int, [ctypes.c_int]),
    "tbg_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "tbg_load_pubkeys": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p]),
    "tbg_pubkey_count": (ctypes.c_uint32, [ctypes.c_void_p]),
    "tbg_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TbgBatch), ctypes.POINTER(ctypes.c_uint64)]),
    "tbg_collect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int]),
    "tbg_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TbgBatch), ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]),
    "tbg_replay": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]),
    "tbg_replay_multi": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p]),
    "tbg_fetch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tbg_fetch_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tbg_fetch_level0": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tbg_fetch_fallback": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tbg_fetch_subgroup": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tbg_fetch_shape": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tbg_host_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tbg_multi_host_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tbg_slot_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "tbg_last_timings": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tbg_sk_to_pk": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    "tbg_sign": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "tbg_poll": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "tbg_submit_group": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    "tbg_replay_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint32)]),
    "tbg_replay_plan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p]),
    "tbg_multi_init": (ctypes.c_int, [ctypes.POINTER(TbgConfig), ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_void_p)]),
    "tbg_multi_destroy": (None, [ctypes.c_void_p]),
    "tbg_multi_size": (ctypes.c_uint32, [ctypes.c_void_p]),
    "tbg_multi_context": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint32]),
    "tbg_multi_load_pubkeys": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p]),
    "tbg_multi_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TbgBatch), ctypes.POINTER(ctypes.c_uint64)]),
    "tbg_multi_submit_group": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    "tbg_multi_collect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int]),
    "tbg_multi_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tbg_sum_pubkeys": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "tbg_sum_sigs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tbg_fast_aggregate_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    # include/tbls_ssz.h (host code)
    "tbg_ssz_size": (ctypes.c_uint32, [ctypes.c_uint32]),
    "tbg_ssz_roots": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_uint32]),
    "tbg_compute_domain": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]),
    "tbg_signing_roots": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                         ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load the engine library (never a CPU fallback)."""
    global _lib
    if _lib is None:
        path = os.environ.get("TBG_LIB", LIB_PATH)  # tuning variants only (tools/ab_variants.py)
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build() (hipcc, gfx950)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib
