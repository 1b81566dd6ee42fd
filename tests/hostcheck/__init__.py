"""Host (CPU) build of the engine's device math, for the CPU test suite.

TEST TOOLING ONLY -- see hostcheck.cpp.  Built on demand with the ROCm clang
(host target) and TBG_BOUNDS_CHECK, which aborts on any violated value bound.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "hostcheck.cpp")
LIB = os.path.join(HERE, "libhostcheck.so")
CSRC = os.path.join(os.path.dirname(os.path.dirname(HERE)), "charon_amd", "csrc")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build():
    if _stale():
        cxx = "/opt/rocm/llvm/bin/clang++"
        if not os.path.exists(cxx):
            cxx = "clang++"
        subprocess.check_call([cxx, "-O1", "-std=c++17", "-fPIC", "-shared", "-DTBG_BOUNDS_CHECK",
                               "-Wno-pass-failed", SRC, "-o", LIB])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
    return _lib
