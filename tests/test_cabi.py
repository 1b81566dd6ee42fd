"""The C-ABI library loads and exports every entry point include/tbls_gpu.h
and include/tbls_ssz.h declare (no GPU compute without a GPU), and fails
loudly without a device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("tbls_gpu.h", "tbls_ssz.h")]


def declared():
    src = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\s*\*|uint32_t|tbg_ctx\s*\*)\s*(tbg_\w+)\s*\(", src, re.M)))


def lib_path():
    from charon_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libtbls_gpu.so not built (run __graft_entry__.build())")
    return _native.LIB_PATH


def test_header_declares_the_boundary():
    names = declared()
    for must in ["tbg_init", "tbg_destroy", "tbg_load_pubkeys", "tbg_submit", "tbg_collect", "tbg_run",
                 "tbg_replay", "tbg_replay_multi", "tbg_fetch", "tbg_strerror", "tbg_sign", "tbg_sk_to_pk",
                 "tbg_poll", "tbg_multi_init", "tbg_multi_submit", "tbg_multi_collect", "tbg_multi_load_pubkeys",
                 "tbg_multi_context", "tbg_multi_layout", "tbg_ssz_roots", "tbg_signing_roots",
                 "tbg_compute_domain", "tbg_ssz_size", "tbg_sum_pubkeys", "tbg_sum_sigs",
                 "tbg_fast_aggregate_verify"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(lib_path())
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from charon_amd import _native
    assert set(declared()) == set(_native.SIGNATURES)


def test_strerror_without_gpu():
    from charon_amd import _native
    lib = _native.load() if os.path.exists(_native.LIB_PATH) else pytest.skip("not built")
    assert lib.tbg_strerror(0) == b"ok"
    assert lib.tbg_strerror(-4) == b"no gfx950 device"


def test_no_cpu_fallback_without_device():
    from charon_amd import _native, engine
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("not built")
    if engine.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(engine.EngineError):
        engine.Engine(0)
    with pytest.raises(engine.EngineError):
        engine.MultiEngine([0, 0])
