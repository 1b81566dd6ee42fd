"""C restatement of the reference tbls path (oracle/c/tbls_oracle.c).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load it as the checker / the timed CPU port.  The product
path (charon_amd/) never imports this package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "tbls_oracle.c")
LIB = os.path.join(HERE, "liboracle_c.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(SRC) > os.path.getmtime(LIB):
        subprocess.check_call(["gcc", "-O3", "-std=c11", "-fPIC", "-shared", "-Wno-unused-function", SRC,
                               "-o", LIB + ".tmp", "-lpthread"])
        os.replace(LIB + ".tmp", LIB)
    return LIB


class OrcBatch(ctypes.Structure):
    """Same field order as tbg_batch (include/tbls_gpu.h)."""
    _fields_ = [("op", ctypes.c_uint32), ("n_duties", ctypes.c_uint32), ("n_partials", ctypes.c_uint32),
                ("n_msgs", ctypes.c_uint32), ("msgs", ctypes.c_void_p), ("msg_off", ctypes.c_void_p),
                ("duty_msg", ctypes.c_void_p), ("duty_first", ctypes.c_void_p), ("duty_threshold", ctypes.c_void_p),
                ("sigs", ctypes.c_void_p), ("identifiers", ctypes.c_void_p), ("pubkey_ids", ctypes.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
        L.orc_init.restype = i32
        L.orc_pk_table.restype = vp
        L.orc_pk_table.argtypes = [vp, u32, vp]
        L.orc_pk_table_free.argtypes = [vp]
        L.orc_run.restype = i32
        L.orc_run.argtypes = [ctypes.POINTER(OrcBatch), vp, u32, i32, vp, vp, vp]
        L.orc_verify.restype = i32
        L.orc_verify.argtypes = [vp, vp, u32, vp]
        L.orc_hash_to_g2.argtypes = [vp, u32, vp]
        L.orc_sign.argtypes = [vp, vp, u32, vp]
        L.orc_sk_to_pk.argtypes = [vp, vp]
        L.orc_g2_decode_status.restype = i32
        L.orc_g2_decode_status.argtypes = [vp]
        L.orc_init()
        _lib = L
    return _lib


def _buf(b):
    return ctypes.create_string_buffer(bytes(b), len(b)) if len(b) else ctypes.create_string_buffer(1)


def verify(pk48: bytes, msg: bytes, sig96: bytes) -> int:
    return lib().orc_verify(_buf(pk48), _buf(msg), len(msg), _buf(sig96))


def hash_to_g2(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    lib().orc_hash_to_g2(_buf(msg), len(msg), out)
    return out.raw


def sign(sk: int, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    lib().orc_sign(_buf(sk.to_bytes(32, "big")), _buf(msg), len(msg), out)
    return out.raw


def sk_to_pk(sk: int) -> bytes:
    out = ctypes.create_string_buffer(48)
    lib().orc_sk_to_pk(_buf(sk.to_bytes(32, "big")), out)
    return out.raw


def g2_decode_status(sig96: bytes) -> int:
    return lib().orc_g2_decode_status(_buf(sig96))


class PubkeyTable:
    """Decoded public keys, indexed like the engine's resident table."""

    def __init__(self, pk48):
        a = np.ascontiguousarray(np.frombuffer(bytes(pk48), dtype=np.uint8) if isinstance(pk48, (bytes, bytearray))
                                 else np.asarray(pk48, dtype=np.uint8)).reshape(-1)
        self.n = a.size // 48
        self.status = np.zeros(self.n, dtype=np.int32)
        self._h = lib().orc_pk_table(a.ctypes.data_as(ctypes.c_void_p), self.n,
                                     self.status.ctypes.data_as(ctypes.c_void_p))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_pk_table_free(self._h)
            self._h = None


def run(op, duty_first, sigs, identifiers, pk_table: PubkeyTable, msgs=None, msg_off=None, duty_msg=None,
        pubkey_ids=None, duty_threshold=None, threads: int = 1):
    """tbg_run semantics on the host: (partial_status, duty_status, agg[n, 96])."""
    u32 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.uint32))  # noqa: E731
    duty_first = u32(duty_first)
    sigs = np.ascontiguousarray(np.asarray(sigs, dtype=np.uint8)).reshape(-1)
    identifiers = np.ascontiguousarray(np.asarray(identifiers, dtype=np.uint8))
    nd, np_ = len(duty_first) - 1, sigs.size // 96
    b = OrcBatch()
    b.op, b.n_duties, b.n_partials = op, nd, np_
    keep = [duty_first, sigs, identifiers]
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    b.duty_first, b.sigs, b.identifiers = ptr(duty_first), ptr(sigs), ptr(identifiers)
    if op != 2:
        msgs = np.ascontiguousarray(np.asarray(msgs, dtype=np.uint8)).reshape(-1)
        msg_off, duty_msg, pubkey_ids = u32(msg_off), u32(duty_msg), u32(pubkey_ids)
        keep += [msgs, msg_off, duty_msg, pubkey_ids]
        b.n_msgs = len(msg_off) - 1
        b.msgs, b.msg_off, b.duty_msg, b.pubkey_ids = ptr(msgs), ptr(msg_off), ptr(duty_msg), ptr(pubkey_ids)
    if op == 3:
        duty_threshold = u32(duty_threshold)
        keep.append(duty_threshold)
        b.duty_threshold = ptr(duty_threshold)
    ps = np.zeros(np_, dtype=np.int32)
    ds = np.zeros(nd, dtype=np.int32)
    agg = np.zeros((nd, 96), dtype=np.uint8)
    rc = lib().orc_run(ctypes.byref(b), pk_table._h, pk_table.n, threads, ptr(ps), ptr(ds), ptr(agg))
    if rc != 0:
        raise RuntimeError(f"orc_run failed: {rc}")
    return ps, ds, agg
