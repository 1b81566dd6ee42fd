"""Python handle on one MI355X threshold-BLS engine context (libtbls_gpu.so).

Thin ctypes layer over include/tbls_gpu.h: resident public keys, batched
submit/collect of DV-duties, and GPU test-vector generation.  Arrays are
numpy; every call goes to the HIP library (no CPU fallback).
"""
from __future__ import annotations

import ctypes
import itertools
from dataclasses import dataclass

import numpy as np

from . import _native

# per-partial status (TBG_PS_*)
PS_INVALID, PS_VALID, PS_NOT_VERIFIED = 0, 1, 2
PS_ERR_FLAGS, PS_ERR_FIELD, PS_ERR_CURVE, PS_ERR_SUBGROUP, PS_ERR_IDENTITY, PS_ERR_PUBKEY = -1, -2, -3, -4, -5, -6
# per-duty status (TBG_DS_*)
DS_OK, DS_NOT_AGGREGATED = 0, 1
DS_INSUFFICIENT, DS_INSUFFICIENT_VALID = -20, -21
DS_AGG_TOO_FEW, DS_AGG_DUPLICATE_ID, DS_AGG_IDENTITY, DS_DECODE = -22, -23, -24, -25
OP_VERIFY, OP_AGGREGATE, OP_VERIFY_AGGREGATE = 1, 2, 3
NO_PUBKEY = 0xFFFFFFFF
TIMING_KEYS = ["decode", "hash", "combine", "h_lines", "verify", "lagrange", "aggregate", "total"]
VERIFY_RLC, VERIFY_EACH = 0, 1
RLC_L0_AUTO, RLC_L0_ON, RLC_L0_OFF = 0, 1, 2   # tbg_config.rlc_batch
GIDENT_OFF, GIDENT_L3, GIDENT_CHUNKS = 0, 1, 2  # tbg_config.gident
SGB_AUTO, SGB_ON, SGB_OFF = 0, 1, 2           # tbg_config.subgroup_batch
EXPRESS_OFF = 0xFFFFFFFF                        # tbg_config.express_partials: no express slot
L0_NOT_RUN, L0_PASSED, L0_FAILED = 0, 1, 2     # tbg_fetch_level0
HOST_STAT_KEYS = ["submits", "partials_submitted", "pack_ns", "enqueue_ns", "collects", "partials_collected",
                  "gather_ns", "wait_ns"]
MULTI_HOST_STAT_KEYS = ["submits", "partials", "build_ns", "submit_wall_ns", "collects", "collect_wall_ns"] + \
    ["ctx_" + k for k in HOST_STAT_KEYS] + ["contexts", "reserved"]
E_PENDING = -6


class EngineError(RuntimeError):
    pass


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _u8(buf, width=None):
    a = np.frombuffer(bytes(buf), dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else np.ascontiguousarray(buf, dtype=np.uint8)
    if width is not None:
        a = a.reshape(-1, width)
    return np.ascontiguousarray(a)


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def pack_messages(msgs):
    """list of bytes -> (concatenated uint8, uint32 offsets)"""
    off = np.zeros(len(msgs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64).astype(np.uint32)
    data = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
    return np.ascontiguousarray(data), off


@dataclass
class BatchResult:
    partial_status: np.ndarray  # int32 [n_partials]
    duty_status: np.ndarray     # int32 [n_duties]
    agg: np.ndarray             # uint8 [n_duties, 96]


_serial = itertools.count(1)


def device_count() -> int:
    """HIP devices visible to the engine library (tbg_device_count)."""
    return int(_native.load().tbg_device_count())


def device_cu_count(device: int = 0) -> int:
    """Compute units of a device, asked through the engine's own HIP runtime
    (tbg_device_cu_count) -- not torch.cuda, whose bundled runtime would be a
    second one in the process."""
    n = int(_native.load().tbg_device_cu_count(device))
    if n <= 0:
        raise EngineError(f"tbg_device_cu_count({device}): {_native.load().tbg_strerror(n).decode()} ({n})")
    return n


class Engine:
    """One context = one GPU (HIP device ordinal)."""

    def __init__(self, device: int = 0, slots: int = 3, verify_mode: int = VERIFY_RLC, rlc_group: int = 0,
                 rlc_seed: int = 0, rlc_chunk: int = 0, streams_per_slot: int = 0, rlc_batch: int = 0,
                 gident: int = GIDENT_OFF, fb_window: int = 0, subgroup_batch: int = SGB_AUTO,
                 express_partials: int = 0):
        self._lib = _native.load()
        cfg = _native.TbgConfig(device=device, max_partials=0, max_duties=0, max_msg_bytes=0, slots=slots,
                                verify_mode=verify_mode, rlc_group=rlc_group, rlc_seed=rlc_seed,
                                rlc_chunk=rlc_chunk, streams_per_slot=streams_per_slot, rlc_batch=rlc_batch,
                                gident=gident, fb_window=fb_window, subgroup_batch=subgroup_batch,
                                express_partials=express_partials)
        h = ctypes.c_void_p()
        rc = self._lib.tbg_init(ctypes.byref(cfg), ctypes.byref(h))
        self._check(rc, "tbg_init")
        self._h = h
        self.device = device
        self.uid = next(_serial)  # never reused, unlike id(): keys per-context caches
        self._keep = {}

    def _check(self, rc, what):
        if rc != 0:
            raise EngineError(f"{what}: {self._lib.tbg_strerror(rc).decode()} ({rc})")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.tbg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ pubkeys
    def load_pubkeys(self, pk48) -> tuple[int, np.ndarray]:
        a = _u8(pk48, 48)
        n = a.shape[0]
        first = ctypes.c_uint32()
        st = np.zeros(n, dtype=np.int32)
        self._check(self._lib.tbg_load_pubkeys(self._h, _ptr(a), n, ctypes.byref(first), _ptr(st)), "tbg_load_pubkeys")
        return first.value, st

    @property
    def pubkey_count(self) -> int:
        return self._lib.tbg_pubkey_count(self._h)

    # ------------------------------------------------------------ batches
    def _batch(self, op, duty_first, sigs, identifiers, msgs=None, duty_msg=None, pubkey_ids=None, duty_threshold=None):
        duty_first = _u32(duty_first)
        sigs = _u8(sigs, 96) if len(sigs) else np.zeros((0, 96), np.uint8)
        identifiers = np.ascontiguousarray(np.asarray(identifiers, dtype=np.uint8))
        nd = len(duty_first) - 1
        np_ = sigs.shape[0]
        keep = [duty_first, sigs, identifiers]
        b = _native.TbgBatch()
        b.op, b.n_duties, b.n_partials = op, nd, np_
        b.duty_first, b.sigs, b.identifiers = _ptr(duty_first), _ptr(sigs), _ptr(identifiers)
        if op != OP_AGGREGATE:
            data, off = msgs if isinstance(msgs, tuple) else pack_messages(msgs)
            data, off = _u8(data), _u32(off)
            duty_msg = _u32(duty_msg)
            pubkey_ids = _u32(pubkey_ids)
            keep += [data, off, duty_msg, pubkey_ids]
            b.n_msgs = len(off) - 1
            b.msgs, b.msg_off, b.duty_msg, b.pubkey_ids = _ptr(data), _ptr(off), _ptr(duty_msg), _ptr(pubkey_ids)
        if op == OP_VERIFY_AGGREGATE:
            duty_threshold = _u32(duty_threshold)
            keep.append(duty_threshold)
            b.duty_threshold = _ptr(duty_threshold)
        return b, keep, nd, np_

    def submit(self, op, duty_first, sigs, identifiers, **kw):
        b, keep, nd, np_ = self._batch(op, duty_first, sigs, identifiers, **kw)
        t = ctypes.c_uint64()
        self._check(self._lib.tbg_submit(self._h, ctypes.byref(b), ctypes.byref(t)), "tbg_submit")
        self._keep[t.value] = (nd, np_)
        return t.value

    def submit_group(self, op, batches):
        """Several batches (dicts of submit()'s arguments) as one device batch
        (tbg_submit_group); one ticket per batch."""
        built = [self._batch(op, **b) for b in batches]
        arr = (ctypes.POINTER(_native.TbgBatch) * len(built))(*[ctypes.pointer(b) for b, _, _, _ in built])
        t = np.zeros(len(built), dtype=np.uint64)
        self._check(self._lib.tbg_submit_group(self._h, arr, len(built), _ptr(t)), "tbg_submit_group")
        for ticket, (_, _, nd, np_) in zip(t.tolist(), built):
            self._keep[ticket] = (nd, np_)
        return t.tolist()

    def collect(self, ticket, block=True):
        nd, np_ = self._keep[ticket]
        ps = np.zeros(np_, dtype=np.int32)
        ds = np.zeros(nd, dtype=np.int32)
        agg = np.zeros((nd, 96), dtype=np.uint8)
        rc = self._lib.tbg_collect(self._h, ticket, _ptr(ps), _ptr(ds), _ptr(agg), 1 if block else 0)
        if rc == E_PENDING:
            return None
        del self._keep[ticket]
        self._check(rc, "tbg_collect")
        return BatchResult(ps, ds, agg)

    def run(self, op, duty_first, sigs, identifiers, **kw) -> BatchResult:
        return self.collect(self.submit(op, duty_first, sigs, identifiers, **kw))

    def poll(self, ticket) -> bool:
        """True once the batch has finished (nothing is consumed)."""
        rc = self._lib.tbg_poll(self._h, ticket)
        if rc == E_PENDING:
            return False
        self._check(rc, "tbg_poll")
        return True

    def synchronize(self):
        """Wait for every stream of this context (tbg_synchronize)."""
        self._check(self._lib.tbg_synchronize(self._h), "tbg_synchronize")

    def replay(self, ticket, iters=1):
        """Re-run a collected batch's kernel chain on its resident inputs."""
        ms = np.zeros(8, dtype=np.float32)
        self._check(self._lib.tbg_replay(self._h, ticket, iters, _ptr(ms)), "tbg_replay")
        return dict(zip(TIMING_KEYS, ms.tolist()))

    def replay_multi(self, tickets, iters=1):
        """Replay several resident batches round-robin, one in flight per slot."""
        t = np.ascontiguousarray(np.asarray(tickets, dtype=np.uint64))
        ms = np.zeros(8, dtype=np.float32)
        self._check(self._lib.tbg_replay_multi(self._h, _ptr(t), len(t), iters, _ptr(ms)), "tbg_replay_multi")
        return dict(zip(TIMING_KEYS, ms.tolist()))

    def replay_plan(self, tickets, n_parts=None):
        """Launch k re-runs the first n_parts[k] batches (0: all) of the
        resident device batch of tickets[k] (tbg_replay_plan)."""
        t = np.ascontiguousarray(np.asarray(tickets, dtype=np.uint64))
        p = None if n_parts is None else np.ascontiguousarray(np.asarray(n_parts, dtype=np.uint32))
        ms = np.zeros(8, dtype=np.float32)
        self._check(self._lib.tbg_replay_plan(self._h, _ptr(t), _ptr(p), len(t), _ptr(ms)), "tbg_replay_plan")
        return dict(zip(TIMING_KEYS, ms.tolist()))

    def replay_profile(self, ticket, max_entries=512):
        """Replay one resident device batch alone with an event pair around
        every kernel (tbg_replay_profile): [(kernel, ms)] in launch order."""
        buf = (_native.TbgKernelTime * max_entries)()
        n = ctypes.c_uint32()
        self._check(self._lib.tbg_replay_profile(self._h, ticket, buf, max_entries, ctypes.byref(n)),
                    "tbg_replay_profile")
        return [(buf[k].name.decode(), float(buf[k].ms)) for k in range(n.value)]

    def fetch(self, ticket, n_duties, n_partials) -> BatchResult:
        ps = np.zeros(n_partials, dtype=np.int32)
        ds = np.zeros(n_duties, dtype=np.int32)
        agg = np.zeros((n_duties, 96), dtype=np.uint8)
        self._check(self._lib.tbg_fetch(self._h, ticket, _ptr(ps), _ptr(ds), _ptr(agg)), "tbg_fetch")
        return BatchResult(ps, ds, agg)

    def stats(self, ticket) -> dict:
        """Verification work of the batch's last run (how much fell back)."""
        out = np.zeros(4, dtype=np.uint32)
        self._check(self._lib.tbg_fetch_stats(self._h, ticket, _ptr(out)), "tbg_fetch_stats")
        return dict(zip(["groups", "duty_checks", "partial_checks", "group_size"], out.tolist()))

    def fallback(self, ticket) -> dict:
        """Work per verification level of the batch's last run (tbg_fetch_fallback)."""
        out = np.zeros(8, dtype=np.uint32)
        self._check(self._lib.tbg_fetch_fallback(self._h, ticket, _ptr(out)), "tbg_fetch_fallback")
        return dict(zip(["groups", "group_searches", "chunks", "chunk_searches", "duty_searches", "partial_checks",
                         "group_size", "level0"], out.tolist()))

    def shape(self, ticket) -> dict:
        """Verification shape of the batch's last submit (tbg_fetch_shape):
        duties per group and per Miller chunk, level 0, P-chunk hexads."""
        out = np.zeros(4, dtype=np.uint32)
        self._check(self._lib.tbg_fetch_shape(self._h, ticket, _ptr(out)), "tbg_fetch_shape")
        return dict(zip(["group", "chunk", "level0", "chunks"], out.tolist()))

    def subgroup(self, ticket) -> dict:
        """Batched subgroup test of the batch's last run (tbg_fetch_subgroup):
        groups of consecutive partials tested by random combinations (0:
        every signature tested alone), how many failed, partials per group."""
        out = np.zeros(3, dtype=np.uint32)
        self._check(self._lib.tbg_fetch_subgroup(self._h, ticket, _ptr(out)), "tbg_fetch_subgroup")
        return dict(zip(["groups", "failed", "group_size"], out.tolist()))

    def host_stats(self, reset=False) -> dict:
        """Host-side work of this context's submit / collect calls (tbg_host_stats)."""
        out = np.zeros(8, dtype=np.uint64)
        self._check(self._lib.tbg_host_stats(self._h, _ptr(out), 1 if reset else 0), "tbg_host_stats")
        return dict(zip(HOST_STAT_KEYS, out.tolist()))

    def slot_bytes(self, ticket) -> tuple:
        """(device bytes, pinned host bytes) of the slot holding the ticket's batch."""
        dev, pin = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._lib.tbg_slot_bytes(self._h, ticket, ctypes.byref(dev), ctypes.byref(pin)), "tbg_slot_bytes")
        return dev.value, pin.value

    def level0(self, ticket) -> int:
        """Level 0 of the batch's last run: L0_NOT_RUN, L0_PASSED or L0_FAILED."""
        st = ctypes.c_int32(0)
        self._check(self._lib.tbg_fetch_level0(self._h, ticket, ctypes.byref(st)), "tbg_fetch_level0")
        return st.value

    def timings(self):
        ms = np.zeros(8, dtype=np.float32)
        self._check(self._lib.tbg_last_timings(self._h, _ptr(ms)), "tbg_last_timings")
        return dict(zip(TIMING_KEYS, ms.tolist()))

    # ------------------------------------------------------------ vector generation
    def sk_to_pk(self, sk32) -> np.ndarray:
        a = _u8(sk32, 32)
        out = np.zeros((a.shape[0], 48), dtype=np.uint8)
        self._check(self._lib.tbg_sk_to_pk(self._h, _ptr(a), a.shape[0], _ptr(out)), "tbg_sk_to_pk")
        return out

    def sign(self, sk32, msgs, item_msg) -> np.ndarray:
        a = _u8(sk32, 32)
        data, off = msgs if isinstance(msgs, tuple) else pack_messages(msgs)
        data, off, im = _u8(data), _u32(off), _u32(item_msg)
        out = np.zeros((a.shape[0], 96), dtype=np.uint8)
        self._check(self._lib.tbg_sign(self._h, _ptr(a), a.shape[0], _ptr(data), _ptr(off), len(off) - 1, _ptr(im),
                                       _ptr(out)), "tbg_sign")
        return out


    # ---- plain sums / FastAggregateVerify (DKG, cluster lock) ----
    def sum_pubkeys(self, pubkey_ids, off):
        """Sums of resident keys per set -> (48-byte sums [n_sets, 48], status [n_sets])."""
        ids, off = _u32(pubkey_ids), _u32(off)
        n = len(off) - 1
        out = np.zeros((n, 48), dtype=np.uint8)
        st = np.zeros(n, dtype=np.int32)
        self._check(self._lib.tbg_sum_pubkeys(self._h, _ptr(ids), _ptr(off), n, _ptr(out), _ptr(st)),
                    "tbg_sum_pubkeys")
        return out, st

    def sum_sigs(self, sigs, off):
        """Decoded sums of 96-byte signatures per set -> (sums [n_sets, 96],
        status [n_sets], per-signature decode status)."""
        a, off = _u8(sigs, 96), _u32(off)
        n = len(off) - 1
        out = np.zeros((n, 96), dtype=np.uint8)
        st = np.zeros(n, dtype=np.int32)
        sst = np.zeros(max(1, a.shape[0]), dtype=np.int32)
        self._check(self._lib.tbg_sum_sigs(self._h, _ptr(a), _ptr(off), n, _ptr(out), _ptr(st), _ptr(sst)),
                    "tbg_sum_sigs")
        return out, st, sst[:a.shape[0]]

    def fast_aggregate_verify(self, pubkey_ids, key_off, msgs, sigs):
        """Per set: CoreVerify(sum of its resident keys, msg, sig) -> status [n_sets]."""
        ids, koff = _u32(pubkey_ids), _u32(key_off)
        data, moff = msgs if isinstance(msgs, tuple) else pack_messages(msgs)
        data, moff, a = _u8(data), _u32(moff), _u8(sigs, 96)
        n = len(koff) - 1
        st = np.zeros(n, dtype=np.int32)
        self._check(self._lib.tbg_fast_aggregate_verify(self._h, _ptr(ids), _ptr(koff), n, _ptr(data), _ptr(moff),
                                                        _ptr(a), _ptr(st)), "tbg_fast_aggregate_verify")
        return st


class MultiEngine:
    """One process, several GPUs (tbg_multi_*): batches are cut into
    contiguous duty ranges, one per context, submitted concurrently and
    gathered back into caller order.  ``devices`` may repeat an ordinal
    (several contexts on one GPU)."""

    def __init__(self, devices, slots: int = 3, verify_mode: int = VERIFY_RLC, rlc_group: int = 0, rlc_seed: int = 0,
                 rlc_chunk: int = 0, streams_per_slot: int = 0, rlc_batch: int = 0, gident: int = GIDENT_OFF,
                 fb_window: int = 0, subgroup_batch: int = SGB_AUTO):
        self._lib = _native.load()
        cfg = _native.TbgConfig(device=0, max_partials=0, max_duties=0, max_msg_bytes=0, slots=slots,
                                verify_mode=verify_mode, rlc_group=rlc_group, rlc_seed=rlc_seed,
                                rlc_chunk=rlc_chunk, streams_per_slot=streams_per_slot, rlc_batch=rlc_batch,
                                gident=gident, fb_window=fb_window, subgroup_batch=subgroup_batch)
        devs = np.ascontiguousarray(np.asarray(devices, dtype=np.int32))
        h = ctypes.c_void_p()
        rc = self._lib.tbg_multi_init(ctypes.byref(cfg), _ptr(devs), len(devs), ctypes.byref(h))
        if rc != 0:
            raise EngineError(f"tbg_multi_init: {self._lib.tbg_strerror(rc).decode()} ({rc})")
        self._h = h
        self.devices = devs.tolist()
        self.uid = next(_serial)
        self._keep = {}
        import weakref
        self._borrowed = weakref.WeakSet()  # per-context Engines handed out by context()

    _check = Engine._check
    _batch = Engine._batch

    @property
    def size(self) -> int:
        return self._lib.tbg_multi_size(self._h)

    def close(self):
        if getattr(self, "_h", None):
            # the borrowed per-context Engines lose their handles first: a
            # later call through one raises EngineError (a NULL context)
            # instead of reaching freed native memory
            for e in list(getattr(self, "_borrowed", ())):
                e._h = None
            self._lib.tbg_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def context(self, i: int) -> "Engine":
        """Context i of the multi-context as an Engine (borrowed: closing it
        does nothing; it lives as long as the multi-context) -- e.g. to
        generate test vectors without opening another context."""
        h = self._lib.tbg_multi_context(self._h, i)
        if not h:
            raise EngineError(f"tbg_multi_context: no context {i}")
        e = _BorrowedEngine(self._lib, h, self.devices[i], self)
        self._borrowed.add(e)
        return e

    def load_pubkeys(self, pk48) -> tuple[int, np.ndarray]:
        a = _u8(pk48, 48)
        n = a.shape[0]
        first = ctypes.c_uint32()
        st = np.zeros(n, dtype=np.int32)
        self._check(self._lib.tbg_multi_load_pubkeys(self._h, _ptr(a), n, ctypes.byref(first), _ptr(st)),
                    "tbg_multi_load_pubkeys")
        return first.value, st

    def submit(self, op, duty_first, sigs, identifiers, **kw):
        b, keep, nd, np_ = self._batch(op, duty_first, sigs, identifiers, **kw)
        t = ctypes.c_uint64()
        self._check(self._lib.tbg_multi_submit(self._h, ctypes.byref(b), ctypes.byref(t)), "tbg_multi_submit")
        self._keep[t.value] = (nd, np_)
        return t.value

    def submit_group(self, op, batches):
        """Several batches (dicts of submit()'s arguments) as one multi-device
        launch (tbg_multi_submit_group): one ticket per batch."""
        built = [self._batch(op, **b) for b in batches]
        arr = (ctypes.POINTER(_native.TbgBatch) * len(built))(*[ctypes.pointer(b) for b, _, _, _ in built])
        t = np.zeros(len(built), dtype=np.uint64)
        self._check(self._lib.tbg_multi_submit_group(self._h, arr, len(built), _ptr(t)), "tbg_multi_submit_group")
        for ticket, (_, _, nd, np_) in zip(t.tolist(), built):
            self._keep[ticket] = (nd, np_)
        return t.tolist()

    def host_stats(self, reset=False) -> dict:
        """Host-side work of the multi-context's calls (tbg_multi_host_stats)."""
        out = np.zeros(16, dtype=np.uint64)
        rc = self._lib.tbg_multi_host_stats(self._h, _ptr(out), 1 if reset else 0)
        if rc != 0:
            raise EngineError(f"tbg_multi_host_stats: {self._lib.tbg_strerror(rc).decode()} ({rc})")
        return dict(zip(MULTI_HOST_STAT_KEYS, out.tolist()))

    def layout(self, ticket) -> list:
        out = np.zeros(self.size + 1, dtype=np.uint32)
        self._check(self._lib.tbg_multi_layout(self._h, ticket, _ptr(out)), "tbg_multi_layout")
        return out.tolist()

    def collect(self, ticket, block=True):
        nd, np_ = self._keep[ticket]
        ps = np.zeros(np_, dtype=np.int32)
        ds = np.zeros(nd, dtype=np.int32)
        agg = np.zeros((nd, 96), dtype=np.uint8)
        rc = self._lib.tbg_multi_collect(self._h, ticket, _ptr(ps), _ptr(ds), _ptr(agg), 1 if block else 0)
        if rc == E_PENDING:
            return None
        del self._keep[ticket]
        self._check(rc, "tbg_multi_collect")
        return BatchResult(ps, ds, agg)

    def run(self, op, duty_first, sigs, identifiers, **kw) -> BatchResult:
        return self.collect(self.submit(op, duty_first, sigs, identifiers, **kw))


class _BorrowedEngine(Engine):
    """An Engine over a context owned by a MultiEngine (tbg_multi_context)."""

    def __init__(self, lib, handle, device, parent):
        self._lib = lib
        self._parent = parent  # keeps the owning MultiEngine (and its contexts) alive
        self._h = ctypes.c_void_p(handle)
        self.device = device
        self.uid = next(_serial)
        self._keep = {}

    def close(self):
        self._h = None  # the multi-context destroys it


from .shard import shard_bounds  # noqa: E402,F401  (re-export)


_default = {}


def default_engine(device: int | None = None) -> Engine:
    import os
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    if device not in _default:
        _default[device] = Engine(device)
    return _default[device]
