"""Sharding of a batch of DV-duties over devices or ranks, and the gather of
the results back into caller order.

Duties are independent (no cross-device math), so a batch is
cut into contiguous duty ranges of about equal partial counts.  This is the
host-side mirror of what tbg_multi_submit / tbg_multi_collect do inside the
library (charon_amd/csrc/tbls_multi.hip) for one process driving several
GPUs, and what a multi-rank deployment (one process per GPU, bench.py under
torch.distributed.run) does across processes.  The gathered order is the
per-DV loop order of the reference (core/parsigex/parsigex.go:101-107,
core/parsigdb/memory.go:96-134 -> core/sigagg/sigagg.go:53-103).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def shard_bounds(duty_first, n_shards: int) -> list:
    """Duty cut points: shard i starts at the first duty whose first partial
    index is >= i * np // n (duties are never split); with no partials at all
    duties are split evenly.  Same rule as tbls_multi.hip."""
    duty_first = np.asarray(duty_first, dtype=np.int64)
    nd, np_ = len(duty_first) - 1, int(duty_first[-1])
    lo = [0]
    for i in range(1, n_shards):
        d = int(np.searchsorted(duty_first, np_ * i // n_shards, side="left")) if np_ else nd * i // n_shards
        lo.append(max(lo[-1], min(d, nd)))
    return lo + [nd]


def group_shard_bounds(duty_firsts, n_shards: int) -> list:
    """tbg_multi_submit_group's cut of several batches taken back to back:
    shard_bounds over the concatenated duties, then each batch's own cut
    points (clamped to its duties) -- one list of n_shards + 1 per batch, what
    tbg_multi_layout reports for that batch's ticket."""
    dfs = [np.asarray(d, dtype=np.int64) for d in duty_firsts]
    d_base = np.cumsum([0] + [len(d) - 1 for d in dfs])
    p_base = np.cumsum([0] + [int(d[-1]) for d in dfs])
    glob = np.concatenate([d[:-1] + p for d, p in zip(dfs, p_base[:-1])] + [[p_base[-1]]])
    cut = shard_bounds(glob, n_shards)
    return [[int(min(max(c, d_base[k]), d_base[k + 1]) - d_base[k]) for c in cut] for k in range(len(dfs))]


@dataclass
class SubBatch:
    """Duties [d0, d1) of a batch as a batch of its own (tbg_batch fields)."""
    d0: int
    d1: int
    p0: int
    p1: int
    duty_first: np.ndarray
    sigs: np.ndarray
    identifiers: np.ndarray
    pubkey_ids: np.ndarray | None
    duty_threshold: np.ndarray | None
    msg_data: np.ndarray | None
    msg_off: np.ndarray | None
    duty_msg: np.ndarray | None


def sub_batch(d0, d1, duty_first, sigs, identifiers, pubkey_ids=None, duty_threshold=None, msg_data=None,
              msg_off=None, duty_msg=None) -> SubBatch:
    """Slice duties [d0, d1): partial arrays by offset, duty_first rebased,
    and the messages the range uses re-indexed in order of first use."""
    duty_first = np.asarray(duty_first, dtype=np.int64)
    p0, p1 = int(duty_first[d0]), int(duty_first[d1])
    sb = SubBatch(d0, d1, p0, p1, (duty_first[d0:d1 + 1] - p0).astype(np.uint32), np.asarray(sigs)[p0:p1],
                  np.asarray(identifiers)[p0:p1], None, None, None, None, None)
    if pubkey_ids is not None:
        sb.pubkey_ids = np.asarray(pubkey_ids)[p0:p1]
    if duty_threshold is not None:
        sb.duty_threshold = np.asarray(duty_threshold)[d0:d1]
    if duty_msg is not None:
        dm = np.asarray(duty_msg, dtype=np.int64)[d0:d1]
        used, first_pos = np.unique(dm, return_index=True)
        order = used[np.argsort(first_pos)]            # messages in order of first use
        local = {int(m): i for i, m in enumerate(order)}
        msg_off = np.asarray(msg_off, dtype=np.int64)
        data = np.asarray(msg_data, dtype=np.uint8)
        parts = [data[msg_off[m]:msg_off[m + 1]] for m in order]
        lens = [len(p) for p in parts]
        sb.msg_data = np.concatenate(parts + [np.zeros(1, np.uint8)])
        sb.msg_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
        sb.duty_msg = np.array([local[int(m)] for m in dm], dtype=np.uint32)
    return sb


def gather(parts, n_duties: int, n_partials: int):
    """Reassemble per-shard results [(sub_batch, partial_status, duty_status,
    agg)] into caller-order arrays."""
    ps = np.zeros(n_partials, dtype=np.int32)
    ds = np.zeros(n_duties, dtype=np.int32)
    agg = np.zeros((n_duties, 96), dtype=np.uint8)
    seen = np.zeros(n_duties, dtype=bool)
    for sb, p, d, a in parts:
        assert not seen[sb.d0:sb.d1].any(), "overlapping shards"
        seen[sb.d0:sb.d1] = True
        ps[sb.p0:sb.p1] = p
        ds[sb.d0:sb.d1] = d
        agg[sb.d0:sb.d1] = a
    assert seen.all(), "a duty range is missing from the gather"
    return ps, ds, agg
