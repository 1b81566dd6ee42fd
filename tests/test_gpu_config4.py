"""BASELINE config 4 as configured: 1,000,000 3-of-4 DV-duties with 1 % mixed
invalid partials, cut 8 ways through the one-process multi-device API
(tbg_multi_*) and gathered back into caller order by the host.

The box has one GPU, so the 8 shards are 8 contexts on that device (one slot
each), the layout of a Charon node that owns 8 GPUs (include/tbls_gpu.h,
SURVEY.md 8e).  The 1M-DV batch goes in as FOUR caller batches of unequal
size through tbg_multi_submit_group (the fan-in of concurrent peer sets,
core/parsigex/parsigex.go:101-107): the 8-way cut runs over the four batches
taken back to back, each context packs its pieces into one device batch, and
every caller ticket is gathered on its own.

Checked:
  * the cut points each ticket reports equal the host mirror
    (charon_amd.shard.group_shard_bounds), uneven last shard included;
  * the WHOLE batch by properties: a partial verifies iff it was not
    injected, every injected kind gets its reference outcome, a duty
    aggregates iff it kept t valid partials and then to the group signature;
  * oracle/c (the CPU restatement of tbls.VerifyAndAggregate, tss.go:153-187)
    bit-exact on two 10k-DV slices that straddle shard cuts.
"""
import time

import numpy as np
import pytest

from conftest import progress
from test_gpu_fullsize import assert_same, oracle_run

pytestmark = pytest.mark.gpu

N_DV = 1_000_000
N_CTX = 8
# four caller batches of unequal size (sum N_DV)
SPLIT = (400_000, 250_000, 250_000, 100_000)


@pytest.fixture(scope="module")
def config4():
    from charon_amd import engine as eng
    from tools.workload import make_mixed_batch
    # contexts of earlier modules' default engines are closed first: this
    # module opens 8 contexts of its own on the one device
    for e in list(eng._default.values()):
        e.close()
    eng._default.clear()
    m = eng.MultiEngine([0] * N_CTX, slots=1)
    try:
        assert m.size == N_CTX
        t0 = time.time()
        # vectors are generated on context 0 of the multi-context itself
        b = make_mixed_batch(m.context(0), N_DV, seed=404, inject=0.01, thresholds=((3, 4),), load=m.load_pubkeys)
        progress(f"config4: 1M-DV batch generated in {time.time() - t0:.1f} s")
        yield m, b
    finally:
        m.close()


def _split_args(b):
    """The four caller batches of the 1M-DV batch (messages re-indexed per batch)."""
    from charon_amd.shard import sub_batch
    out, d0 = [], 0
    for n in SPLIT:
        sb = sub_batch(d0, d0 + n, b.duty_first, b.sigs, b.identifiers, pubkey_ids=b.pubkey_ids,
                       duty_threshold=b.threshold, msg_data=b.msg_data, msg_off=b.msg_off, duty_msg=b.duty_msg)
        out.append((d0, sb))
        d0 += n
    return out


def test_config4_1m_dvs_cut_8_ways_with_host_gather(config4):
    from charon_amd import engine as eng
    from charon_amd.shard import group_shard_bounds, shard_bounds
    from tools.workload import INJECT_KINDS
    m, b = config4
    parts = _split_args(b)
    args = [dict(duty_first=sb.duty_first, sigs=sb.sigs, identifiers=sb.identifiers, msgs=(sb.msg_data, sb.msg_off),
                 duty_msg=sb.duty_msg, pubkey_ids=sb.pubkey_ids, duty_threshold=sb.duty_threshold)
            for _, sb in parts]
    t0 = time.time()
    tickets = m.submit_group(eng.OP_VERIFY_AGGREGATE, args)
    layouts = [m.layout(t) for t in tickets]
    assert layouts == group_shard_bounds([sb.duty_first for _, sb in parts], N_CTX)
    # the cut over the four batches back to back is the cut of the whole 1M
    # batch: every context holds ~125k DVs (duties are never split)
    cut = shard_bounds(b.duty_first, N_CTX)
    inner = {d0 + c for (d0, _), lo in zip(parts, layouts) for c in lo if 0 < c < lo[-1]}
    assert inner == set(cut[1:-1])
    assert max(np.diff(cut)) - min(np.diff(cut)) <= 2
    # gather: each caller ticket into the caller's order (collected out of order)
    ps = np.zeros(len(b.identifiers), dtype=np.int32)
    ds = np.zeros(N_DV, dtype=np.int32)
    agg = np.zeros((N_DV, 96), dtype=np.uint8)
    for (d0, sb), t in reversed(list(zip(parts, tickets))):
        r = m.collect(t)
        ps[sb.p0:sb.p1] = r.partial_status
        ds[d0:d0 + len(sb.duty_first) - 1] = r.duty_status
        agg[d0:d0 + len(sb.duty_first) - 1] = r.agg
    progress(f"config4: 1M DVs through 8 contexts in {time.time() - t0:.1f} s (PCIe and host packing included)")
    # the whole batch by properties
    assert np.array_equal(ps == eng.PS_VALID, ~b.injected)
    want = {"wrong_msg": {eng.PS_INVALID}, "wrong_share": {eng.PS_INVALID},
            "random_bytes": {eng.PS_ERR_FLAGS, eng.PS_ERR_FIELD, eng.PS_ERR_CURVE, eng.PS_ERR_SUBGROUP,
                             eng.PS_ERR_IDENTITY},
            "non_subgroup": {eng.PS_ERR_SUBGROUP}, "off_curve": {eng.PS_ERR_CURVE}, "bad_flags": {eng.PS_ERR_FLAGS},
            "identity": {eng.PS_ERR_IDENTITY}, "missing_pubshare": {eng.PS_ERR_PUBKEY}}
    for k, name in enumerate(INJECT_KINDS):
        got = set(np.unique(ps[b.inject_kind == k]).tolist())
        assert got and got <= want[name], (name, got)
    ok = ds == eng.DS_OK
    assert np.array_equal(ok, b.expect_ok)
    assert np.array_equal(agg[ok], b.group_sig[ok])
    assert set(np.unique(ds[~ok]).tolist()) <= {eng.DS_INSUFFICIENT_VALID, eng.DS_DECODE}
    # oracle/c on two 10k-DV slices that straddle shard cuts (the first cut of
    # the first caller batch, and the cut nearest the batch boundary at 650k)
    cuts = [d0 + c for (d0, _), lo in zip(parts, layouts) for c in lo[1:-1] if 0 < c]
    c1 = cuts[0]
    c2 = min(cuts, key=lambda c: abs(c - 650_000))
    res = eng.BatchResult(ps, ds, agg)
    for c in (c1, c2):
        s0 = max(0, c - 5000)
        assert_same(res, oracle_run(b, s0, s0 + 10000), s0, s0 + 10000, int(b.duty_first[s0]))
        progress(f"config4: oracle/c slice [{s0}, {s0 + 10000}) bit-exact")


def test_config4_single_ticket_matches_group(config4):
    """tbg_multi_submit of one 100k-DV caller batch (cut 8 ways on its own)
    gives the same statuses and aggregates as the grouped submit's pieces."""
    from charon_amd import engine as eng
    from charon_amd.shard import shard_bounds
    m, b = config4
    d0, sb = _split_args(b)[3]
    t = m.submit(eng.OP_VERIFY_AGGREGATE, sb.duty_first, sb.sigs, sb.identifiers, msgs=(sb.msg_data, sb.msg_off),
                 duty_msg=sb.duty_msg, pubkey_ids=sb.pubkey_ids, duty_threshold=sb.duty_threshold)
    assert m.layout(t) == shard_bounds(sb.duty_first, N_CTX)
    r = m.collect(t)
    inj = b.injected[sb.p0:sb.p1]
    assert np.array_equal(r.partial_status == eng.PS_VALID, ~inj)
    ok = r.duty_status == eng.DS_OK
    n = len(sb.duty_first) - 1
    assert np.array_equal(ok, b.expect_ok[d0:d0 + n])
    assert np.array_equal(r.agg[ok], b.group_sig[d0:d0 + n][ok])
