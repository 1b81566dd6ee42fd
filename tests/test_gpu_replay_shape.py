"""tbg_replay_plan with the level-0 shape of the launches it runs together
(tbls_engine.hip: l0_shape over their duties, applied where each slot's
arena fits it).  Three slots of 16 caller batches of 2,500 3-of-4 DVs
(40k duties each, submitted at (G, C) = (16, 4)) replayed as the bench's
prefixes of 7 + 7 + 6 batches: 50k duties together take the cheapest shape
every launch's arena holds -- (14, 7), where (5, 5), cheaper, would need
more groups than the (16, 4) arenas have (round 6).  Level 0
must still PASS on the clean slots and FAIL on the slot holding one
wrong-share partial, and every replayed batch must equal its known answer
(the fallback levels run at the replay's shape too)."""
from dataclasses import replace

import numpy as np
import pytest

from tests.test_gpu_headline import _call, _known_answer

pytestmark = pytest.mark.gpu
SLOTS, PER_SLOT, DVS = 3, 16, 2500
PREFIX = [7, 7, 6]


def test_replay_plan_reshaped_launches():
    from charon_amd import engine as eng
    from tests.test_gpu_shape import expected_shape, shape_fits
    from tools.workload import make_batch
    n_cu = eng.device_cu_count(0)
    assert expected_shape(DVS * PER_SLOT, n_cu) == (16, 4)
    assert expected_shape(DVS * sum(PREFIX), n_cu) == (5, 5)
    fits = lambda g, c: all(shape_fits(DVS * PER_SLOT, 16, 4, DVS * n, g, c) for n in PREFIX)  # noqa: E731
    assert expected_shape(DVS * sum(PREFIX), n_cu, fits=fits) == (14, 7)
    e = eng.Engine(0, slots=SLOTS)
    try:
        groups = [[make_batch(e, DVS, 3, 4, seed=9000 + 100 * s + k) for k in range(PER_SLOT)] for s in range(SLOTS)]
        # one wrong-share partial in slot 1, batch 3 (inside its replayed prefix)
        b = groups[1][3]
        i = 4 * 1234 + 2
        sigs = b.sigs.copy()
        sigs[i] = b.sigs[i - 1]
        inj = b.injected.copy()
        inj[i] = True
        groups[1][3] = replace(b, sigs=sigs, injected=inj, expect_ok=b.expect_ok.copy())
        tickets = []
        for g in groups:
            ts = e.submit_group(eng.OP_VERIFY_AGGREGATE, [_call(x) for x in g])
            tickets.append(ts)
        for ts, g in zip(tickets, groups):
            for t, x in zip(ts, g):
                _known_answer(e.collect(t), x)
        assert [e.shape(ts[0])["chunk"] for ts in tickets] == [4, 4, 4]
        e.replay_plan([ts[0] for ts in tickets], PREFIX)
        assert [(e.shape(ts[0])["group"], e.shape(ts[0])["chunk"]) for ts in tickets] == [(14, 7)] * 3
        assert e.level0(tickets[0][0]) == eng.L0_PASSED
        assert e.level0(tickets[1][0]) == eng.L0_FAILED
        assert e.level0(tickets[2][0]) == eng.L0_PASSED
        for ts, g, n in zip(tickets, groups, PREFIX):
            for t, x in zip(ts[:n], g[:n]):
                _known_answer(e.fetch(t, x.n_dv, len(x.identifiers)), x)
        r = e.fetch(tickets[1][3], groups[1][3].n_dv, len(groups[1][3].identifiers))
        assert np.flatnonzero(r.partial_status != eng.PS_VALID).tolist() == [i]
    finally:
        e.close()


def test_replay_prefix_keeps_shape_its_chunk_arena_cannot_hold():
    """a replay may only reshape a launch where EVERY
    group / chunk section of the slot's arena holds the new shape.  A slot
    submitted as 90k + 70k duties is sized at (16, 8) (20,000 chunks); its
    90k-duty prefix takes the cheapest shape that arena holds -- never (16,
    4) (22,500 chunks, more than the chunk lists and chunk values hold, the
    overflow ADVICE r05 found), which the prefix alone would otherwise take.  With 20 % invalid partials nearly every
    group fails level 0 and level 1, so the chunk-level kernels write every
    chunk slot: the prefix must still equal its known answer."""
    from charon_amd import engine as eng
    from tests.test_gpu_shape import expected_shape, shape_fits
    from tools.workload import make_batch
    n_cu = eng.device_cu_count(0)
    assert expected_shape(160000, n_cu) == (16, 8)
    assert not shape_fits(160000, 16, 8, 90000, 16, 4)
    G, C = expected_shape(90000, n_cu, fits=lambda g, c: shape_fits(160000, 16, 8, 90000, g, c))
    assert (G, C) != (16, 4)
    e = eng.Engine(0, slots=1, rlc_batch=eng.RLC_L0_ON)
    try:
        a = make_batch(e, 90000, 3, 4, seed=9901, inject=0.2)
        b = make_batch(e, 70000, 3, 4, seed=9902, inject=0.2)
        ta, tb = e.submit_group(eng.OP_VERIFY_AGGREGATE, [_call(a), _call(b)])
        _known_answer(e.collect(ta), a)
        _known_answer(e.collect(tb), b)
        assert (e.shape(ta)["group"], e.shape(ta)["chunk"]) == (16, 8)
        assert e.level0(ta) == eng.L0_FAILED
        e.replay_plan([ta], [1])
        # the launch ran at the cheapest shape its arena holds, over the prefix's duties
        sh = e.shape(ta)
        assert (sh["group"], sh["chunk"]) == (G, C) and shape_fits(160000, 16, 8, 90000, G, C)
        assert sh["chunks"] == -(-90000 // G) * -(-G // C)
        _known_answer(e.fetch(ta, a.n_dv, len(a.identifiers)), a)
    finally:
        e.close()


def test_express_slot_yields_to_the_stream_bound():
    """slots x streams_per_slot at the stream bound leaves
    no stream for the express slot; the context runs without one instead of
    being refused."""
    from charon_amd import engine as eng
    e = eng.Engine(0, slots=8, streams_per_slot=2)  # 16 streams: TBG_MAX_SLOT_STREAMS
    e.close()
