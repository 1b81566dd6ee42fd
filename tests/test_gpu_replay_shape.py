"""tbg_replay_plan with the level-0 shape of the launches it runs together
(tbls_engine.hip: l0_shape over their duties, applied where each slot's
arena fits it).  Three slots of 16 caller batches of 2,500 3-of-4 DVs
(40k duties each, submitted at (G, C) = (16, 4)) replayed as the bench's
prefixes of 7 + 7 + 6 batches: 50k duties together take (14, 7).  Level 0
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
    import torch
    from charon_amd import engine as eng
    from tests.test_gpu_shape import expected_shape
    from tools.workload import make_batch
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count  # (before the engine's own HIP calls)
    assert expected_shape(DVS * PER_SLOT, n_cu) == (16, 4)
    assert expected_shape(DVS * sum(PREFIX), n_cu) == (14, 7)
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
