"""The level-0 launch shape (tbls_engine.hip l0_shape):
a level-0 launch whose Miller hexads at (G, C) = (16, 4) need more than one
round of the device's wave slots takes the (G, C) with the fewest rounds x
hexad length (round 6: one-chunk groups of 5 .. 10 duties among the
candidates).  Config 4's 125k-DV shard runs at (14, 7) on MI355X, and its
verdicts -- level 0 passing, and one wrong-share partial found through the
G = 14 group levels -- equal the known answers and oracle/c on a 10k slice."""
import numpy as np
import pytest

from tests.conftest import progress
from tests.test_gpu_fullsize import assert_same, oracle_run
from tests.test_gpu_headline import _call, _known_answer

pytestmark = pytest.mark.gpu
DVS = 125000


def shape_fits(nd0, G0, C0, nd, G, C):
    """Mirror of l0_shape_fits: a launch of nd duties at (G, C) in an arena
    sized for nd0 duties at (G0, C0)."""
    ng0, nch0 = -(-nd0 // G0), -(-G0 // C0)
    ng, nch = -(-nd // G), -(-G // C)
    return (ng <= ng0 and ng * (nch + 1) <= ng0 * (nch0 + 1) and ng * nch <= ng0 * nch0
            and ng * nch * C <= ng0 * nch0 * C0 and ng * G <= ng0 * G0
            and max(ng * nch, nd) <= max(ng0 * nch0, nd0) and (G <= 64) == (G0 <= 64))


def expected_shape(nd, n_cu, g_free=True, G=16, fits=lambda g, c: True):
    """Mirror of l0_shape: the hexad cost 0.948 + 1.395 C (M u32 mul-adds,
    profiles/work_model.json) x ceil(waves / SIMDs), SIMDs = CUs x 4, over the
    candidates `fits` keeps (a replay's arenas)."""
    n_simd = n_cu * 4

    def cost(g, c):
        waves = -(-(-(-nd // g) * -(-g // c)) // 10)
        return (0.948 + 1.395 * c) * -(-waves // n_simd)

    if G < 8:
        return G, 4
    cand = [(16 if g_free else G, 4), (16 if g_free else G, 8)] + ([(14, 7)] if g_free else [])
    if g_free:
        cand += [(c, c) for c in range(5, 11)]  # round 6: one chunk per group, 5 .. 10 duties
    best = None
    for gc in cand:
        if fits(*gc) and (best is None or cost(*gc) < cost(*best) - 1e-9):
            best = gc
    return best


def test_shape_mirror():
    # round 6: one-chunk groups of 5 .. 10 duties fill whole wave-slot rounds
    assert expected_shape(160000, 256) == (16, 8)
    assert expected_shape(125000, 256) == (14, 7)  # config 4's shard
    assert expected_shape(10000, 256) == (16, 4)
    assert expected_shape(100000, 256) == (10, 10)  # config 3's launch: 1,000 waves, one round
    assert expected_shape(125000, 256, g_free=False, G=16) == (16, 8)
    # the 20-step bench plan: 7 + 7 + 6 batches of the (16, 8) slots replayed together
    fits = lambda g, c: all(shape_fits(160000, 16, 8, n, g, c) for n in (70000, 70000, 60000))  # noqa: E731
    assert expected_shape(200000, 256, fits=fits) == (10, 10)
    assert expected_shape(480000, 256) == (16, 8)


@pytest.fixture(scope="module")
def shard():
    from charon_amd import engine as eng
    from tools.workload import make_batch
    n_cu = eng.device_cu_count(0)
    e = eng.Engine(0, slots=1)  # group size and chunk not configured: the engine picks them
    b = make_batch(e, DVS, 3, 4, seed=4125)
    yield e, b, n_cu
    e.close()


def _submit(e, b):
    from charon_amd import engine as eng
    t = e.submit(eng.OP_VERIFY_AGGREGATE, **_call(b))
    return t, e.collect(t)


def test_config4_shard_shape_level0_passes(shard):
    from charon_amd import engine as eng
    e, b, n_cu = shard
    t, res = _submit(e, b)
    G, C = expected_shape(DVS, n_cu)
    sh = e.shape(t)
    progress(f"shape {sh}")
    assert (sh["group"], sh["chunk"], sh["level0"]) == (G, C, 1)
    assert sh["chunks"] == -(-DVS // G) * -(-G // C)
    assert e.level0(t) == eng.L0_PASSED
    _known_answer(res, b)
    s0 = 60000
    assert_same(res, oracle_run(b, s0, s0 + 10000), s0, s0 + 10000, int(b.duty_first[s0]))


def test_config4_shard_shape_one_invalid_partial(shard):
    from dataclasses import replace
    from charon_amd import engine as eng
    e, b, _ = shard
    rng = np.random.default_rng(125)
    i = int(rng.integers(0, len(b.identifiers)))
    d = i // 4
    sigs = b.sigs.copy()
    sigs[i] = b.sigs[4 * d + (i - 4 * d + 1) % 4]  # wrong share
    injected = b.injected.copy()
    injected[i] = True
    bad = replace(b, sigs=sigs, injected=injected, expect_ok=b.expect_ok.copy())
    t, res = _submit(e, bad)
    assert e.level0(t) == eng.L0_FAILED
    assert e.shape(t)["chunk"] > 4  # the group levels ran on the wide launch shape
    assert np.flatnonzero(res.partial_status != eng.PS_VALID).tolist() == [i]
    _known_answer(res, bad)
    s0 = max(0, min(d - 5000, DVS - 10000))
    assert_same(res, oracle_run(bad, s0, s0 + 10000), s0, s0 + 10000, int(bad.duty_first[s0]))
