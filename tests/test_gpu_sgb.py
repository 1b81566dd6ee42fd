"""The batched G2 subgroup test on the GPU (k_sgb.hip) against oracle/c.

Signatures crafted against random combinations (tests/golden/sgb_points.json:
13- and 23-torsion components, a bare torsion point, a pair whose components
cancel in a plain sum) and a random non-subgroup point are placed at the
first and last position of a group of 1,024 partials, two in one group, the
cancelling pair in one group, and the last partial of a short final group.
Every partial's status, every duty status and every aggregate must equal
oracle/c's per-item schedule (tblsconv.SigFromCore's subgroup check,
tblsconv/tblsconv.go:125-132, then tbls.VerifyAndAggregate), with the
batched test forced on, forced off, and in its adaptive mode.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
M = 1024  # SGB_M


def crafted_batch(engine):
    from tools.workload import invalid_pool, make_batch
    with open(os.path.join(HERE, "golden", "sgb_points.json")) as f:
        pts = {k: [bytes.fromhex(h) for h in v] for k, v in json.load(f)["points"].items()}
    b = make_batch(engine, 1500, 3, 4, seed=4242)  # 6000 partials: 5 full groups + one of 880
    n_p = len(b.sigs)
    place = {
        0: pts["t13"][0],                      # group 0, first member
        M - 1: pts["t23"][0],                  # group 0, last member
        M + 100: pts["torsion13"][0],          # group 1: two bad members
        M + 300: pts["t13"][1],
        2 * M + 7: pts["pair_a"][0],           # group 2: the cancelling pair
        2 * M + 8: pts["pair_b"][0],
        5 * M + 255: invalid_pool()["non_subgroup"][0],
        n_p - 1: pts["t13"][2],                # the short last group, last member
    }
    sigs = np.array(b.sigs, copy=True)
    for i, s in place.items():
        sigs[i] = np.frombuffer(s, dtype=np.uint8)
    b.sigs = sigs
    return b, sorted(place)


def run(engine, b):
    from charon_amd import engine as eng
    t = engine.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                      duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
    res = engine.collect(t)
    return res, engine.subgroup(t)


@pytest.fixture(scope="module")
def engines():
    from charon_amd import engine as eng
    es = {m: eng.Engine(0, slots=1, subgroup_batch=m) for m in (eng.SGB_ON, eng.SGB_OFF, eng.SGB_AUTO)}
    yield es
    for e in es.values():
        e.close()


def test_crafted_points_match_oracle_batched_and_alone(engines):
    from charon_amd import engine as eng
    from tests.test_gpu_fullsize import assert_same, oracle_run
    e_on, e_off = engines[eng.SGB_ON], engines[eng.SGB_OFF]
    b, bad = crafted_batch(e_on)
    res, sg = run(e_on, b)
    ref = oracle_run(b)
    assert_same(res, ref)
    assert np.flatnonzero(res.partial_status == eng.PS_ERR_SUBGROUP).tolist() == bad
    n_sg = (len(b.sigs) + M - 1) // M
    # the groups holding a crafted point failed; every other group passed whole
    assert sg == {"groups": n_sg, "failed": len({i // M for i in bad}), "group_size": M}, sg
    # the same batch with every signature tested alone: identical results
    b2, _ = crafted_batch(e_off)
    res2, sg2 = run(e_off, b2)
    assert sg2["groups"] == 0
    assert np.array_equal(res2.partial_status, res.partial_status)
    assert np.array_equal(res2.duty_status, res.duty_status) and np.array_equal(res2.agg, res.agg)


def sgb_plan(rho):
    """Mirror of tbls_engine.hip sgb_plan: (on, partials per group)."""
    best, m = None, None
    k = M
    while k >= 64:
        cost = 0.55 + 1.1 * 18 / k + 1 - (1 - min(rho, 1.0)) ** k
        if best is None or cost < best - 1e-12:
            best, m = cost, k
        k //= 2
    return best < 0.95, m


def test_adaptive_mode_group_size_and_off(engines):
    """The group size follows the non-subgroup share of collected batches
    (VERDICT r05 item 3): 1,024 while clean, smaller groups at a few per
    thousand, every signature alone past TBG_SGB_AUTO_MAX -- and back."""
    from charon_amd import engine as eng
    from tools.workload import make_batch
    e = engines[eng.SGB_AUTO]
    b, bad = crafted_batch(e)
    res, sg = run(e, b)  # first batch: clean history, groups of 1,024
    assert sg["groups"] > 0 and sg["failed"] == len({i // M for i in bad}) and sg["group_size"] == M
    assert np.flatnonzero(res.partial_status == eng.PS_ERR_SUBGROUP).tolist() == bad
    # 8 / 6000 non-subgroup partials (average 6.7e-4): smaller groups (256)
    ema = 0.5 * len(bad) / len(b.sigs)
    on, m = sgb_plan(ema)
    assert on and m < M
    clean = make_batch(e, 1500, 3, 4, seed=4343)
    res, sg = run(e, clean)
    assert sg == {"groups": -(-len(clean.sigs) // m), "failed": 0, "group_size": m}, sg
    assert (res.partial_status == eng.PS_VALID).all()
    ema *= 0.5
    # 2 % non-subgroup partials: past TBG_SGB_AUTO_MAX, the next batch tests every signature alone
    dense = make_batch(e, 1500, 3, 4, seed=4545)
    ns = invalid_nonsub()
    pos = np.arange(0, len(dense.sigs), 50)
    sigs = np.array(dense.sigs, copy=True)
    for k, i in enumerate(pos):
        sigs[i] = np.frombuffer(ns[k % len(ns)], dtype=np.uint8)
    dense.sigs = sigs
    res, sg = run(e, dense)
    assert np.flatnonzero(res.partial_status == eng.PS_ERR_SUBGROUP).tolist() == pos.tolist()
    ema = 0.5 * ema + 0.5 * len(pos) / len(sigs)
    assert not sgb_plan(ema)[0]
    res, sg = run(e, clean)
    assert sg["groups"] == 0 and (res.partial_status == eng.PS_VALID).all()
    # clean batches bring the average back down: groups of 1,024 again
    for _ in range(12):
        res, sg = run(e, clean)
    assert sg["groups"] > 0 and sg["failed"] == 0 and sg["group_size"] == M
    assert (res.partial_status == eng.PS_VALID).all()


def invalid_nonsub():
    from tools.workload import invalid_pool
    with open(os.path.join(HERE, "golden", "sgb_points.json")) as f:
        pts = {k: [bytes.fromhex(h) for h in v] for k, v in json.load(f)["points"].items()}
    return invalid_pool()["non_subgroup"] + pts["t13"] + pts["t23"] + pts["torsion13"]


def test_config5_density_matches_oracle(engines):
    """Config 5's non-subgroup density (1/8 of 1 % = 1.25e-3 of the partials,
    VERDICT r05 item 3) in a 16k-partial batch, twice on an automatic-mode
    context: first at 1,024 per group (clean history), then at the size the
    collected share picks (256); both runs' verdicts equal oracle/c's."""
    from charon_amd import engine as eng
    from tests.test_gpu_fullsize import assert_same, oracle_run
    from tools.workload import make_batch
    e = eng.Engine(0, slots=1, subgroup_batch=eng.SGB_AUTO)
    try:
        b = make_batch(e, 4000, 3, 4, seed=4646)
        rng = np.random.default_rng(4747)
        n_bad = round(1.25e-3 * len(b.sigs))
        pos = np.sort(rng.choice(len(b.sigs), size=n_bad, replace=False))
        ns = invalid_nonsub()
        sigs = np.array(b.sigs, copy=True)
        for k, i in enumerate(pos):
            sigs[i] = np.frombuffer(ns[k % len(ns)], dtype=np.uint8)
        b.sigs = sigs
        ref = oracle_run(b)
        res, sg = run(e, b)
        assert sg["group_size"] == M and sg["failed"] == len({int(i) // M for i in pos})
        assert_same(res, ref)
        assert np.flatnonzero(res.partial_status == eng.PS_ERR_SUBGROUP).tolist() == pos.tolist()
        on, m = sgb_plan(0.5 * n_bad / len(sigs))
        assert on and m < M
        res, sg = run(e, b)
        assert sg["group_size"] == m and sg["groups"] == -(-len(sigs) // m)
        assert sg["failed"] == len({int(i) // m for i in pos})
        assert_same(res, ref)
    finally:
        e.close()


def test_small_batches_test_each_signature(engines):
    from charon_amd import engine as eng
    from tools.workload import make_batch
    e = engines[eng.SGB_ON]
    b = make_batch(e, 200, 3, 4, seed=4444)  # 800 partials < 2 groups: no batched test
    res, sg = run(e, b)
    assert sg["groups"] == 0 and (res.partial_status == eng.PS_VALID).all()
