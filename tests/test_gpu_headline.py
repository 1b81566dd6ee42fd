"""GPU parity at the bench's headline launch shape and at config 3's stated
size (VERDICT r02 "What's weak": the 16 x 10k-DV level-0 launch was only
checked by bench.py against the engine's own signer).

  * 16 caller batches of 10,000 3-of-4 DVs packed by ONE tbg_submit_group
    (640,000 partials, ~78 bucket entries per level-0 bucket, multi-slice
    bucket sums), level 0 forced on: the batch-wide check PASSES and the
    first and last 10k batches equal oracle/c bit for bit (every other batch
    against its known answer);
  * the same group with ONE wrong-share partial at a seeded position: level 0
    FAILS, the fallback levels find exactly that partial, the affected 10k
    batch equals oracle/c bit for bit (per-partial and per-duty verdicts,
    aggregates), every other batch its known answer (reference tss.go:153-187,
    parsigex.go:101-107);
  * config 3 at its stated size: one 100,000-DV 7-of-10 batch (1,000,000
    partials, 1 % wrong-message partials) through the property checks, and
    oracle/c on a 10,000-DV slice;
  * the C-ABI thread test (tests/cabi/cabi_threads.c: 8 threads submitting,
    polling and collecting through the header, as the cgo binding does).
"""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import progress
from tests.test_gpu_fullsize import assert_same, oracle_run

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
N_BATCHES, DVS = 16, 10000


def _call(b):
    return dict(duty_first=b.duty_first, sigs=b.sigs, identifiers=b.identifiers, msgs=(b.msg_data, b.msg_off),
                duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)


def _known_answer(res, b):
    """Every partial verifies iff it was not injected; every duty with t valid
    partials aggregates to the group signature (tbg_sign of the group secret)."""
    from charon_amd import engine as eng
    assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
    ok = res.duty_status == eng.DS_OK
    assert np.array_equal(ok, b.expect_ok)
    assert np.array_equal(res.agg[ok], b.group_sig[ok])


@pytest.fixture(scope="module")
def l0_engine():
    from charon_amd import engine as eng
    e = eng.Engine(0, slots=1, rlc_group=16, rlc_batch=eng.RLC_L0_ON)
    yield e
    e.close()


@pytest.fixture(scope="module")
def headline_batches(l0_engine):
    from tools.workload import make_batch
    return [make_batch(l0_engine, DVS, 3, 4, seed=7100 + k) for k in range(N_BATCHES)]


def test_headline_group_level0_passes_and_matches_oracle(l0_engine, headline_batches):
    from charon_amd import engine as eng
    e, bs = l0_engine, headline_batches
    ts = e.submit_group(eng.OP_VERIFY_AGGREGATE, [_call(b) for b in bs])
    res = [e.collect(t) for t in ts]
    assert e.level0(ts[0]) == eng.L0_PASSED
    st = e.stats(ts[0])
    assert st["partial_checks"] == 0 and st["duty_checks"] == 0  # nothing fell back
    for r, b in zip(res, bs):
        _known_answer(r, b)
    for k in (0, N_BATCHES - 1):
        assert_same(res[k], oracle_run(bs[k]))


def test_headline_group_one_invalid_partial(l0_engine, headline_batches):
    from charon_amd import engine as eng
    e, bs = l0_engine, list(headline_batches)
    rng = np.random.default_rng(4242)
    k = int(rng.integers(1, N_BATCHES - 1))
    bad = bs[k]
    i = int(rng.integers(0, len(bad.identifiers)))
    d = i // 4
    # wrong share: partial i carries the signature of another share of its DV
    j = 4 * d + (i - 4 * d + 1) % 4
    sigs = bad.sigs.copy()
    sigs[i] = bad.sigs[j]
    injected = bad.injected.copy()
    injected[i] = True
    from dataclasses import replace
    bad = replace(bad, sigs=sigs, injected=injected, expect_ok=bad.expect_ok.copy())  # 3 of 4 still valid
    bs[k] = bad
    ts = e.submit_group(eng.OP_VERIFY_AGGREGATE, [_call(b) for b in bs])
    res = [e.collect(t) for t in ts]
    assert e.level0(ts[0]) == eng.L0_FAILED
    assert res[k].partial_status[i] == eng.PS_INVALID
    assert np.flatnonzero(res[k].partial_status != eng.PS_VALID).tolist() == [i]
    for r, b in zip(res, bs):
        _known_answer(r, b)
    assert_same(res[k], oracle_run(bad))


def test_config3_100k_7of10(l0_engine):
    """BASELINE config 3 at its stated size on the HIP path (default engine
    schedule), property-checked in full and oracle-checked on a slice."""
    import time
    from charon_amd import engine as eng
    from tools.workload import make_batch
    e = eng.Engine(0, slots=1)
    try:
        t0 = time.time()
        b = make_batch(e, 100000, 7, 10, seed=3100, inject=0.01)
        assert len(b.identifiers) == 1000000
        progress(f"config3: batch generated ({time.time() - t0:.1f} s)")
        res = e.run(eng.OP_VERIFY_AGGREGATE, **_call(b))
        progress(f"config3: engine run done ({time.time() - t0:.1f} s)")
        _known_answer(res, b)
        s0 = 45000
        assert_same(res, oracle_run(b, s0, s0 + 10000), s0, s0 + 10000, int(b.duty_first[s0]))
        progress(f"config3: oracle slice checked ({time.time() - t0:.1f} s)")
    finally:
        e.close()


def test_cabi_threads():
    """tests/cabi/cabi_threads.c through the C ABI from 8 threads (plain build)."""
    exe = os.path.join(HERE, "cabi", "cabi_threads")
    src = os.path.join(HERE, "cabi", "cabi_threads.c")
    lib = os.path.join(os.path.dirname(HERE), "charon_amd", "libtbls_gpu.so")
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(lib)):
        subprocess.run(["make", "-C", os.path.join(HERE, "cabi"), "cabi_threads"], check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "cabi_threads: PASS" in r.stdout
