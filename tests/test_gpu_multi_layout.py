"""tbg_multi_submit_group's cut in the C++ library against its host mirror
(charon_amd.shard.group_shard_bounds) on irregular tiny batches:
duties with no partials at batch boundaries, batches whose duties have no
partials at all (NP == 0), cut targets that fall exactly on a batch's first
partial -- the shapes tests/test_shard_dist.py fuzzes on the mirror alone.
Every ticket's layout (tbg_multi_layout) must equal the mirror's, and every
batch must still collect (the sub-batches were valid).  Three contexts on
device 0; OP_AGGREGATE, so no keys or messages are needed."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_multi_layout_matches_mirror_on_irregular_batches():
    from charon_amd import engine as eng
    from charon_amd.shard import group_shard_bounds
    with open(os.path.join(HERE, "golden", "cfg1_3of4_single.json")) as f:
        v = json.load(f)["vectors"][0]
    sig = np.frombuffer(bytes.fromhex(v["partials"][0]["sig"]), np.uint8)
    n_ctx = 3
    m = eng.MultiEngine([0] * n_ctx, slots=2)
    try:
        rng = np.random.default_rng(11)
        shapes = []
        for trial in range(40):
            k = int(rng.integers(1, 5))
            dfs = []
            for _ in range(k):
                nd = int(rng.integers(1, 24))
                counts = rng.integers(0, 6, size=nd) * (rng.random(nd) < 0.8)
                if rng.random() < 0.15:
                    counts[:] = 0  # a batch with no partials
                if nd > 1 and rng.random() < 0.3:
                    counts[0] = counts[-1] = 0  # empty duties at the boundaries
                dfs.append(np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32))
            shapes.append(dfs)
        # a cut target equal to a batch's first partial: 2 batches of 6 partials, 2 shards
        shapes.append([np.array([0, 3, 6], np.uint32), np.array([0, 3, 6], np.uint32)])
        for dfs in shapes:
            calls = []
            for d in dfs:
                n_p = int(d[-1])
                calls.append(dict(duty_first=d, sigs=np.tile(sig, (n_p, 1)) if n_p else np.zeros((0, 96), np.uint8),
                                  identifiers=np.tile(np.arange(1, 5, dtype=np.uint8), n_p)[:n_p]))
            ts = m.submit_group(eng.OP_AGGREGATE, calls)
            want = group_shard_bounds(dfs, n_ctx)
            got = [m.layout(t) for t in ts]
            assert got == want, (dfs, got, want)
            for t, d in zip(ts, dfs):
                r = m.collect(t)
                assert len(r.partial_status) == int(d[-1]) and len(r.duty_status) == len(d) - 1
    finally:
        m.close()


def test_borrowed_context_fails_loudly_after_close():
    """a per-context Engine handed out by MultiEngine.context keeps
    its owner alive, and once the owner is closed a call through it raises
    instead of reaching freed native memory."""
    import gc

    from charon_amd import engine as eng
    e = eng.MultiEngine([0, 0], slots=1).context(1)
    gc.collect()  # the MultiEngine is only reachable through e
    assert e.pubkey_count == 0
    e._parent.close()
    with pytest.raises(eng.EngineError):
        e.host_stats()
