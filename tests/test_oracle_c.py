"""The C restatement (oracle/c) against the pinned Python oracle and the
golden fixtures.  Both are test infrastructure; the C one is fast enough to
check the HIP engine at batch scale (tests/test_gpu_parity.py) and is the
timed CPU port of bench.py's cpu_baseline."""
import json
import os
import random

import numpy as np
import pytest

from oracle import bls12_381 as bls
from oracle import c as oc
from oracle import tbls_oracle as tb

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
PS_NAMES = {1: "valid", 0: "invalid", -1: "err_flags", -2: "err_field", -3: "err_curve", -4: "err_subgroup",
            -5: "err_identity", -6: "err_pubkey"}
DS_NAMES = {0: "ok", -20: "insufficient", -21: "insufficient_valid", -22: "too_few", -23: "duplicate",
            -24: "identity", -25: "decode"}


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)["vectors"]


@pytest.fixture(scope="module", autouse=True)
def built():
    oc.build()


def test_primitives_match_python_oracle():
    rng = random.Random(99)
    for i in range(4):
        msg = bytes(rng.getrandbits(8) for _ in range(i * 13))
        assert oc.hash_to_g2(msg) == bls.g2_compress(bls.hash_to_g2(msg))
        sk = rng.randrange(1, bls.R)
        assert oc.sk_to_pk(sk) == bls.g1_compress(tb.sk_to_pk(sk))
        assert oc.sign(sk, msg) == bls.g2_compress(tb.sign(sk, msg))


def test_kat_verify():
    for v in load("kat_verify.json"):
        st = oc.verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))
        assert (st == 1) == (v["expect"] == "valid"), v


def _va(vecs, threads):
    pks, sigs, ids, pk_ids, duty_first, msgs, thr = [], [], [], [], [0], [], []
    for v in vecs:
        for p in v["partials"]:
            sigs.append(bytes.fromhex(p["sig"]))
            ids.append(p["identifier"])
            share = v["tss"]["pubshares"].get(str(p["identifier"]))
            if share is None:
                pk_ids.append(0xFFFFFFFF)
            else:
                pk_ids.append(len(pks))
                pks.append(bytes.fromhex(share))
        duty_first.append(duty_first[-1] + len(v["partials"]))
        msgs.append(bytes.fromhex(v["msg"]))
        thr.append(v["tss"]["threshold"])
    table = oc.PubkeyTable(b"".join(pks))
    off = np.cumsum([0] + [len(m) for m in msgs])
    return oc.run(3, duty_first, np.frombuffer(b"".join(sigs), np.uint8), ids, table,
                  msgs=np.frombuffer(b"".join(msgs) + b"\0", np.uint8), msg_off=off, duty_msg=np.arange(len(vecs)),
                  pubkey_ids=pk_ids, duty_threshold=thr, threads=threads), duty_first


@pytest.mark.parametrize("name", ["cfg1_3of4_single.json", "cfg2_3of4_sample.json", "cfg3_7of10_sample.json",
                                  "cfg5_mixed_invalid.json", "va_id_modes.json"])
def test_verify_and_aggregate_golden(name):
    vecs = load(name)
    (ps, ds, agg), duty_first = _va(vecs, threads=4)
    for d, v in enumerate(vecs):
        exp = v["expect"]
        got = [PS_NAMES[s] for s in ps[duty_first[d]:duty_first[d + 1]].tolist()]
        if exp["status"] != "insufficient":
            assert got == exp["partial_status"], v["label"]
        assert DS_NAMES[int(ds[d])] == exp["status"], v["label"]
        if exp["status"] == "ok":
            assert bytes(agg[d]).hex() == exp["agg"], v["label"]


def test_aggregate_golden():
    vecs = load("aggregate_edges.json")
    duty_first = np.cumsum([0] + [len(v["partials"]) for v in vecs])
    sigs = b"".join(bytes.fromhex(p["sig"]) for v in vecs for p in v["partials"])
    ids = [p["identifier"] for v in vecs for p in v["partials"]]
    ps, ds, agg = oc.run(2, duty_first, np.frombuffer(sigs, np.uint8), ids, oc.PubkeyTable(b""))
    for d, v in enumerate(vecs):
        assert DS_NAMES[int(ds[d])] == v["expect"]["status"], v["label"]
        if v["expect"]["status"] == "ok":
            assert bytes(agg[d]).hex() == v["expect"]["agg"], v["label"]


PK_NAMES = {0: "valid", 1: "identity", -1: "err_flags", -2: "err_field", -3: "err_curve", -4: "err_subgroup"}


def test_g1_pubkey_rejections():
    """tblsconv.KeyFromBytes (tblsconv.go:30-37) classes: the C restatement's
    pubkey table decode gives the oracle's class for every fixture key."""
    vecs = load("g1_pubkeys.json")
    table = oc.PubkeyTable(b"".join(bytes.fromhex(v["pk"]) for v in vecs))
    assert [PK_NAMES[s] for s in table.status.tolist()] == [v["expect"] for v in vecs]


def test_invalid_pool_classes():
    """The committed invalid G2 encodings decode to the class they are named by."""
    with open(os.path.join(GOLD, "invalid_g2.json")) as f:
        pools = json.load(f)["pools"]
    for kind, code in (("non_subgroup", -4), ("off_curve", -3)):
        for h in pools[kind]:
            assert oc.g2_decode_status(bytes.fromhex(h)) == code, kind
