#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The oracle (oracle/bls12_381.py, oracle/tbls_oracle.py) is first pinned by the
reference's own known-answer vectors (tests/test_oracle_kat.py).  This script
then freezes inputs and expected outputs for every BASELINE config slice:

  cfg1_3of4_single.json     3-of-4, 1 DV, 1 attestation (config 1)
  cfg2_3of4_sample.json     3-of-4, 64 DVs (sample of config 2 / 4)
  cfg3_7of10_sample.json    7-of-10, 64 DVs (sample of config 3)
  cfg5_mixed_invalid.json   mixed duties, thresholds {3/4, 5/7, 7/10}, injected
                            wrong-message, wrong-share, random-bytes,
                            non-subgroup, off-curve, bad-flag, identity partials
  aggregate_edges.json      tbls.Aggregate edge cases (identifier 0, duplicate
                            identifiers, < 2 partials, > t partials, identity,
                            several D > 1 participant sets, identifier sets whose
                            integer Lagrange form overflows for some or all
                            participants)
  va_id_modes.json          VerifyAndAggregate over clusters with arbitrary
                            share identifiers (1..255): Lagrange denominators
                            D > 1, mixed integer / mod-r overflow sets

Seeded with Python's random.Random(seed); run:  python tests/golden/make_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import tbls_oracle as tb  # noqa: E402

R = bls.R
DOMAINS = {  # domain types used to build distinct signing roots (signing.go:38-48)
    "attestation": b"\x01\x00\x00\x00",
    "sync_committee": b"\x07\x00\x00\x00",
    "randao": b"\x02\x00\x00\x00",
    "proposal": b"\x00\x00\x00\x00",
}


def hx(b):
    return b.hex()


def signing_root(rng, duty):
    import hashlib
    obj = bytes(rng.getrandbits(8) for _ in range(32))
    return hashlib.sha256(obj + DOMAINS[duty] + bytes(28)).digest()


def make_dv(rng, t, n):
    secret = rng.randrange(1, R)
    coeffs = [rng.randrange(1, R) for _ in range(t - 1)]
    tss, shares = tb.generate_tss(secret, t, n, coeffs)
    return secret, tss, shares


def tss_json(tss):
    return {"threshold": tss.threshold, "num_shares": tss.num_shares,
            "public_key": hx(bls.g1_compress(tss.public_key)),
            "pubshares": {str(i): hx(bls.g1_compress(pk)) for i, pk in sorted(tss.pubshares.items())}}


def rand_e2_not_in_g2(rng):
    while True:
        x = (rng.randrange(bls.P), rng.randrange(bls.P))
        y2 = bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2)
        y = bls.f2_sqrt(y2)
        if y is not None:
            pt = (x, y)
            assert not bls.g2_in_subgroup(pt)
            return bls.g2_compress(pt)


def off_curve_bytes(rng):
    while True:
        x = (rng.randrange(bls.P), rng.randrange(bls.P))
        y2 = bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2)
        if bls.f2_sqrt(y2) is None:
            b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
            b[0] |= 0x80
            return bytes(b)


def classify(sig_bytes):
    try:
        pt = bls.g2_decompress(sig_bytes)
    except bls.DecodeError as e:
        m = str(e)
        if "flag" in m or "infinity" in m:
            return None, "err_flags"
        if "field" in m:
            return None, "err_field"
        if "curve" in m:
            return None, "err_curve"
        if "subgroup" in m:
            return None, "err_subgroup"
        return None, "err_flags"
    if pt is None:
        return None, "err_identity"
    return pt, "decoded"


def expected_va(tss, partials, msg):
    """partials: list of (identifier, sig_bytes).  Engine batch semantics."""
    statuses, valid = [], []
    for ident, sb in partials:
        pt, st = classify(sb)
        if st != "decoded":
            statuses.append(st)
            continue
        pk = tss.public_share(ident)
        if pk is None:
            statuses.append("err_pubkey")
            continue
        ok = tb.core_verify(pk, msg, pt)
        statuses.append("valid" if ok else "invalid")
        if ok:
            valid.append((ident, pt))
    if len(partials) < tss.threshold:
        return statuses, "insufficient", None, []
    if len(valid) < tss.threshold:
        return statuses, "insufficient_valid", None, []
    try:
        agg = tb.combine_signatures(valid)
    except tb.TblsError as e:
        return statuses, "agg_error:" + str(e), None, []
    return statuses, "ok", hx(bls.g2_compress(agg)), [i for i, _ in valid]


def duty_record(rng, secret, tss, shares, msg, partials, label):
    statuses, status, agg, signers = expected_va(tss, partials, msg)
    rec = {"label": label, "msg": hx(msg), "tss": tss_json(tss),
           "partials": [{"identifier": i, "sig": hx(s)} for i, s in partials],
           "expect": {"partial_status": statuses, "status": status, "agg": agg, "signers": signers}}
    if status == "ok":
        group_sig = tb.sign(secret, msg)
        assert agg == hx(bls.g2_compress(group_sig)), "aggregate must equal the group signature"
        rec["expect"]["group_sig"] = hx(bls.g2_compress(group_sig))
    return rec


def honest_partials(shares, msg, ids):
    return [(i, bls.g2_compress(tb.sign(shares[i], msg))) for i in ids]


def gen_cfg(rng, t, n, dvs, duty_kinds=("attestation",)):
    recs = []
    for k in range(dvs):
        secret, tss, shares = make_dv(rng, t, n)
        msg = signing_root(rng, duty_kinds[k % len(duty_kinds)])
        recs.append(duty_record(rng, secret, tss, shares, msg, honest_partials(shares, msg, range(1, n + 1)), "honest"))
    return recs


def gen_mixed(rng):
    recs = []
    kinds = ["attestation", "sync_committee", "randao", "proposal"]
    injections = ["wrong_msg", "wrong_share", "random_bytes", "non_subgroup", "off_curve", "bad_flags", "identity",
                  "missing_pubshare", "too_few", "honest_subset"]
    for k, inj in enumerate(injections):
        t, n = [(3, 4), (5, 7), (7, 10)][k % 3]
        secret, tss, shares = make_dv(rng, t, n)
        msg = signing_root(rng, kinds[k % 4])
        ids = list(range(1, n + 1))
        parts = honest_partials(shares, msg, ids)
        j = rng.randrange(n)
        if inj == "wrong_msg":
            parts[j] = (parts[j][0], bls.g2_compress(tb.sign(shares[ids[j]], msg + b"x")))
        elif inj == "wrong_share":
            other = ids[(j + 1) % n]
            parts[j] = (parts[j][0], bls.g2_compress(tb.sign(shares[other], msg)))
        elif inj == "random_bytes":
            parts[j] = (parts[j][0], bytes(rng.getrandbits(8) for _ in range(96)))
        elif inj == "non_subgroup":
            parts[j] = (parts[j][0], rand_e2_not_in_g2(rng))
        elif inj == "off_curve":
            parts[j] = (parts[j][0], off_curve_bytes(rng))
        elif inj == "bad_flags":
            b = bytearray(parts[j][1])
            b[0] &= 0x7F
            parts[j] = (parts[j][0], bytes(b))
        elif inj == "identity":
            parts[j] = (parts[j][0], bytes([0xC0]) + bytes(95))
        elif inj == "missing_pubshare":
            # identifier outside 1..n: TSS.PublicShare returns nil (tss.go:87-89)
            parts[j] = (n + 5, parts[j][1])
        elif inj == "too_few":
            parts = parts[: t - 1]
        elif inj == "honest_subset":
            parts = [parts[i] for i in sorted(rng.sample(range(n), t))]
        recs.append(duty_record(rng, secret, tss, shares, msg, parts, inj))
    # more invalid than n - t: insufficient valid signatures
    secret, tss, shares = make_dv(rng, 3, 4)
    msg = signing_root(rng, "attestation")
    parts = honest_partials(shares, msg, [1, 2, 3, 4])
    parts[0] = (1, bls.g2_compress(tb.sign(shares[1], msg + b"!")))
    parts[1] = (2, bls.g2_compress(tb.sign(shares[2], msg + b"!")))
    recs.append(duty_record(rng, secret, tss, shares, msg, parts, "two_invalid"))
    return recs


def gen_aggregate_edges(rng):
    out = []
    msg = b"data"

    def case(label, partials):
        pts = []
        err = None
        for i, sb in partials:
            pt, st = classify(sb)
            if st == "err_identity":
                err = err or "identity"
            elif st != "decoded":
                err = err or "decode"
            pts.append((i, pt))
        if err is None:
            try:
                agg = hx(bls.g2_compress(tb.combine_signatures(pts)))
                status = "ok"
            except tb.TblsError as e:
                agg, status = None, ("duplicate" if "duplicate" in str(e) else "too_few" if "insufficient" in str(e)
                                     else "identity")
        else:
            agg, status = None, err
        out.append({"label": label, "partials": [{"identifier": i, "sig": hx(s)} for i, s in partials],
                    "expect": {"status": status, "agg": agg}})

    sks = [rng.randrange(1, R) for _ in range(4)]
    sigs = [bls.g2_compress(tb.sign(s, msg)) for s in sks]
    # dkg/dkg_test.go:174-195: identifiers start at 0
    case("identifier_zero", [(0, sigs[0]), (1, sigs[1]), (2, sigs[2])])
    case("duplicate_ids", [(1, sigs[0]), (1, sigs[1]), (2, sigs[2])])
    case("single_partial", [(1, sigs[0])])
    case("identity_partial", [(1, sigs[0]), (2, bytes([0xC0]) + bytes(95))])
    case("bad_encoding", [(1, sigs[0]), (2, bytes(96))])
    # 3-of-4 with all 4 partials passed (core/sigagg/sigagg_test.go style)
    secret, tss, shares = make_dv(rng, 3, 4)
    parts = honest_partials(shares, msg, [1, 2, 3, 4])
    case("all_four_of_3of4", parts)
    case("subset_124", [parts[0], parts[1], parts[3]])
    case("large_ids", [(200, sigs[0]), (255, sigs[1]), (17, sigs[2]), (99, sigs[3])])
    # several duties with a Lagrange denominator D > 1 in one batch (the
    # engine's deferred [1/D] list, k_aggregate_finish)
    more = [bls.g2_compress(tb.sign(rng.randrange(1, R), msg)) for _ in range(10)]
    for ids in ([1, 2, 4], [1, 2, 5], [2, 3, 7], [1, 4, 6, 7], [1, 3, 5]):
        assert lagrange_den(ids) > 1, ids
        case("den_%s" % "_".join(map(str, ids)), list(zip(ids, more)))
    # identifier sets whose integer form fits for some participants and not
    # for others: the encoding must be chosen per duty
    for tag, ids in (("a", [6, 220, 144, 5, 3, 154]), ("b", [6, 1, 177, 224, 69, 19]),
                     ("c", [5, 220, 144, 6, 3, 154])):
        case("mixed_mode_" + tag, list(zip(ids, more)))
    # every participant overflows the integer form: mod-r coefficients only
    case("all_modr", list(zip(range(246, 256), more)))
    return out


def lagrange_den(ids):
    """Common denominator of the reduced Lagrange coefficients at 0."""
    from fractions import Fraction
    from math import lcm
    d = 1
    for i in ids:
        f = Fraction(1)
        for j in ids:
            if j != i:
                f *= Fraction(j, j - i)
        d = lcm(d, f.denominator)
    return d


def make_dv_ids(rng, t, ids):
    """A t-of-len(ids) cluster whose shares sit at arbitrary identifiers."""
    secret = rng.randrange(1, R)
    poly = [secret] + [rng.randrange(1, R) for _ in range(t - 1)]
    shares = {}
    for x in ids:
        acc = 0
        for c in reversed(poly):
            acc = (acc * x + c) % R
        shares[x] = acc
    tss = tb.TSS(pubshares={x: tb.sk_to_pk(s) for x, s in shares.items()}, num_shares=len(ids), threshold=t,
                 public_key=tb.sk_to_pk(secret))
    return secret, tss, shares


def gen_id_modes(rng):
    """VerifyAndAggregate with identifier sets that exercise every Lagrange
    encoding of the engine: D > 1 (deferred [1/D]), mixed integer / mod-r
    overflow sets and all-mod-r sets; one invalid partial in some duties so
    the participating set is a strict subset."""
    recs = []
    specs = [  # (threshold, identifiers, index of an injected wrong-message partial or None)
        (3, [1, 2, 3, 4], 2),            # {1,2,4} participate: D = 3
        (3, [1, 2, 3, 4, 5], 2),         # {1,2,4,5}
        (2, [1, 2, 4], None),            # D = 3
        (6, [6, 220, 144, 5, 3, 154], None),
        (5, [6, 1, 177, 224, 69, 19], 3),
        (6, [5, 220, 144, 6, 3, 154], None),
        (10, list(range(246, 256)), None),
        (4, [200, 255, 17, 99, 1], 0),
    ]
    for t, ids, bad in specs:
        secret, tss, shares = make_dv_ids(rng, t, ids)
        msg = signing_root(rng, "attestation")
        parts = honest_partials(shares, msg, ids)
        if bad is not None:
            parts[bad] = (parts[bad][0], bls.g2_compress(tb.sign(shares[ids[bad]], msg + b"?")))
        recs.append(duty_record(rng, secret, tss, shares, msg, parts, "ids_" + "_".join(map(str, ids))))
    return recs


def kat_verify_vectors():
    from tests.test_oracle_kat import DEPOSIT_GOLDEN, deposit_signing_root, teku_signing_root, TEKU_SK, TEKU_SIG
    vecs = []
    for pk_hex, sig_hex, root in DEPOSIT_GOLDEN:
        m = deposit_signing_root(root)
        vecs.append({"pk": pk_hex, "msg": hx(m), "sig": sig_hex, "expect": "valid"})
        bad = bytearray(m)
        bad[5] ^= 0x40
        vecs.append({"pk": pk_hex, "msg": hx(bytes(bad)), "sig": sig_hex, "expect": "invalid"})
    pk = hx(bls.g1_compress(tb.sk_to_pk(int(TEKU_SK, 16))))
    vecs.append({"pk": pk, "msg": hx(teku_signing_root()), "sig": TEKU_SIG, "expect": "valid"})
    # wrong key for a valid signature
    vecs.append({"pk": DEPOSIT_GOLDEN[1][0], "msg": hx(deposit_signing_root(DEPOSIT_GOLDEN[0][2])),
                 "sig": DEPOSIT_GOLDEN[0][1], "expect": "invalid"})
    return vecs


def invalid_pool_file():
    """tests/golden/invalid_g2.json: encodings the full-size workloads inject
    (tools/workload.py make_mixed_batch) that need curve arithmetic to find:
    points on E2 outside G2 (kryptology: subgroup error) and x coordinates
    with no point on E2 (not-on-curve error), each classified by the oracle."""
    rng = random.Random(0x1A7A)
    pools = {"non_subgroup": [], "off_curve": []}
    for _ in range(24):
        b = rand_e2_not_in_g2(rng)
        assert classify(b)[1] == "err_subgroup"
        pools["non_subgroup"].append(hx(b))
        b = off_curve_bytes(rng)
        assert classify(b)[1] == "err_curve"
        pools["off_curve"].append(hx(b))
    with open(os.path.join(HERE, "invalid_g2.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py invalid_pool", "seed": "0x1A7A", "pools": pools}, f,
                  indent=1)
    # 48-byte G1 public keys for tblsconv.KeyFromBytes (tblsconv.go:30-37):
    # valid keys and every rejection class, each classified by the oracle
    g1 = []

    def g1_case(label, b):
        try:
            pt = bls.g1_decompress(b)
            st = "identity" if pt is None else "valid"
        except bls.DecodeError as e:
            m = str(e)
            st = ("err_flags" if ("flag" in m or "infinity" in m) else "err_field" if "field" in m
                  else "err_curve" if "curve" in m else "err_subgroup")
        g1.append({"label": label, "pk": hx(b), "expect": st})

    for k in range(4):
        g1_case("valid", bls.g1_compress(tb.sk_to_pk(rng.randrange(1, R))))
    good = bls.g1_compress(tb.sk_to_pk(rng.randrange(1, R)))
    g1_case("bad_flags", bytes([good[0] & 0x7F]) + good[1:])
    g1_case("identity", bytes([0xC0]) + bytes(47))
    g1_case("infinity_with_sign", bytes([0xE0]) + bytes(47))
    g1_case("infinity_with_x", bytes([0xC0]) + good[1:])
    g1_case("x_ge_p", (bls.P + 5).to_bytes(48, "big")[:0] + bytes([0x80 | ((bls.P + 5) >> 376)]) +
            (bls.P + 5).to_bytes(48, "big")[1:])
    g1_case("all_ones", bytes([0x9F]) + bytes([0xFF]) * 47)
    while len([c for c in g1 if c["label"] == "off_curve"]) < 3:
        x = rng.randrange(bls.P)
        y2 = (x * x * x + 4) % bls.P
        if pow(y2, (bls.P - 1) // 2, bls.P) != 1:
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80
            g1_case("off_curve", bytes(b))
    while len([c for c in g1 if c["label"] == "non_subgroup"]) < 3:
        x = rng.randrange(bls.P)
        y2 = (x * x * x + 4) % bls.P
        if pow(y2, (bls.P - 1) // 2, bls.P) == 1:
            y = pow(y2, (bls.P + 1) // 4, bls.P)
            assert not bls.g1_in_subgroup((x, y))
            g1_case("non_subgroup", bls.g1_compress((x, y)))
    expected = {"valid": "valid", "bad_flags": "err_flags", "identity": "identity", "infinity_with_sign": "err_flags",
                "infinity_with_x": "err_flags", "x_ge_p": "err_field", "all_ones": "err_field",
                "off_curve": "err_curve", "non_subgroup": "err_subgroup"}
    for c in g1:
        assert c["expect"] == expected[c["label"]], c
    with open(os.path.join(HERE, "g1_pubkeys.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py invalid_pool", "seed": "0x1A7A", "vectors": g1}, f,
                  indent=1)


def main():
    if sys.argv[1:] == ["invalid_pool"]:
        invalid_pool_file()
        return
    rng = random.Random(0xC4A2)
    files = {
        "kat_verify.json": kat_verify_vectors(),
        "cfg1_3of4_single.json": gen_cfg(rng, 3, 4, 1),
        "cfg2_3of4_sample.json": gen_cfg(rng, 3, 4, 64),
        "cfg3_7of10_sample.json": gen_cfg(rng, 7, 10, 64),
        "cfg5_mixed_invalid.json": gen_mixed(rng),
        "aggregate_edges.json": gen_aggregate_edges(rng),
        "va_id_modes.json": gen_id_modes(rng),
    }
    for name, data in files.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py", "seed": "0xC4A2", "vectors": data}, f, indent=1)
        print(name, len(data))


if __name__ == "__main__":
    main()
