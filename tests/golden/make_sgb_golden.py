"""tests/golden/sgb_points.json: signatures crafted against the batched
subgroup test (charon_amd/csrc/k_sgb.hip), written with the Python oracle
(test infrastructure; data only in the JSON).

A point of E2(Fp2) outside G2 is s = g + t with g in G2 and t != 0 in the
cofactor part H (|H| = h2).  The random-combination test is weakest against
t of the smallest prime order dividing h2, 13 (a combination hides it with
probability 1/13), and against several bad signatures whose components
cancel in a plain sum.  Kinds:

  t13          g + t, t of order 13
  t23          g + t, t of order 23
  torsion13    t itself (order 13): on the curve, outside G2
  pair_a/pair_b  g_a + t and g_b - t (t of order 13): they cancel in g_a + g_b

Every encoding is checked against the oracle's exact decode (subgroup error).
    python tests/golden/make_sgb_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402

# the G2 cofactor: #E2(Fp2) = H2 * R
H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5


def rand_e2(rng):
    while True:
        x = (rng.randrange(bls.P), rng.randrange(bls.P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None:
            return (x, y)


def torsion(rng, ell):
    """A point of order exactly ell (prime, ell | H2): the ell-part of a random
    point (every other prime power of the group order multiplied out), brought
    down to order ell."""
    n, e = H2 * bls.R, 0
    while n % ell == 0:
        n //= ell
        e += 1
    while True:
        t = bls.g2_mul_raw(rand_e2(rng), n)  # order divides ell^e
        if t is None:
            continue
        while bls.g2_mul_raw(t, ell) is not None:
            t = bls.g2_mul_raw(t, ell)
        return t


def g2_point(rng):
    return bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))


def check_bad(b):
    try:
        bls.g2_decompress(b)
    except bls.DecodeError as e:
        assert "subgroup" in str(e), e
        return
    raise AssertionError("decodes as a G2 point")


def main():
    rng = random.Random(0x5CB)
    assert bls.g2_mul_raw(rand_e2(rng), H2 * bls.R) is None  # the group order
    t13, t23 = torsion(rng, 13), torsion(rng, 23)
    out = {"t13": [], "t23": [], "torsion13": [], "pair_a": [], "pair_b": []}
    for _ in range(6):
        out["t13"].append(bls.g2_compress(bls.g2_add(g2_point(rng), bls.g2_mul_raw(t13, rng.randrange(1, 13)))))
        out["t23"].append(bls.g2_compress(bls.g2_add(g2_point(rng), bls.g2_mul_raw(t23, rng.randrange(1, 23)))))
        t = bls.g2_mul_raw(t13, rng.randrange(1, 13))
        out["torsion13"].append(bls.g2_compress(t))
        out["pair_a"].append(bls.g2_compress(bls.g2_add(g2_point(rng), t)))
        out["pair_b"].append(bls.g2_compress(bls.g2_add(g2_point(rng), bls.g2_neg(t))))
    for v in out.values():
        for b in v:
            check_bad(b)
    with open(os.path.join(HERE, "sgb_points.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_sgb_golden.py", "seed": "0x5CB",
                   "points": {k: [b.hex() for b in v] for k, v in out.items()}}, f, indent=1)


if __name__ == "__main__":
    main()
