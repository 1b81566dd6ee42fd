"""The engine's device arithmetic, compiled for the host, against the oracle.

The HIP kernels include exactly these headers (charon_amd/csrc/bls_*.h); the
host build runs with TBG_BOUNDS_CHECK so a violated lazy-reduction bound
aborts the test process.  GPU parity is covered separately (-m gpu)."""
import random

import pytest

from oracle import bls12_381 as bls
from oracle import tbls_oracle as tb
from tests.hostcheck import lib

P = bls.P
rng = random.Random(20241015)


def be(x):
    return x.to_bytes(48, "big")


def fe(b):
    return int.from_bytes(b, "big")


def call(fn, *args, out=48):
    buf = (bytes(out))
    import ctypes
    ob = ctypes.create_string_buffer(out)
    getattr(lib(), fn)(*args, ob)
    return ob.raw


EDGE = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, (1 << 380) % P, (1 << 381) - 1 - P]


def samples(n=40):
    return EDGE + [rng.randrange(P) for _ in range(n)]


def test_fp_ops():
    vals = samples()
    for a in vals:
        for b in vals[:12] + [rng.randrange(P)]:
            assert fe(call("hc_fp_mul", be(a), be(b))) == a * b % P
            assert fe(call("hc_fp_add", be(a), be(b))) == (a + b) % P
            assert fe(call("hc_fp_sub", be(a), be(b))) == (a - b) % P
        assert fe(call("hc_fp_sqr", be(a))) == a * a % P
    for a in vals[1:10]:
        if a % P:
            assert fe(call("hc_fp_inv", be(a))) == pow(a, P - 2, P)
            assert fe(call("hc_fp_inv_fermat", be(a))) == pow(a, P - 2, P)


def f2b(x):
    return be(x[0]) + be(x[1])


def b2f(b):
    return (fe(b[:48]), fe(b[48:96]))


def test_fp2_mul_and_sqrt():
    # Karatsuba fp2_mul: c0 = REDC(a0 b0 - a1 b1) goes negative when a1 b1
    # dominates (the conditional +p path); edge magnitudes on both sides
    edges = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, 1 << 380]
    for a0 in edges:
        for a1 in edges[:4]:
            a, b = (a0, a1), (edges[3], a0)
            assert b2f(call("hc_fp2_mul", f2b(a), f2b(b), out=96)) == bls.f2_mul(a, b)
            assert b2f(call("hc_fp2_mul", f2b(b), f2b(a), out=96)) == bls.f2_mul(b, a)
    for _ in range(30):
        a = (rng.randrange(P), rng.randrange(P))
        b = (rng.randrange(P), rng.randrange(P))
        assert b2f(call("hc_fp2_mul", f2b(a), f2b(b), out=96)) == bls.f2_mul(a, b)
        sq = bls.f2_sqr(a)
        import ctypes
        ob = ctypes.create_string_buffer(96)
        assert lib().hc_fp2_sqrt(f2b(sq), ob) == 1
        r = b2f(ob.raw)
        assert bls.f2_sqr(r) == sq
    # non-squares and the a1 == 0 branch
    for _ in range(10):
        a = (rng.randrange(P), rng.randrange(P))
        import ctypes
        ob = ctypes.create_string_buffer(96)
        ok = lib().hc_fp2_sqrt(f2b(a), ob)
        assert ok == (1 if bls.f2_is_square(a) else 0)
        if ok:
            assert bls.f2_sqr(b2f(ob.raw)) == a
    for a0 in [0, 1, 2, 3, P - 1, rng.randrange(P)]:
        import ctypes
        ob = ctypes.create_string_buffer(96)
        ok = lib().hc_fp2_sqrt(f2b((a0, 0)), ob)
        assert ok == 1  # every Fp element is a square in Fp2
        assert bls.f2_sqr(b2f(ob.raw)) == (a0, 0)


def f12b(f):
    (a, b, c), (d, e, g) = f
    return b"".join(f2b(x) for x in (a, b, c, d, e, g))


def b2f12(bb):
    xs = [b2f(bb[96 * i:96 * i + 96]) for i in range(6)]
    return ((xs[0], xs[1], xs[2]), (xs[3], xs[4], xs[5]))


def rand_f12():
    return tuple(tuple((rng.randrange(P), rng.randrange(P)) for _ in range(3)) for _ in range(2))


def test_fp12_ops():
    for _ in range(6):
        a, b = rand_f12(), rand_f12()
        assert b2f12(call("hc_fp12_mul", f12b(a), f12b(b), out=576)) == bls.f12_mul(a, b)
        assert b2f12(call("hc_fp12_sqr", f12b(a), out=576)) == bls.f12_sqr(a)
        assert b2f12(call("hc_fp12_inv", f12b(a), out=576)) == bls.f12_inv(a)
        assert b2f12(call("hc_fp12_frob", f12b(a), out=576)) == bls.f12_frob(a)


def test_cyclotomic_square():
    a = rand_f12()
    # project into the cyclotomic subgroup with the easy part of the final exponentiation
    f = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
    f = bls.f12_mul(bls.f12_frob_n(f, 2), f)
    assert b2f12(call("hc_fp12_cyc_sqr", f12b(f), out=576)) == bls.f12_sqr(f)


def test_final_exp_matches_oracle():
    a = rand_f12()
    assert b2f12(call("hc_final_exp", f12b(a), out=576)) == bls.final_exp(a)


def aff2b(q):
    return f2b(q[0]) + f2b(q[1])


def test_miller_loop_after_final_exp():
    p = bls.g1_mul(bls.G1_GEN, rng.randrange(1, bls.R))
    q = bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))
    m = b2f12(call("hc_miller", be(p[0]) + be(p[1]), aff2b(q), out=576))
    # the device scales its lines by Fp2 factors; only the final-exponentiated values must agree
    assert bls.final_exp(m) == bls.pairing(p, q)


def test_g2_decompress_matches_oracle():
    import ctypes
    for _ in range(6):
        q = bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))
        enc = bls.g2_compress(q)
        ob = ctypes.create_string_buffer(192)
        assert lib().hc_g2_decompress(enc, ob) == 0
        assert (b2f(ob.raw[:96]), b2f(ob.raw[96:])) == q
    # error classes
    ob = ctypes.create_string_buffer(192)
    assert lib().hc_g2_decompress(bytes([0xC0]) + bytes(95), ob) == 1          # identity
    assert lib().hc_g2_decompress(bytes(96), ob) == -1                         # no compression flag
    assert lib().hc_g2_decompress(bytes([0x9F]) + b"\xff" * 95, ob) == -2      # x >= p


def test_g2_decompress_rejects_off_curve_and_non_subgroup():
    import ctypes
    n_off = n_sub = 0
    for _ in range(12):
        x = (rng.randrange(P), rng.randrange(P))
        y2 = bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2)
        enc = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
        enc[0] |= 0x80
        ob = ctypes.create_string_buffer(192)
        st = lib().hc_g2_decompress(bytes(enc), ob)
        if bls.f2_sqrt(y2) is None:
            assert st == -3
            n_off += 1
        else:
            assert st == -4  # random curve points are outside G2 (cofactor h2 is huge)
            n_sub += 1
    assert n_off and n_sub


def test_hash_to_g2_matches_oracle():
    # 30 messages = 60 SSWU maps: both the square and the non-square branch of
    # map_to_curve_g2_pair are taken many times
    msgs = [b"", b"abc", bytes(32), bytes(range(32)), b"Hello Obol", bytes(range(200))]
    msgs += [bytes([i]) * (i + 1) for i in range(24)]
    for msg in msgs:
        h = call("hc_hash_to_g2", msg, len(msg), out=96)
        assert h == bls.g2_compress(bls.hash_to_g2(msg))


def test_core_verify_kat_and_rejects():
    from tests.test_oracle_kat import DEPOSIT_GOLDEN, deposit_signing_root
    for pk_hex, sig_hex, root_hex in DEPOSIT_GOLDEN[:2]:
        pk, sig, root = bytes.fromhex(pk_hex), bytes.fromhex(sig_hex), deposit_signing_root(root_hex)
        assert lib().hc_verify(pk, root, len(root), sig) == 1
        bad = bytearray(root)
        bad[0] ^= 1
        assert lib().hc_verify(pk, bytes(bad), len(bad), sig) == 0
    # wrong key
    pk2 = bytes.fromhex(DEPOSIT_GOLDEN[2][0])
    pk, sig, root = bytes.fromhex(DEPOSIT_GOLDEN[0][0]), bytes.fromhex(DEPOSIT_GOLDEN[0][1]), deposit_signing_root(DEPOSIT_GOLDEN[0][2])
    assert lib().hc_verify(pk2, root, len(root), sig) == 0


def test_g1_decompress_matches_oracle():
    import ctypes
    for _ in range(4):
        p = bls.g1_mul(bls.G1_GEN, rng.randrange(1, bls.R))
        ob = ctypes.create_string_buffer(96)
        assert lib().hc_g1_decompress(bls.g1_compress(p), ob) == 0
        assert (fe(ob.raw[:48]), fe(ob.raw[48:])) == p


def test_aggregate_integer_and_modr_paths_match_golden():
    """Lagrange recombination (integer numerators / common denominator, or the
    mod-r fallback) reproduces every golden aggregate."""
    import ctypes
    import json
    import os
    gold = os.path.join(os.path.dirname(__file__), "golden")
    cases = []
    for v in json.load(open(os.path.join(gold, "aggregate_edges.json")))["vectors"]:
        if v["expect"]["status"] == "ok":
            cases.append(([p["identifier"] for p in v["partials"]], [p["sig"] for p in v["partials"]], v["expect"]["agg"]))
    for name in ["cfg1_3of4_single.json", "cfg3_7of10_sample.json", "cfg5_mixed_invalid.json", "va_id_modes.json"]:
        for v in json.load(open(os.path.join(gold, name)))["vectors"]:
            if v["expect"]["status"] != "ok":
                continue
            ps = [p for p, st in zip(v["partials"], v["expect"]["partial_status"]) if st == "valid"]
            cases.append(([p["identifier"] for p in ps], [p["sig"] for p in ps], v["expect"]["agg"]))
    assert len(cases) >= 10
    # the round-1 advisor's mixed integer / mod-r identifier sets are among them
    assert any(sorted(ids) == [3, 5, 6, 144, 154, 220] for ids, _, _ in cases)
    for ids, sigs, agg in cases:
        if len(ids) > 16:
            continue  # hc_stage_aggregate's fixed arrays
        ob = ctypes.create_string_buffer(96)
        rc = lib().hc_stage_aggregate(bytes(ids), b"".join(bytes.fromhex(s) for s in sigs), len(ids), ob)
        assert rc == 0 and ob.raw.hex() == agg, ids


def test_quad_lane_algebra_matches_tower():
    """The per-lane pieces of the lane-cooperative Fp12 arithmetic (bls_quad.h),
    run as an emulated quad on the host, equal the oracle's tower arithmetic."""
    for _ in range(4):
        a, b = rand_f12(), rand_f12()
        assert b2f12(call("hc_quad_mul", f12b(a), f12b(b), out=576)) == bls.f12_mul(a, b)
        assert b2f12(call("hc_quad_sqr", f12b(a), out=576)) == bls.f12_sqr(a)
        assert b2f12(call("hc_quad_frob", f12b(a), out=576)) == bls.f12_frob(a)
        assert b2f12(call("hc_quad_conj", f12b(a), out=576)) == bls.f12_conj(a)
        l0, l1, l4 = [(rng.randrange(P), rng.randrange(P)) for _ in range(3)]
        line = ((l0, l1, bls.F2_ZERO), (bls.F2_ZERO, l4, bls.F2_ZERO))
        got = b2f12(call("hc_quad_line", f12b(a), f2b(l0) + f2b(l1) + f2b(l4), out=576))
        assert got == bls.f12_mul(a, line)
    f = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
    f = bls.f12_mul(bls.f12_frob_n(f, 2), f)
    assert b2f12(call("hc_quad_cyc_sqr", f12b(f), out=576)) == bls.f12_sqr(f)


def test_hex_lane_algebra_matches_tower():
    """The hexad pieces (bls_hex.h: the trio with every Fp2 split over a lane
    pair, the level-0 Miller kernel's layout), run as six emulated lanes,
    equal the oracle's tower squaring and sparse line product."""
    for _ in range(4):
        a = rand_f12()
        assert b2f12(call("hc_hex_sqr", f12b(a), out=576)) == bls.f12_sqr(a)
        l0, l1, l4 = [(rng.randrange(P), rng.randrange(P)) for _ in range(3)]
        line = ((l0, l1, bls.F2_ZERO), (bls.F2_ZERO, l4, bls.F2_ZERO))
        got = b2f12(call("hc_hex_line", f12b(a), f2b(l0) + f2b(l1) + f2b(l4), out=576))
        assert got == bls.f12_mul(a, line)


def test_quad_verify_pipeline_emulated():
    """Line precomputation + quad Miller accumulation + quad final
    exponentiation (the k_lines_* / k_verify_quad algorithm) on the host."""
    from tests.test_oracle_kat import DEPOSIT_GOLDEN, deposit_signing_root
    pk_hex, sig_hex, root_hex = DEPOSIT_GOLDEN[0]
    root = deposit_signing_root(root_hex)
    assert lib().hc_stage_lines(bytes.fromhex(sig_hex), root, len(root)) == 0
    assert lib().hc_stage_verify_quad(bytes.fromhex(pk_hex)) == 1
    assert lib().hc_stage_verify_quad(bytes.fromhex(DEPOSIT_GOLDEN[1][0])) == 0   # wrong key
    bad = bytearray(root)
    bad[3] ^= 8
    assert lib().hc_stage_lines(bytes.fromhex(sig_hex), bytes(bad), len(bad)) == 0
    assert lib().hc_stage_verify_quad(bytes.fromhex(pk_hex)) == 0                 # wrong message


def test_rlc_digit_scalars_match_plain_scalar_multiplication():
    """k_rlc_partial applies r = a0 + a1 x + a2 x^2 + a3 x^3 (signed digits) through psi on G2
    and phi / [x]pk on G1; both must equal [r mod order] P."""
    import ctypes
    L = lib()
    L.hc_rlc_check.restype = ctypes.c_int
    L.hc_rlc_check.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
    x = -bls.X_ABS
    for trial in range(6):
        sk = rng.randrange(1, bls.R)
        msg = bytes([trial]) * 32
        sig = bls.g2_compress(tb.sign(sk, msg))
        pk = bls.g1_compress(tb.sk_to_pk(sk))
        r64 = rng.getrandbits(64) if trial else 0xFFFF_FFFF_FFFF_FFFF
        # signed binary digits: bit set -> +1, clear -> -1 (bls_rlc.h)
        a = [2 * ((r64 >> (16 * k)) & 0xFFFF) - 0xFFFF for k in range(4)]
        r = sum(a[k] * x ** k for k in range(4)) % bls.R
        words = (ctypes.c_uint32 * 8)(*[(r >> (32 * k)) & 0xFFFFFFFF for k in range(8)])
        assert L.hc_rlc_check(sig, pk, r64, words) == 3
        # inversion-free Jacobian tables: G1, single-lane G2, lane-pair G2 (emulated)
        L.hc_rlc_check_j.restype = ctypes.c_int
        L.hc_rlc_check_j.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
        assert L.hc_rlc_check_j(sig, pk, r64, words) == 7
        # the per-key window table of level 0 / the group levels (k_pubkey_tables)
        L.hc_rlc_check_w2.restype = ctypes.c_int
        L.hc_rlc_check_w2.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
        assert L.hc_rlc_check_w2(pk, r64, words) == 1


def test_base_x_msm_matches_plain_scalar_multiplication():
    """k_aggregate_finish's [1/D] as a 4-way MSM over the base-|x| digits of
    the scalar (bls_tss.h): digits reconstruct k, each below |x|, and the MSM
    equals the plain double-and-add, on edge and random scalars."""
    import ctypes
    L = lib()
    L.hc_base_x_check.restype = ctypes.c_int
    L.hc_base_x_check.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p]
    xa = bls.X_ABS
    sig = bls.g2_compress(tb.sign(rng.randrange(1, bls.R), b"base-x"))
    ks = [0, 1, xa - 1, xa, xa + 1, xa ** 2, xa ** 3 - 1, xa ** 3, bls.R - 1, (bls.R + 1) // 2]
    ks += [pow(D, -1, bls.R) for D in (2, 3, 4, 6, 8, 15, 2 ** 61 - 1)]
    ks += [rng.randrange(bls.R) for _ in range(4)]
    for k in ks:
        words = (ctypes.c_uint32 * 8)(*[(k >> (32 * j)) & 0xFFFFFFFF for j in range(8)])
        d = (ctypes.c_uint64 * 4)()
        assert L.hc_base_x_check(sig, words, d) == 1, hex(k)
        assert all(v < xa for v in d) and sum(v * xa ** i for i, v in enumerate(d)) == k


def test_rlc_digit_scalars_are_distinct_mod_r():
    """Distinct digit vectors give distinct scalars (the 2^-64 soundness bound):
    |x| > 2^16 and 2^16 |x|^3 < r, checked on the extreme digit values."""
    x = bls.X_ABS
    # signed digits a_k = 2 u_k - (2^16 - 1): differences of two are < 2^17
    assert (1 << 17) < x and (1 << 17) * x ** 3 < bls.R


def test_lane_pair_fp2_matches_tower():
    """bls_pair.h: Fp2 split over two lanes (host-emulated pair) equals the
    oracle's Fp2 arithmetic for every operation the pair kernels use."""
    import ctypes
    L = lib()
    psi_x = bls.f2_inv(bls.f2_pow((1, 1), (P - 1) // 3))  # tools/gen_constants.py PSI_X
    for _ in range(6):
        a = (rng.randrange(P), rng.randrange(P))
        b = (rng.randrange(P), rng.randrange(P))
        out = ctypes.create_string_buffer(6 * 96)
        enc = lambda x: x[0].to_bytes(48, "big") + x[1].to_bytes(48, "big")  # noqa: E731
        L.hc_pair_ops(enc(a), enc(b), out)
        got = [(int.from_bytes(out.raw[96 * k:96 * k + 48], "big") % P, int.from_bytes(out.raw[96 * k + 48:96 * k + 96], "big") % P)
               for k in range(6)]
        assert got[0] == bls.f2_mul(a, b)
        assert got[1] == bls.f2_sqr(a)
        assert got[2] == bls.f2_inv(a)
        assert got[3] == bls.f2_conj(a)
        assert got[4] == bls.f2_mul_xi(a)
        assert got[5] == bls.f2_mul(a, psi_x)


def test_lane_pair_subgroup_check_matches_decode():
    """k_decode_sigs + k_subgroup_sigs (pair-emulated) classify like the
    single-lane decode: valid signatures, non-subgroup points, off-curve."""
    import json
    import os
    L = lib()
    gold = os.path.join(os.path.dirname(__file__), "golden")
    pools = json.load(open(os.path.join(gold, "invalid_g2.json")))["pools"]
    for h in pools["non_subgroup"][:4]:
        assert L.hc_pair_decode_sig(bytes.fromhex(h)) == -4
    for h in pools["off_curve"][:2]:
        assert L.hc_pair_decode_sig(bytes.fromhex(h)) == -3
    for v in json.load(open(os.path.join(gold, "cfg1_3of4_single.json")))["vectors"]:
        for p in v["partials"]:
            assert L.hc_pair_decode_sig(bytes.fromhex(p["sig"])) == 0


def test_lane_pair_lines_and_cofactor_clearing():
    """k_lines_h and k_hash_clear_* (pair-emulated, lazy sums in the group
    law) equal the single-lane lines and cofactor clearing; the bound checks
    of the host build (limbs, 64-bit columns) hold along the way."""
    import json
    import os
    L = lib()
    gold = os.path.join(os.path.dirname(__file__), "golden")
    sigs = [p["sig"] for v in json.load(open(os.path.join(gold, "cfg1_3of4_single.json")))["vectors"]
            for p in v["partials"]]
    pools = json.load(open(os.path.join(gold, "invalid_g2.json")))["pools"]
    for h in sigs[:4] + pools["non_subgroup"][:2]:  # E2 points in and outside G2
        assert L.hc_pair_lines_clear(bytes.fromhex(h)) == 7, h


def test_level0_bucket_msm_matches_rlc_products():
    """Level 0's signature side (bls_msm.h, k_msm.hip): the bucket method over
    the signed base-x digits equals the sum of the per-partial RLC products,
    including a bucket that meets the same point twice (doubling), a point and
    its negation cancelling in one bucket, and extreme digit words."""
    import ctypes
    L = lib()
    L.hc_msm_check.restype = ctypes.c_int
    L.hc_msm_check.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32]
    sigs = [bls.g2_compress(tb.sign(rng.randrange(1, bls.R), bytes([k]) * 32)) for k in range(6)]
    neg = bls.g2_compress(bls.g2_neg(bls.g2_decompress(sigs[1])))
    rs = [rng.getrandbits(64) for _ in range(6)]
    cases = [
        (sigs, rs),
        (sigs[:2] + [sigs[0]], rs[:2] + [rs[0]]),           # same point, same digits: doubling in 4 buckets
        ([sigs[1], neg, sigs[2]], [rs[1], rs[1], rs[2]]),   # s and -s with the same digits cancel
        (sigs[:3], [0, 0xFFFF_FFFF_FFFF_FFFF, 0x8000_7FFF_0000_FFFF]),
    ]
    for ss, rr in cases:
        buf = b"".join(ss)
        arr = (ctypes.c_uint64 * len(rr))(*rr)
        assert L.hc_msm_check(buf, arr, len(ss)) == 1


def test_group_msm_windows_match_per_partial_products():
    """Level 1's group MSM (k_gmsm.hip: each 16-bit psi digit as four 4-bit
    windows of signed binary digits, 32 buckets, running sums, base-16
    combination; bls_msm.h gm_reference) equals the sum of the per-partial RLC
    products rlc_mul_g2 it replaces -- with a group lead (r = 1), a point
    added twice with the same digits (bucket doublings), s and -s cancelling,
    and the extreme digit words."""
    import ctypes
    L = lib()
    L.hc_gm_check.restype = ctypes.c_int
    L.hc_gm_check.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    sigs = [bls.g2_compress(tb.sign(rng.randrange(1, bls.R), bytes([k + 40]) * 32)) for k in range(6)]
    neg = bls.g2_compress(bls.g2_neg(bls.g2_decompress(sigs[1])))
    rs = [rng.getrandbits(64) for _ in range(6)]
    cases = [
        (sigs, rs, 99),
        (sigs, rs, 0),                                       # the first partial as the group lead
        (sigs[:2] + [sigs[0]], rs[:2] + [rs[0]], 99),        # same point, same digits: doublings in 16 buckets
        ([sigs[1], neg, sigs[2]], [rs[1], rs[1], rs[2]], 99),  # s and -s with the same digits cancel
        (sigs[:3], [0, 0xFFFF_FFFF_FFFF_FFFF, 0x8000_7FFF_0000_FFFF], 1),
    ]
    for ss, rr, lead in cases:
        buf = b"".join(ss)
        arr = (ctypes.c_uint64 * len(rr))(*rr)
        assert L.hc_gm_check(buf, arr, len(ss), lead) == 1, lead


def test_word_sha_expand_message_matches_byte_stream():
    """The kernels' expand_message_xmd (16-word blocks in registers, unrolled
    SHA-256 schedule) equals the byte-stream form on every message length
    around the block boundaries (b_0's input is 64 + len + 47 bytes)."""
    import ctypes
    L = lib()
    L.hc_h2f_check.restype = ctypes.c_int
    L.hc_h2f_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    for n in list(range(0, 20)) + [31, 32, 33, 63, 64, 65, 71, 72, 73, 127, 128, 136, 200, 255, 300]:
        msg = bytes((7 * k + n) & 0xFF for k in range(n))
        assert L.hc_h2f_check(msg, n) == 1, n


def test_split_sswu_matches_reference_map():
    """k_hash.hip's split map (k_hash_map: the denominators' shared inverse
    and x1; k_hash_sswu: g(x1), the closed-form root at window width SSWU_WIN, x and
    y, the Horner-form isogeny) gives the same point as the RFC 9380 6.6.2
    reference map on both field elements of each message."""
    import ctypes
    L = lib()
    L.hc_sswu_split_check.restype = ctypes.c_int
    L.hc_sswu_split_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    for n in [0, 1, 5, 32, 33, 64, 77, 96, 200]:
        msg = bytes((11 * k + 3 * n + 1) & 0xFF for k in range(n))
        assert L.hc_sswu_split_check(msg, n) == 1, n


def test_workgroup_batch_inversion_matches_per_value_inverse():
    """bls_batchinv.h (Montgomery's trick over a workgroup: wave scans, one
    inversion, back-substitution), emulated lane by lane: every present value
    gets its own inverse, absent ones (a zero among them, the point at
    infinity's Z) get 1 and do not disturb their neighbours; blocks of 1 and 4
    waves, a partial last workgroup."""
    import ctypes
    for waves, n in ((4, 300), (1, 64), (4, 256), (2, 129)):
        vals = [rng.randrange(1, P) for _ in range(n)]
        present = [1] * n
        for k in (0, 63, 64, 200, n - 1):
            if k < n:
                present[k] = 0
        vals[min(5, n - 1)] = 0
        present[min(5, n - 1)] = 0  # a zero element, marked absent as the kernels do
        vals[min(7, n - 1)] = 1
        out = ctypes.create_string_buffer(48 * n)
        lib().hc_batch_inv(b"".join(be(v) for v in vals), bytes(present), n, waves, out)
        got = [fe(out.raw[48 * i:48 * i + 48]) for i in range(n)]
        for v, pz, g in zip(vals, present, got):
            assert g == (pow(v, P - 2, P) if pz else 1)


def test_hex_final_exp_pieces_match_tower():
    """bls_hex.h final exponentiation on the hexad (the fallback-check kernels'
    layout): product, cyclotomic squaring, Frobenius, conjugation and the
    whole f^(3 (p^12 - 1) / r), the six lanes emulated phase by phase, equal
    the oracle's tower; the lanes' is-one test agrees."""
    a, b = rand_f12(), rand_f12()
    assert b2f12(call("hc_hex_mul", f12b(a), f12b(b), out=576)) == bls.f12_mul(a, b)
    assert b2f12(call("hc_hex_frob", f12b(a), out=576)) == bls.f12_frob_n(a, 1)
    assert b2f12(call("hc_hex_conj", f12b(a), out=576)) == bls.f12_conj(a)
    f = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
    f = bls.f12_mul(bls.f12_frob_n(f, 2), f)
    assert b2f12(call("hc_hex_cyc_sqr", f12b(f), out=576)) == bls.f12_sqr(f)
    import ctypes
    out = ctypes.create_string_buffer(576)
    one = lib().hc_hex_final_exp(f12b(a), out)
    assert b2f12(out.raw) == bls.final_exp(a) and one == 0
    # a product of pairings that cancels: e(P, Q) e(-P, Q) before the final exponentiation
    p = bls.g1_mul(bls.G1_GEN, rng.randrange(1, bls.R))
    q = bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))
    m1 = b2f12(call("hc_miller", be(p[0]) + be(p[1]), aff2b(q), out=576))
    m2 = b2f12(call("hc_miller", be(p[0]) + be((P - p[1]) % P), aff2b(q), out=576))
    assert lib().hc_hex_final_exp(f12b(bls.f12_mul(m1, m2)), out) == 1


def _val(l):
    return sum(v << (28 * j) for j, v in enumerate(l))


def _i32(l):
    import ctypes
    return (ctypes.c_int32 * 14)(*l)


def _redundant(x):
    """x with every limb but the top shifted by a random signed amount
    carried into the next limb (same value, |limb| < 2^29)."""
    l = [(x >> (28 * j)) & ((1 << 28) - 1) for j in range(13)] + [x >> (28 * 13)]
    for j in range(13):
        d = rng.randrange(-3, 4)
        l[j] += d << 28
        l[j + 1] -= d
    return l


def test_row_fp_product_and_reduction():
    """bls_row.h: REDC(a b + c d) with one limb column per lane of a 16-lane
    row (signed redundant limbs, ds_swizzle broadcasts and DPP shifts run as
    array operations on the host) equals the oracle's Montgomery product;
    the reduction brings a value into (-p, 2p) with the same residue."""
    import ctypes
    Rinv = pow(1 << 392, -1, P)
    out = (ctypes.c_int32 * 14)()
    for trial in range(60):
        vals = [rng.randrange(P) for _ in range(4)]
        if trial < 8:
            vals = [EDGE[trial % len(EDGE)] % P, P - 1, 0, 1][: 4]
        neg = trial % 3 == 1
        ls = [_redundant(v) for v in vals]
        if neg:  # signed inputs: -a, -d
            ls[0] = [-v for v in ls[0]]
            ls[3] = [-v for v in ls[3]]
        a, b, c, d = (_val(l) for l in ls)
        mx = lib().hc_row_mul2(_i32(ls[0]), _i32(ls[1]), _i32(ls[2]), _i32(ls[3]), out)
        got = _val(list(out))
        assert mx >= 0 and mx <= (1 << 28)
        assert (got - (a * b + c * d) * Rinv) % P == 0
        assert -P < got < 2 * P
        lib().hc_row_mul(_i32(ls[0]), _i32(ls[1]), out)
        got1 = _val(list(out))
        assert (got1 - a * b * Rinv) % P == 0 and -P < got1 < 2 * P
    for _ in range(40):
        x = rng.randrange(-(1 << 388), 1 << 388)
        l = [(abs(x) >> (28 * j)) & ((1 << 28) - 1) for j in range(13)] + [abs(x) >> (28 * 13)]
        if x < 0:
            l = [-v for v in l]
        lib().hc_row_reduce(_i32(l), out)
        got = _val(list(out))
        assert (got - x) % P == 0 and -P < got < 2 * P, (x, got)


def test_row_fp12_final_exp_matches_oracle():
    """bls_row.h Fp12 on rows (k_l0_final's layout: one Fp per 16-lane row,
    products on 36 rows, a phase per row role), rows emulated in turn:
    product, cyclotomic squaring, Frobenius and the whole final
    exponentiation equal the oracle's; a cancelling pairing product
    exponentiates to 1."""
    import ctypes
    a, b = rand_f12(), rand_f12()
    assert b2f12(call("hc_row_fp12_mul", f12b(a), f12b(b), out=576)) == bls.f12_mul(a, b)
    assert b2f12(call("hc_row_fp12_frob", f12b(a), out=576)) == bls.f12_frob_n(a, 1)
    f = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
    f = bls.f12_mul(bls.f12_frob_n(f, 2), f)
    assert b2f12(call("hc_row_fp12_cyc", f12b(f), out=576)) == bls.f12_sqr(f)
    out = ctypes.create_string_buffer(576)
    assert lib().hc_row_final_exp(f12b(a), out) == 0
    assert b2f12(out.raw) == bls.final_exp(a)
    p = bls.g1_mul(bls.G1_GEN, rng.randrange(1, bls.R))
    q = bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))
    m1 = b2f12(call("hc_miller", be(p[0]) + be(p[1]), aff2b(q), out=576))
    m2 = b2f12(call("hc_miller", be(p[0]) + be((P - p[1]) % P), aff2b(q), out=576))
    assert lib().hc_row_final_exp(f12b(bls.f12_mul(m1, m2)), out) == 1


def test_bernstein_yang_inversion():
    """fp_inv (bls_field.h, Bernstein-Yang divsteps in 62-bit batches, the
    inversion of every public value) equals Fermat's and the oracle's inverse
    on edge values and random ones; 0 maps to 0."""
    vals = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 1 << 380, (1 << 381) % P, 0xDEADBEEF]
    vals += [pow(2, k, P) for k in range(0, 381, 37)] + [rng.randrange(P) for _ in range(300)]
    import ctypes
    for v in vals:
        ob = ctypes.create_string_buffer(48)
        rc = lib().hc_inv_bgcd(be(v), ob)
        assert rc == 0, v
        assert fe(ob.raw) == (pow(v, P - 2, P) if v else 0)
        # the Montgomery form of v plus p, in [p, 2p) as device callers pass it
        # (v = p - 1 gives 2p - 1's representative)
        rc = lib().hc_inv_bgcd_plus_p(be(v), ob)
        assert rc == 0, v
        assert fe(ob.raw) == (pow(v, P - 2, P) if v else 0)


def test_row_g2_lines_match_lane_lines():
    """Level 0's S lines on rows (bls_row.h: each Fp2 product of a doubling /
    addition phase on two 16-lane rows) equal g2_lines's 68 lines, -g1
    folded in, Fp for Fp."""
    for _ in range(3):
        q = bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))
        assert lib().hc_row_lines(aff2b(q)) == 0
