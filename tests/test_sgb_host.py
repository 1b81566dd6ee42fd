"""The batched G2 subgroup test (charon_amd/csrc/k_sgb.hip) on the host:
the kernels' math compiled for the CPU (tests/hostcheck, lane pairs
emulated) against the oracle's exact subgroup decisions.

A group of decoded signatures passes iff all 18 random combinations
sum c_i s_i (c_i uniform mod 13, bls_rlc.h sgb_digits) satisfy
psi(Q) == [x] Q.  Checked here: the digits' range and distribution, a group
of G2 points passes, and every crafted non-subgroup kind of
tests/golden/sgb_points.json (13- and 23-torsion components, a bare torsion
point, a pair whose components cancel in a plain sum) fails the group at any
position, with decode failures left out of the sums.  The per-item verdicts
(k_subgroup_sigs after a failed group) are checked on the GPU against
oracle/c (tests/test_gpu_sgb.py).
"""
import ctypes
import json
import os
import random

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hc():
    from tests.hostcheck import lib
    h = lib()
    h.hc_sgb_group.restype = ctypes.c_int
    h.hc_sgb_group.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32]
    h.hc_sgb_digits.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    return h


@pytest.fixture(scope="module")
def crafted():
    with open(os.path.join(HERE, "golden", "sgb_points.json")) as f:
        return {k: [bytes.fromhex(h) for h in v] for k, v in json.load(f)["points"].items()}


@pytest.fixture(scope="module")
def g2_points():
    from oracle import bls12_381 as bls
    rng = random.Random(0x5B)
    return [bls.g2_compress(bls.g2_mul(bls.G2_GEN, rng.randrange(1, bls.R))) for _ in range(48)]


SEED = np.array([0x01234567, 0x89ABCDEF, 0x0F1E2D3C, 0x4B5A6978, 0x11111111, 0x22222222, 0x33333333, 0x44444444],
                dtype=np.uint32)


def group_mask(hc, sigs, i0=0, seed=SEED):
    buf = b"".join(sigs)
    return hc.hc_sgb_group(buf, len(sigs), seed.ctypes.data_as(ctypes.c_void_p), i0)


def test_digits_uniform_mod_13(hc):
    out = np.zeros(18, dtype=np.int32)
    counts = np.zeros(13, dtype=np.int64)
    n = 4000
    for i in range(n):
        hc.hc_sgb_digits(SEED.ctypes.data_as(ctypes.c_void_p), i, out.ctypes.data_as(ctypes.c_void_p))
        assert out.min() >= -6 and out.max() <= 6
        np.add.at(counts, out + 6, 1)
    exp = n * 18 / 13
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    assert chi2 < 40, counts  # 12 degrees of freedom: p ~ 1e-4 at 40


def test_digits_depend_on_seed_and_index(hc):
    a, b, c = (np.zeros(18, dtype=np.int32) for _ in range(3))
    other = SEED.copy()
    other[7] ^= 1
    hc.hc_sgb_digits(SEED.ctypes.data_as(ctypes.c_void_p), 5, a.ctypes.data_as(ctypes.c_void_p))
    hc.hc_sgb_digits(SEED.ctypes.data_as(ctypes.c_void_p), 6, b.ctypes.data_as(ctypes.c_void_p))
    hc.hc_sgb_digits(other.ctypes.data_as(ctypes.c_void_p), 5, c.ctypes.data_as(ctypes.c_void_p))
    assert not np.array_equal(a, b) and not np.array_equal(a, c)


def test_group_of_g2_points_passes(hc, g2_points):
    assert group_mask(hc, g2_points) == 0
    assert group_mask(hc, g2_points, i0=512 * 7) == 0


@pytest.mark.parametrize("kind", ["t13", "t23", "torsion13"])
@pytest.mark.parametrize("pos", [0, 17, 47])
def test_crafted_point_fails_the_group(hc, g2_points, crafted, kind, pos):
    from oracle import bls12_381 as bls
    sigs = list(g2_points)
    sigs[pos] = crafted[kind][pos % len(crafted[kind])]
    with pytest.raises(bls.DecodeError):
        bls.g2_decompress(sigs[pos])  # the oracle's exact decision: outside G2
    assert group_mask(hc, sigs) != 0


def test_cancelling_pair_fails_the_group(hc, g2_points, crafted):
    from oracle import bls12_381 as bls
    a, b = crafted["pair_a"][0], crafted["pair_b"][0]
    # their torsion components cancel in a plain sum: both decode outside G2,
    # their sum is in G2 -- only the random coefficients separate them
    pa, pb = bls.g2_decompress(a, subgroup_check=False), bls.g2_decompress(b, subgroup_check=False)
    assert bls.g2_in_subgroup(bls.g2_add(pa, pb))
    sigs = list(g2_points)
    sigs[3], sigs[40] = a, b
    assert group_mask(hc, sigs) != 0
    for seed_word in range(1, 6):  # every seed separates them (13^-18 per seed)
        seed = SEED.copy()
        seed[0] = seed_word
        assert group_mask(hc, sigs, seed=seed) != 0


def test_two_bad_points_in_one_group(hc, g2_points, crafted):
    sigs = list(g2_points)
    sigs[1], sigs[2] = crafted["t13"][1], crafted["t13"][2]
    assert group_mask(hc, sigs) != 0


def test_decode_failures_are_left_out(hc, g2_points):
    sigs = list(g2_points)
    bad = bytearray(sigs[5])
    bad[0] &= 0x7F  # no compression flag: a decode error, not a member of any sum
    sigs[5] = bytes(bad)
    assert group_mask(hc, sigs) == 0
