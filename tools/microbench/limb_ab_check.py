"""Checks limb_ab's printed 13 x 30-bit Montgomery products against big
integers: r = a b 2^-390 mod p (in [0, 2p)), r2 = 2 a b 2^-390 mod p."""
import sys

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab


def val(ws):
    return sum(int(w, 16) << (30 * i) for i, w in enumerate(ws))


for line in open(sys.argv[1]):
    if not line.startswith("check"):
        continue
    t = line.split()
    a, b, r, r2 = val(t[2:15]), val(t[16:29]), val(t[30:43]), val(t[44:57])
    rinv = pow(2, -390, P)
    assert r % P == a * b * rinv % P and r < 2 * P, "fp30_mul"
    assert r2 % P == 2 * a * b * rinv % P and r2 < 2 * P, "fp30_mul2"
    print("limb_ab check ok")
