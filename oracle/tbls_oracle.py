"""CPU oracle for Charon's threshold-BLS facade (``tbls``).

TEST INFRASTRUCTURE ONLY (see ``oracle/bls12_381.py``).  The product path never
imports this module.

Restates the control flow and error behaviour of
  * ``tbls.Verify``              reference ``tbls/tss.go:190-197``
  * ``tbls.Aggregate``           reference ``tbls/tss.go:142-149``
  * ``tbls.VerifyAndAggregate``  reference ``tbls/tss.go:153-187``
  * ``TSS`` / ``PublicShare``    reference ``tbls/tss.go:62-116``
  * ``tblsconv.SigFromCore`` / ``SigToCore``  reference ``tbls/tblsconv/tblsconv.go:119-132``
and of the kryptology calls they make (``SigEth2.Verify``,
``SigEth2.CombineSignatures``, ``SigEth2.Sign``), the latter restated from the
IETF BLS draft (POP ciphersuite) because kryptology is not vendored.

Edge cases NOT pinned by any reference test (kryptology's internal checks are
not visible in the reference snapshot) are marked "unpinned" below; the
GPU engine implements the same choices so the two agree, and DESIGN.md lists
them.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from . import bls12_381 as bls

R = bls.R


class TblsError(Exception):
    """Mirrors the Go ``error`` return (message text follows the reference)."""


# ----------------------------------------------------------------------------
# Keys and signing (test-vector generation; kryptology SigEth2 semantics)
# ----------------------------------------------------------------------------
def sk_to_pk(sk: int):
    return bls.g1_mul(bls.G1_GEN, sk)


def sign(sk: int, msg: bytes):
    """bls_sig SigEth2.Sign: sk * H(msg) with the POP DST."""
    return bls.g2_mul(bls.hash_to_g2(msg), sk)


def core_verify(pk_aff, msg: bytes, sig_aff) -> bool:
    """BLS CoreVerify: e(pk, H(m)) * e(-g1, sig) == 1.

    Unpinned edge cases (kryptology internals): an identity public key or an
    identity signature is rejected (returns False); the Go side sees this as
    a failed verification either way (``tss.go:170`` skips on ``err || !ok``).
    """
    if pk_aff is None or sig_aff is None:
        return False
    h = bls.hash_to_g2(msg)
    return bls.pairing_product_is_one([(pk_aff, h), (bls.g1_neg(bls.G1_GEN), sig_aff)])


def verify(pk_aff, msg: bytes, sig_aff) -> bool:
    """tbls.Verify (tss.go:190-197)."""
    return core_verify(pk_aff, msg, sig_aff)


# ----------------------------------------------------------------------------
# Lagrange recombination (SigEth2.CombineSignatures)
# ----------------------------------------------------------------------------
def lagrange_at_zero(ids):
    """lambda_i(0) = prod_{j != i} x_j / (x_j - x_i) mod r, x_i = Identifier."""
    out = []
    for i, xi in enumerate(ids):
        num, den = 1, 1
        for j, xj in enumerate(ids):
            if i == j:
                continue
            num = num * xj % R
            d = (xj - xi) % R
            if d == 0:
                raise TblsError("aggregate signatures: duplicate identifier")
            den = den * d % R
        out.append(num * pow(den, R - 2, R) % R)
    return out


def combine_signatures(partials):
    """partials: list of (identifier:int 0..255, sig_aff).  Returns the affine
    aggregate.  Errors (unpinned messages, pinned behaviour where noted):
      * fewer than 2 partials -> error (unpinned);
      * an identity partial -> error (unpinned);
      * duplicate identifiers -> error (Lagrange denominator is zero);
      * identity result -> error (unpinned).
    Identifier 0 is accepted (pinned by ``dkg/dkg_test.go:174-195``)."""
    if len(partials) < 2:
        raise TblsError("aggregate signatures: insufficient partial signatures")
    if len(partials) > 255:
        raise TblsError("aggregate signatures: too many partial signatures")
    ids = [int(i) for i, _ in partials]
    for _, s in partials:
        if s is None:
            raise TblsError("aggregate signatures: identity partial signature")
    lam = lagrange_at_zero(ids)
    acc = None
    for (_, s), l in zip(partials, lam):
        acc = bls.g2_add(acc, bls.g2_mul(s, l))
    if acc is None:
        raise TblsError("aggregate signatures: identity aggregate")
    return acc


def aggregate(partials):
    """tbls.Aggregate (tss.go:142-149)."""
    return combine_signatures(partials)


# ----------------------------------------------------------------------------
# TSS container and VerifyAndAggregate
# ----------------------------------------------------------------------------
@dataclass
class TSS:
    pubshares: dict  # int -> G1 affine
    num_shares: int
    threshold: int
    public_key: object = None

    def public_share(self, idx: int):
        return self.pubshares.get(idx)


def verify_and_aggregate(tss: TSS, partials, msg: bytes):
    """tbls.VerifyAndAggregate (tss.go:153-187).  Returns (agg_aff, signers).

    * len < threshold -> "insufficient signatures";
    * every partial is verified against PublicShare(Identifier) (a missing
      share verifies false), no early break (tss.go:164);
    * valid ones are kept in input order, with their identifiers;
    * < threshold valid -> "insufficient valid signatures";
    * CombineSignatures over ALL valid partials."""
    if len(partials) < tss.threshold:
        raise TblsError("insufficient signatures")
    valid, signers = [], []
    for ident, sig in partials:
        pk = tss.public_share(int(ident))
        if pk is None or sig is None:
            continue
        if not core_verify(pk, msg, sig):
            continue
        valid.append((ident, sig))
        signers.append(int(ident))
    if len(valid) < tss.threshold:
        raise TblsError("insufficient valid signatures")
    return combine_signatures(valid), signers


# ----------------------------------------------------------------------------
# Shamir / Feldman helpers for fixture generation (tss.go:120-139, 256-325)
# ----------------------------------------------------------------------------
def split_secret(secret: int, t: int, n: int, coeffs):
    """Shares f(1..n) of f(x) = secret + c_1 x + ... + c_{t-1} x^{t-1} mod r.
    ``coeffs`` are the t-1 random coefficients (supplied by a seeded PRNG)."""
    poly = [secret % R] + [c % R for c in coeffs]
    assert len(poly) == t
    shares = {}
    for i in range(1, n + 1):
        acc = 0
        for c in reversed(poly):
            acc = (acc * i + c) % R
        shares[i] = acc
    return shares, poly


def generate_tss(secret: int, t: int, n: int, coeffs):
    shares, poly = split_secret(secret, t, n, coeffs)
    pubshares = {i: sk_to_pk(s) for i, s in shares.items()}
    return TSS(pubshares=pubshares, num_shares=n, threshold=t, public_key=sk_to_pk(secret)), shares
