"""ORACLE (test infrastructure only) -- independent derivation of the 3-isogeny
E2' -> E2 used by hash_to_G2 (RFC 9380 section 8.8.2, suite BLS12381G2_XMD:SHA-256_SSWU_RO_).

blst (un-vendored, @chainsafe/blst@0.2.8) hard-codes the isogeny's rational-map
coefficients.  Rather than trusting transcribed hex, the oracle *derives* them here
with Velu's formulas from the SSWU curve E2': y^2 = x^3 + 240u x + 1012(1+u):
  1. find the roots x0 in Fp2 of the 3-division polynomial of E2',
  2. Velu's isogeny for kernel <(x0, .)> gives a codomain y^2 = x^3 + A x + B,
  3. keep the kernels whose codomain has A = 0 and compose with each isomorphism
     (x, y) -> (mu^2 x, mu^3 y), mu^6 = 4(1+u)/B, onto E2: y^2 = x^3 + 4(1+u).
That leaves a handful of candidate maps differing by an automorphism of E2; the genesis
known-answer signature (tests/test_oracle_kat.py) selects the one blst uses.
"""
import random

from .fields import (
    P, F2_ZERO, F2_ONE, f2_add, f2_sub, f2_mul, f2_sqr, f2_inv, f2_is_zero, f2_neg, f2_pow, f2_eq,
)

A_ISO = (0, 240)
B_ISO = (1012, 1012)
B_E2 = (4, 4)


# --- polynomials over Fp2 as lists of coefficients, lowest degree first
def _trim(a):
    a = list(a)
    while a and f2_is_zero(a[-1]):
        a.pop()
    return a


def _pmul(a, b):
    if not a or not b:
        return []
    out = [F2_ZERO] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            out[i + j] = f2_add(out[i + j], f2_mul(x, y))
    return _trim(out)


def _pdivmod(a, b):
    a = _trim(a)
    b = _trim(b)
    inv_lead = f2_inv(b[-1])
    q = [F2_ZERO] * max(len(a) - len(b) + 1, 1)
    while len(a) >= len(b) and a:
        c = f2_mul(a[-1], inv_lead)
        d = len(a) - len(b)
        q[d] = c
        for i, y in enumerate(b):
            a[i + d] = f2_sub(a[i + d], f2_mul(c, y))
        a = _trim(a)
    return _trim(q), a


def _pmod(a, b):
    return _pdivmod(a, b)[1]


def _pgcd(a, b):
    a = _trim(a)
    b = _trim(b)
    while b:
        a, b = b, _pmod(a, b)
    inv = f2_inv(a[-1])
    return [f2_mul(c, inv) for c in a]


def _ppowmod(base, e, m):
    res = [F2_ONE]
    base = _pmod(base, m)
    while e > 0:
        if e & 1:
            res = _pmod(_pmul(res, base), m)
        base = _pmod(_pmul(base, base), m)
        e >>= 1
    return res


def _roots(f, rng):
    """All roots in Fp2 of a squarefree-ish polynomial f (Cantor-Zassenhaus)."""
    q = P * P
    xq = _ppowmod([F2_ZERO, F2_ONE], q, f)
    g = _pgcd(f, _trim(f2_lst_sub(xq, [F2_ZERO, F2_ONE])))
    out = []

    def split(h):
        h = _trim(h)
        if len(h) <= 1:
            return
        if len(h) == 2:
            out.append(f2_neg(f2_mul(h[0], f2_inv(h[1]))))
            return
        while True:
            a = (rng.randrange(P), rng.randrange(P))
            t = _ppowmod([a, F2_ONE], (q - 1) // 2, h)
            d = _pgcd(h, _trim(f2_lst_sub(t, [F2_ONE])))
            if 1 < len(d) < len(h):
                split(d)
                split(_pdivmod(h, d)[0])
                return

    split(g)
    return out


def _padd(a, b):
    n = max(len(a), len(b))
    a = list(a) + [F2_ZERO] * (n - len(a))
    b = list(b) + [F2_ZERO] * (n - len(b))
    return _trim([f2_add(x, y) for x, y in zip(a, b)])


def f2_lst_sub(a, b):
    n = max(len(a), len(b))
    a = list(a) + [F2_ZERO] * (n - len(a))
    b = list(b) + [F2_ZERO] * (n - len(b))
    return [f2_sub(x, y) for x, y in zip(a, b)]


def _f2_sixth_roots(c, rng):
    """All mu with mu^6 = c."""
    return _roots(_trim([f2_neg(c), F2_ZERO, F2_ZERO, F2_ZERO, F2_ZERO, F2_ZERO, F2_ONE]), rng)


def derive_iso3_candidates(seed=1):
    """Return a list of candidate maps (xnum, xden, ynum, yden), each a coefficient list
    (lowest degree first, Fp2 coefficients) with x = xnum/xden, y = y' * ynum/yden."""
    rng = random.Random(seed)
    a, b = A_ISO, B_ISO
    # 3-division polynomial psi_3 = 3x^4 + 6a x^2 + 12 b x - a^2
    psi3 = _trim([f2_neg(f2_sqr(a)), f2_mul((12, 0), b), f2_mul((6, 0), a), F2_ZERO, (3, 0)])
    cands = []
    for x0 in _roots(psi3, rng):
        gx = f2_add(f2_mul((3, 0), f2_sqr(x0)), a)  # 3 x0^2 + a
        v = f2_add(gx, gx)  # 6 x0^2 + 2a
        u = f2_mul((4, 0), f2_add(f2_add(f2_mul(f2_sqr(x0), x0), f2_mul(a, x0)), b))  # 4 y0^2
        w = f2_add(u, f2_mul(x0, v))
        A = f2_sub(a, f2_mul((5, 0), v))
        B = f2_sub(b, f2_mul((7, 0), w))
        if not f2_is_zero(A):
            continue
        # X = x + v/(x-x0) + u/(x-x0)^2 = (x (x-x0)^2 + v (x-x0) + u) / (x-x0)^2
        lin = [f2_neg(x0), F2_ONE]
        sq = _pmul(lin, lin)
        cu = _pmul(sq, lin)
        xnum = _padd(_padd(_pmul([F2_ZERO, F2_ONE], sq), _pmul([v], lin)), [u])
        # Y = y (1 - v/(x-x0)^2 - 2u/(x-x0)^3) = y ((x-x0)^3 - v (x-x0) - 2u) / (x-x0)^3
        ynum = f2_lst_sub(f2_lst_sub(cu, _pmul([v], lin)), [f2_add(u, u)])
        for mu in _f2_sixth_roots(f2_mul(B_E2, f2_inv(B)), rng):
            mu2 = f2_sqr(mu)
            mu3 = f2_mul(mu2, mu)
            cands.append(([f2_mul(c, mu2) for c in xnum], sq, [f2_mul(c, mu3) for c in ynum], cu))
    return cands
