"""ORACLE (test infrastructure only) -- BLS12-381 field tower in pure Python big ints.

This file is part of the CPU *checker*.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``lodestar_amd``) never does.

What it restates: the field arithmetic that @chainsafe/blst@0.2.8 (supranational
blst, un-vendored npm dependency; pinned in /root/reference/yarn.lock:492-497)
performs underneath ``Signature.verifyMultipleSignatures`` / ``Signature.verify``
(called from packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37).

Tower (the standard BLS12-381 tower, identical to blst's):
  Fp2  = Fp[u]  / (u^2 + 1)
  Fp6  = Fp2[v] / (v^3 - xi),  xi = 1 + u
  Fp12 = Fp6[w] / (w^2 - v)
Representation: Fp = int, Fp2 = (a0, a1), Fp6 = (c0, c1, c2), Fp12 = (d0, d1).
"""

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
# group order r (also in /root/reference/packages/state-transition/src/util/interop.ts:9)
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
# BLS parameter x (negative)
X_ABS = 0xD201000000010000
X = -X_ABS

# ---------------------------------------------------------------- Fp

def fp_inv(a):
    if a % P == 0:
        raise ZeroDivisionError("fp_inv(0)")
    return pow(a, -1, P)


def fp_sqrt(a):
    """Return a square root of a in Fp or None (p = 3 mod 4)."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


# ---------------------------------------------------------------- Fp2
F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (1, 1)


def f2(a0, a1=0):
    return (a0 % P, a1 % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_mul_fp(a, k):
    return (a[0] * k % P, a[1] * k % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_mul_xi(a):
    # (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = fp_inv(n)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def f2_is_zero(a):
    return a[0] % P == 0 and a[1] % P == 0


def f2_eq(a, b):
    return (a[0] - b[0]) % P == 0 and (a[1] - b[1]) % P == 0


def f2_pow(a, e):
    res = F2_ONE
    base = a
    while e > 0:
        if e & 1:
            res = f2_mul(res, base)
        base = f2_sqr(base)
        e >>= 1
    return res


def f2_is_square(a):
    # a is a square in Fp2 iff its norm is a square in Fp
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """A square root of a in Fp2 or None.  Which root is returned is irrelevant to
    callers: every caller fixes the sign afterwards (compression flag or sgn0)."""
    a = (a[0] % P, a[1] % P)
    if f2_is_zero(a):
        return F2_ZERO
    a0, a1 = a
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0)
        return (0, s)  # (s u)^2 = -s^2 = a0
    n = fp_sqrt(a0 * a0 + a1 * a1)
    if n is None:
        return None
    inv2 = fp_inv(2)
    for cand in ((a0 + n) * inv2 % P, (a0 - n) * inv2 % P):
        x0 = fp_sqrt(cand)
        if x0 is not None and x0 != 0:
            x1 = a1 * fp_inv(2 * x0) % P
            res = (x0, x1)
            if f2_eq(f2_sqr(res), a):
                return res
    return None


def f2_sgn0(a):
    """RFC 9380 sgn0 for Fp2."""
    sign_0 = a[0] % 2
    zero_0 = a[0] == 0
    sign_1 = a[1] % 2
    return sign_0 | (zero_0 and sign_1)


def f2_lexi_largest(y):
    """ZCash 'y is lexicographically largest' flag (blst sgn0_pty bit 1)."""
    half = (P - 1) // 2
    if y[1] != 0:
        return y[1] > half
    return y[0] > half


# ---------------------------------------------------------------- Fp6
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    # c0 = a0 b0 + xi (a1 b2 + a2 b1)
    c0 = f2_add(t0, f2_mul_xi(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    # c1 = a0 b1 + a1 b0 + xi a2 b2
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_xi(t2))
    # c2 = a0 b2 + a1 b1 + a2 b0
    c2 = f2_add(f2_add(f2_mul(a0, b2), t1), f2_mul(a2, b0))
    return (c0, c1, c2)


def f6_mul_v(a):
    # (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_mul_f2(a, k):
    return (f2_mul(a[0], k), f2_mul(a[1], k), f2_mul(a[2], k))


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    den = f2_add(f2_mul(a0, t0), f2_mul_xi(f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(den)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


# ---------------------------------------------------------------- Fp12
F12_ONE = (F6_ONE, F6_ZERO)
F12_ZERO = (F6_ZERO, F6_ZERO)


def f12_add(a, b):
    return (f6_add(a[0], b[0]), f6_add(a[1], b[1]))


def f12_sub(a, b):
    return (f6_sub(a[0], b[0]), f6_sub(a[1], b[1]))


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
    c0 = f6_add(t0, f6_mul_v(t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e):
    if e < 0:
        a = f12_inv(a)
        e = -e
    res = F12_ONE
    base = a
    while e > 0:
        if e & 1:
            res = f12_mul(res, base)
        base = f12_sqr(base)
        e >>= 1
    return res


def f12_eq(a, b):
    return all(f2_eq(x, y) for x, y in zip(a[0] + a[1], b[0] + b[1]))


def f12_is_one(a):
    return f12_eq(a, F12_ONE)


def f12_from_f2(c):
    return ((c, F2_ZERO, F2_ZERO), F6_ZERO)


def f12_coeffs(a):
    """Flatten to the 6 Fp2 coefficients in order (d0.c0, d0.c1, d0.c2, d1.c0, d1.c1, d1.c2)."""
    return list(a[0]) + list(a[1])


# Frobenius: a^p.  Computed generically from the definition (conjugate coefficients
# and multiply by gamma constants = powers of xi).  Used by the textbook paths and
# the fast final exponentiation.
def _gamma(k, i):
    # gamma_{k,i} = xi^{i (p^k - 1)/6}
    return f2_pow(XI, i * (P ** k - 1) // 6)


GAMMA1 = [_gamma(1, i) for i in range(6)]
GAMMA2 = [_gamma(2, i) for i in range(6)]


def f12_frob(a):
    """a^p.  Element a = sum_{j} c_j w^j with c_j in Fp2, where w^j for j = 0..5
    indexes (d0.c0, d1.c0, d0.c1, d1.c1, d0.c2, d1.c2) (since v = w^2)."""
    (c00, c01, c02), (c10, c11, c12) = a
    # coefficient of w^j : j = 0: c00, 1: c10, 2: c01, 3: c11, 4: c02, 5: c12
    def fr(c, j):
        return f2_mul(f2_conj(c), GAMMA1[j])
    return ((fr(c00, 0), fr(c01, 2), fr(c02, 4)), (fr(c10, 1), fr(c11, 3), fr(c12, 5)))


def f12_frob2(a):
    (c00, c01, c02), (c10, c11, c12) = a
    def fr(c, j):
        return f2_mul(c, GAMMA2[j])
    return ((fr(c00, 0), fr(c01, 2), fr(c02, 4)), (fr(c10, 1), fr(c11, 3), fr(c12, 5)))
