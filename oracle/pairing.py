"""ORACLE (test infrastructure only) -- optimal-ate pairing on BLS12-381.

Restates blst's ``miller_loop_n`` / ``final_exp`` (un-vendored @chainsafe/blst@0.2.8),
reached from ``Signature.verifyMultipleSignatures`` / ``verify``
(packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37).

Two independent Miller loops are kept:
- ``miller_loop_textbook``: affine points untwisted into E(Fp12), full Fp12 line values.
  Obviously-correct reference; slow.
- ``miller_loop_fast``: homogeneous-projective G2 steps with sparse lines
  (c0 = (A, B, 0), c1 = (0, C, 0)), the *same formulas, operation for operation*, as the
  HIP kernels (lodestar_amd/csrc/pairing.hip), so intermediate values can be compared
  bit-exactly with the GPU.
They agree after the final exponentiation (tests/test_oracle_pairing.py).

Final exponentiation ``final_exp_fast`` computes f^(3 (p^12-1)/r) (hard part via
3*Phi12(p)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3); ``final_exp_textbook`` is pow(f, (p^12-1)/r).
The verdict "== 1" is the same for both because gcd(3, r) = 1.
"""
from .fields import (
    P, R, X, X_ABS, F2_ZERO, F2_ONE, F6_ZERO, F12_ONE,
    f2_add, f2_sub, f2_mul, f2_sqr, f2_neg, f2_mul_fp, f2_mul_xi, f2_is_zero,
    f6_add, f6_sub, f6_mul, f6_mul_v,
    f12_mul, f12_sqr, f12_conj, f12_inv, f12_pow, f12_frob, f12_frob2, f12_sub, f12_add,
    f12_from_f2, f12_is_one,
)

# ---------------------------------------------------------------- textbook Miller loop
_W = (F6_ZERO, (F2_ONE, F2_ZERO, F2_ZERO))  # w
_W_INV = f12_inv(_W)
_W_INV2 = f12_mul(_W_INV, _W_INV)
_W_INV3 = f12_mul(_W_INV2, _W_INV)


def _f12_fp(a):
    return f12_from_f2((a % P, 0))


def untwist(Q):
    x, y = Q
    return (f12_mul(f12_from_f2(x), _W_INV2), f12_mul(f12_from_f2(y), _W_INV3))


def _f12_div(a, b):
    return f12_mul(a, f12_inv(b))


def miller_loop_textbook(Pt, Q):
    """f_{x,Q}(P) with the ate loop over |x| then conjugated (x < 0).  P in E(Fp), Q in E2."""
    if Pt is None or Q is None:
        return F12_ONE
    xP, yP = _f12_fp(Pt[0]), _f12_fp(Pt[1])
    Qx, Qy = untwist(Q)
    Tx, Ty = Qx, Qy
    f = F12_ONE
    for i in range(X_ABS.bit_length() - 2, -1, -1):
        # tangent at T
        lam = _f12_div(f12_mul(_f12_fp(3), f12_sqr(Tx)), f12_add(Ty, Ty))
        line = f12_sub(f12_sub(yP, Ty), f12_mul(lam, f12_sub(xP, Tx)))
        f = f12_mul(f12_sqr(f), line)
        nx = f12_sub(f12_sqr(lam), f12_add(Tx, Tx))
        Ty = f12_sub(f12_mul(lam, f12_sub(Tx, nx)), Ty)
        Tx = nx
        if (X_ABS >> i) & 1:
            lam = _f12_div(f12_sub(Qy, Ty), f12_sub(Qx, Tx))
            line = f12_sub(f12_sub(yP, Ty), f12_mul(lam, f12_sub(xP, Tx)))
            f = f12_mul(f, line)
            nx = f12_sub(f12_sub(f12_sqr(lam), Tx), Qx)
            Ty = f12_sub(f12_mul(lam, f12_sub(Tx, nx)), Ty)
            Tx = nx
    return f12_conj(f)


def final_exp_textbook(f):
    return f12_pow(f, (P ** 12 - 1) // R)


# ---------------------------------------------------------------- fast (GPU-mirrored) path
B3_E2 = (12, 12)  # 3 * 4 * (1 + u)


def f2_mul_b3(a):
    # (12 + 12u)(a0 + a1 u) = 12 (a0 - a1) + 12 (a0 + a1) u
    return ((12 * (a[0] - a[1])) % P, (12 * (a[0] + a[1])) % P)


def dbl_step(T, xP, yP):
    """T <- 2T (homogeneous projective on E2), returns (line, T') with
    line = (l00, l01, l11): l00 = 3b'Z^2 - Y^2, l01 = 3X^2 * xP, l11 = -2YZ * yP."""
    X1, Y1, Z1 = T
    t0 = f2_sqr(Y1)
    t1 = f2_mul(Y1, Z1)
    t2 = f2_mul_b3(f2_sqr(Z1))
    XX = f2_sqr(X1)
    l00 = f2_sub(t2, t0)
    XX3 = f2_add(f2_add(XX, XX), XX)
    l01 = f2_mul_fp(XX3, xP)
    l11 = f2_mul_fp(f2_neg(f2_add(t1, t1)), yP)
    # Renes-Costello-Batina 2016, algorithm 9 (a = 0)
    Z3 = f2_add(t0, t0)
    Z3 = f2_add(Z3, Z3)
    Z3 = f2_add(Z3, Z3)
    X3 = f2_mul(t2, Z3)
    Y3 = f2_add(t0, t2)
    Z3 = f2_mul(t1, Z3)
    u1 = f2_add(t2, t2)
    u2 = f2_add(u1, t2)
    s0 = f2_sub(t0, u2)
    Y3 = f2_mul(s0, Y3)
    Y3 = f2_add(X3, Y3)
    v1 = f2_mul(X1, Y1)
    X3 = f2_mul(s0, v1)
    X3 = f2_add(X3, X3)
    return (l00, l01, l11), (X3, Y3, Z3)


def add_step(T, Q, xP, yP):
    """T <- T + Q (Q affine), returns (line, T') with theta = Y - yQ Z, delta = X - xQ Z,
    l00 = delta*yQ - theta*xQ, l01 = theta * xP, l11 = -delta * yP."""
    X1, Y1, Z1 = T
    xQ, yQ = Q
    theta = f2_sub(Y1, f2_mul(yQ, Z1))
    delta = f2_sub(X1, f2_mul(xQ, Z1))
    l00 = f2_sub(f2_mul(delta, yQ), f2_mul(theta, xQ))
    l01 = f2_mul_fp(theta, xP)
    l11 = f2_mul_fp(f2_neg(delta), yP)
    C = f2_sqr(theta)
    D = f2_sqr(delta)
    E = f2_mul(D, delta)
    F = f2_mul(Z1, C)
    G = f2_mul(X1, D)
    H = f2_sub(f2_add(E, F), f2_add(G, G))
    X3 = f2_mul(delta, H)
    Y3 = f2_sub(f2_mul(theta, f2_sub(G, H)), f2_mul(E, Y1))
    Z3 = f2_mul(E, Z1)
    return (l00, l01, l11), (X3, Y3, Z3)


def f6_mul_01(a, b0, b1):
    """(a0 + a1 v + a2 v^2)(b0 + b1 v)."""
    a0, a1, a2 = a
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    c0 = f2_add(f2_mul_xi(f2_mul(a2, b1)), t0)
    c1 = f2_sub(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), t0), t1)
    c2 = f2_add(f2_mul(a2, b0), t1)
    return (c0, c1, c2)


def f6_mul_1(a, b1):
    """(a0 + a1 v + a2 v^2)(b1 v)."""
    a0, a1, a2 = a
    return (f2_mul_xi(f2_mul(a2, b1)), f2_mul(a0, b1), f2_mul(a1, b1))


def f12_mul_line(f, line):
    """f * ((l00 + l01 v) + (l11 v) w)."""
    l00, l01, l11 = line
    f0, f1 = f
    t0 = f6_mul_01(f0, l00, l01)
    t1 = f6_mul_1(f1, l11)
    s = f6_add(f0, f1)
    c1 = f6_sub(f6_sub(f6_mul_01(s, l00, f2_add(l01, l11)), t0), t1)
    c0 = f6_add(t0, f6_mul_v(t1))
    return (c0, c1)


def line_to_f12(line):
    l00, l01, l11 = line
    return ((l00, l01, F2_ZERO), (F2_ZERO, l11, F2_ZERO))


def miller_loop_fast(Pt, Q):
    if Pt is None or Q is None:
        return F12_ONE
    xP, yP = Pt
    T = (Q[0], Q[1], F2_ONE)
    f = F12_ONE
    first = True
    for i in range(X_ABS.bit_length() - 2, -1, -1):
        if not first:
            f = f12_sqr(f)
        line, T = dbl_step(T, xP, yP)
        f = line_to_f12(line) if first else f12_mul_line(f, line)
        first = False
        if (X_ABS >> i) & 1:
            line, T = add_step(T, Q, xP, yP)
            f = f12_mul_line(f, line)
    return f12_conj(f)


def miller_loop_lines(Pt, Q):
    """The sequence of (kind, line) the fast loop multiplies in -- for GPU stage tests."""
    xP, yP = Pt
    T = (Q[0], Q[1], F2_ONE)
    out = []
    for i in range(X_ABS.bit_length() - 2, -1, -1):
        line, T = dbl_step(T, xP, yP)
        out.append(("dbl", line))
        if (X_ABS >> i) & 1:
            line, T = add_step(T, Q, xP, yP)
            out.append(("add", line))
    return out


def f12_exp_by_x(g):
    """g^x for g in the cyclotomic subgroup (x < 0: conjugate of g^|x|)."""
    res = F12_ONE
    for i in range(X_ABS.bit_length() - 1, -1, -1):
        res = f12_sqr(res)
        if (X_ABS >> i) & 1:
            res = f12_mul(res, g)
    return f12_conj(res)


def final_exp_easy(f):
    f1 = f12_mul(f12_conj(f), f12_inv(f))
    return f12_mul(f12_frob2(f1), f1)


def final_exp_hard(g):
    t0 = f12_mul(f12_exp_by_x(g), f12_conj(g))
    t0 = f12_mul(f12_exp_by_x(t0), f12_conj(t0))
    t1 = f12_mul(f12_exp_by_x(t0), f12_frob(t0))
    t2 = f12_mul(f12_mul(f12_exp_by_x(f12_exp_by_x(t1)), f12_frob2(t1)), f12_conj(t1))
    return f12_mul(t2, f12_mul(f12_sqr(g), g))


def final_exp_fast(f):
    return final_exp_hard(final_exp_easy(f))


def pairing(Pt, Q):
    return final_exp_fast(miller_loop_fast(Pt, Q))


def multi_miller_loop(pairs):
    f = F12_ONE
    for Pt, Q in pairs:
        f = f12_mul(f, miller_loop_fast(Pt, Q))
    return f


def pairing_check(pairs):
    """prod e(P_i, Q_i) == 1 ?"""
    return f12_is_one(final_exp_fast(multi_miller_loop(pairs)))


# ---------------------------------------------------------------- cyclotomic squaring
def _fp4_square(a, b):
    """(a + b t)^2 in Fp4 = Fp2[t]/(t^2 - xi): returns (c0, c1)."""
    from .fields import f2_mul_xi
    t0 = f2_sqr(a)
    t1 = f2_sqr(b)
    c0 = f2_add(f2_mul_xi(t1), t0)
    t2 = f2_sub(f2_sub(f2_sqr(f2_add(a, b)), t0), t1)
    return c0, t2


def f12_cyclotomic_sqr(f):
    """Granger-Scott squaring, valid for f in the cyclotomic subgroup (after the easy part);
    the GPU's fp12_cyclotomic_sqr (lodestar_amd/csrc/lsg_tower.hpp) mirrors it."""
    (z0, z4, z3), (z2, z1, z5) = f
    t0, t1 = _fp4_square(z0, z1)
    z0 = f2_sub(t0, z0)
    z0 = f2_add(f2_add(z0, z0), t0)
    z1 = f2_add(t1, z1)
    z1 = f2_add(f2_add(z1, z1), t1)
    t0, t1 = _fp4_square(z2, z3)
    t2, t3 = _fp4_square(z4, z5)
    z4 = f2_sub(t0, z4)
    z4 = f2_add(f2_add(z4, z4), t0)
    z5 = f2_add(t1, z5)
    z5 = f2_add(f2_add(z5, z5), t1)
    t0 = f2_mul_xi(t3)
    z2 = f2_add(t0, z2)
    z2 = f2_add(f2_add(z2, z2), t0)
    z3 = f2_sub(t2, z3)
    z3 = f2_add(f2_add(z3, z3), t2)
    return ((z0, z4, z3), (z2, z1, z5))
