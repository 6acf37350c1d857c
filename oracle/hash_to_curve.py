"""ORACLE (test infrastructure only) -- hash_to_G2 as blst performs it for
@chainsafe/blst's ``Pairing(hash_or_encode=true, DST)`` contexts (the call chain under
``Signature.verifyMultipleSignatures`` / ``verify``,
packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37).

Suite: BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380 section 8.8.2) with the Ethereum
proof-of-possession DST ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_``.

Steps (RFC 9380 sections 5.3.1, 5.2, 6.6.2, 6.6.3, 7, appendix G.3):
  expand_message_xmd(SHA-256, 256 bytes) -> 4 Fp -> u0, u1 in Fp2
  -> simplified SWU on E2' (A' = 240u, B' = 1012(1+u), Z = -(2+u))
  -> 3-isogeny E2' -> E2 -> Q0 + Q1 -> clear_cofactor (Budroni-Pintore psi form).
The isogeny coefficients are derived (oracle/iso3_derive.py) and the candidate is
selected by the genesis known-answer test; ISO_CANDIDATE records that choice.
"""
import hashlib

from .fields import (
    P, X, F2_ZERO, F2_ONE, f2_add, f2_sub, f2_mul, f2_sqr, f2_inv, f2_is_zero, f2_neg,
    f2_is_square, f2_sqrt, f2_sgn0,
)
from .curves import E2, psi

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)


def expand_message_xmd(msg, dst, len_in_bytes):
    b_in_bytes = 32
    r_in_bytes = 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(r_in_bytes)
    l_i_b_str = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b_str + b"\x00" + dst_prime).digest()
    b = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(2, ell + 1):
        prev = bytes(x ^ y for x, y in zip(b0, b[-1]))
        b.append(hashlib.sha256(prev + bytes([i]) + dst_prime).digest())
    return b"".join(b)[:len_in_bytes]


def hash_to_field_fp2(msg, dst, count=2):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off:off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


def map_to_curve_sswu(u):
    """RFC 9380 section 6.6.2 (simple, non-constant-time form).  Returns a point on E2'."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    tv1 = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(tv1)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


# --- 3-isogeny coefficients (lowest degree first; Fp2 = (c0, c1)).
# Derived by Velu's formulas in oracle/iso3_derive.py (candidate index 5 of
# derive_iso3_candidates(seed=1)); the candidate is the unique one of the six for which
# sign(interop sk #0, signing_root) reproduces the genesis KAT signature
# (packages/beacon-node/test/e2e/interop/genesisState.test.ts:54-55).
# tests/test_oracle_kat.py re-derives and re-checks both facts.
XNUM = [
    (0x05c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6,
     0x05c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6),
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000,
     0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a),
    (0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e,
     0x08ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d),
    (0x171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1,
     0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000),
]
XDEN = [
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000,
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63),
    (0x00000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000c,
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f),
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000001,
     0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000),
]
YNUM = [
    (0x1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706,
     0x1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706),
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000,
     0x05c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be),
    (0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c,
     0x08ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f),
    (0x124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10,
     0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000),
]
YDEN = [
    (0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb,
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb),
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000,
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3),
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000012,
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99),
    (0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000001,
     0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000),
]
ISO3 = (XNUM, XDEN, YNUM, YDEN)


def iso_coeffs():
    return ISO3


def _peval(c, x):
    acc = F2_ZERO
    for coef in reversed(c):
        acc = f2_add(f2_mul(acc, x), coef)
    return acc


def iso_map(Pt):
    if Pt is None:
        return None
    xnum, xden, ynum, yden = iso_coeffs()
    x, y = Pt
    xd = _peval(xden, x)
    yd = _peval(yden, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None  # kernel point -> infinity
    return (f2_mul(_peval(xnum, x), f2_inv(xd)), f2_mul(y, f2_mul(_peval(ynum, x), f2_inv(yd))))


def clear_cofactor(Pt):
    """h_eff * P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)  (RFC 9380 appendix G.3)."""
    t1 = E2.mul(Pt, X * X - X - 1)
    t2 = E2.mul(psi(Pt), X - 1)
    t3 = psi(psi(E2.dbl(Pt)))
    return E2.add(E2.add(t1, t2), t3)


# RFC 9380 section 8.8.2 h_eff (cross-checked against the psi form in the tests)
H_EFF_G2 = int(
    "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551",
    16,
)


def map_to_curve_g2(u):
    return iso_map(map_to_curve_sswu(u))


def hash_to_g2(msg, dst=DST_POP):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    Q0 = map_to_curve_g2(u0)
    Q1 = map_to_curve_g2(u1)
    return clear_cofactor(E2.add(Q0, Q1))
