"""ORACLE (test infrastructure only) -- BLS12-381 G1/G2 group law, ZCash serialization,
subgroup checks, psi endomorphism.  Pure Python; affine coordinates, ``None`` = infinity.

Restates what @chainsafe/blst@0.2.8 / blst does for PublicKey/Signature (de)serialization
(called from packages/beacon-node/src/chain/bls/multithread/worker.ts:110 and
packages/beacon-node/src/chain/bls/maybeBatch.ts:23,36) and pubkey aggregation
(packages/beacon-node/src/chain/bls/utils.ts:11).  Only tests/, smoke() and bench.py's
cpu_baseline leg may import this module.
"""
from .fields import (
    P, R, X, X_ABS, fp_inv, fp_sqrt, F2_ZERO, F2_ONE, XI,
    f2_add, f2_sub, f2_neg, f2_mul, f2_sqr, f2_inv, f2_is_zero, f2_eq, f2_conj, f2_pow,
    f2_sqrt, f2_lexi_largest, f2_mul_fp,
)

# ------------------------------------------------------------------ field adapters
class _Fp:
    zero = 0
    one = 1
    add = staticmethod(lambda a, b: (a + b) % P)
    sub = staticmethod(lambda a, b: (a - b) % P)
    neg = staticmethod(lambda a: (-a) % P)
    mul = staticmethod(lambda a, b: a * b % P)
    sqr = staticmethod(lambda a: a * a % P)
    inv = staticmethod(fp_inv)
    is_zero = staticmethod(lambda a: a % P == 0)
    eq = staticmethod(lambda a, b: (a - b) % P == 0)
    small = staticmethod(lambda k: k % P)


class _Fp2:
    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    neg = staticmethod(f2_neg)
    mul = staticmethod(f2_mul)
    sqr = staticmethod(f2_sqr)
    inv = staticmethod(f2_inv)
    is_zero = staticmethod(f2_is_zero)
    eq = staticmethod(f2_eq)
    small = staticmethod(lambda k: (k % P, 0))


B1 = 4
B2 = (4, 4)  # 4 * (1 + u)

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)


class Curve:
    def __init__(self, F, b):
        self.F = F
        self.b = b

    def on_curve(self, Pt):
        if Pt is None:
            return True
        F = self.F
        x, y = Pt
        return F.eq(F.sqr(y), F.add(F.mul(F.sqr(x), x), self.b))

    def neg(self, Pt):
        if Pt is None:
            return None
        return (Pt[0], self.F.neg(Pt[1]))

    def add(self, A, B):
        F = self.F
        if A is None:
            return B
        if B is None:
            return A
        x1, y1 = A
        x2, y2 = B
        if F.eq(x1, x2):
            if F.eq(y1, y2) and not F.is_zero(y1):
                return self.dbl(A)
            return None
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
        x3 = F.sub(F.sub(F.sqr(lam), x1), x2)
        y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
        return (x3, y3)

    def dbl(self, A):
        F = self.F
        if A is None:
            return None
        x1, y1 = A
        if F.is_zero(y1):
            return None
        lam = F.mul(F.mul(F.small(3), F.sqr(x1)), F.inv(F.add(y1, y1)))
        x3 = F.sub(F.sqr(lam), F.add(x1, x1))
        y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
        return (x3, y3)

    def mul(self, A, k):
        if k < 0:
            A = self.neg(A)
            k = -k
        res = None
        base = A
        while k > 0:
            if k & 1:
                res = self.add(res, base)
            base = self.dbl(base)
            k >>= 1
        return res

    def eq(self, A, B):
        if A is None or B is None:
            return A is None and B is None
        return self.F.eq(A[0], B[0]) and self.F.eq(A[1], B[1])


E1 = Curve(_Fp, B1)
E2 = Curve(_Fp2, B2)

# ------------------------------------------------------------------ psi endomorphism on E2
# psi = untwist o Frobenius o twist:  psi(x, y) = (conj(x) * PSI_CX, conj(y) * PSI_CY)
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def psi(Pt):
    if Pt is None:
        return None
    return (f2_mul(f2_conj(Pt[0]), PSI_CX), f2_mul(f2_conj(Pt[1]), PSI_CY))


# ------------------------------------------------------------------ subgroup checks
def in_g1(Pt):
    return E1.on_curve(Pt) and E1.mul(Pt, R) is None


def in_g2(Pt):
    """Definitional check [r]P == O (slow, used as the checker of the GPU's psi test)."""
    return E2.on_curve(Pt) and E2.mul(Pt, R) is None


def in_g2_psi(Pt):
    """Scott's test psi(P) == [x]P (the form the GPU uses); equivalent to in_g2 on E2."""
    if Pt is None:
        return True
    return E2.eq(psi(Pt), E2.mul(Pt, X))


# ------------------------------------------------------------------ BLST error codes
# Enum values of blst's BLST_ERROR (C) plus the @chainsafe/blst wrapper's size error.
BLST_SUCCESS = 0
BLST_BAD_ENCODING = 1
BLST_POINT_NOT_ON_CURVE = 2
BLST_POINT_NOT_IN_GROUP = 3
BLST_AGGR_TYPE_MISMATCH = 4
BLST_VERIFY_FAIL = 5
BLST_PK_IS_INFINITY = 6
BLST_BAD_SCALAR = 7
BLST_INVALID_SIZE = 10
BLST_NAMES = {
    0: "BLST_SUCCESS", 1: "BLST_BAD_ENCODING", 2: "BLST_POINT_NOT_ON_CURVE",
    3: "BLST_POINT_NOT_IN_GROUP", 4: "BLST_AGGR_TYPE_MISMATCH", 5: "BLST_VERIFY_FAIL",
    6: "BLST_PK_IS_INFINITY", 7: "BLST_BAD_SCALAR", 10: "BLST_INVALID_SIZE",
}


class BlstError(Exception):
    def __init__(self, code):
        self.code = code
        super().__init__("BLST_ERROR: " + BLST_NAMES[code])


# ------------------------------------------------------------------ serialization (ZCash)
def _fp_to_be(a):
    return int(a).to_bytes(48, "big")


def g1_compress(Pt):
    if Pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = Pt
    out = bytearray(_fp_to_be(x))
    out[0] |= 0x80
    if y > (P - 1) // 2:
        out[0] |= 0x20
    return bytes(out)


def g1_serialize(Pt):
    """Uncompressed 96 bytes."""
    if Pt is None:
        return bytes([0x40]) + bytes(95)
    return _fp_to_be(Pt[0]) + _fp_to_be(Pt[1])


def g2_compress(Pt):
    if Pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = Pt
    out = bytearray(_fp_to_be(x[1]) + _fp_to_be(x[0]))
    out[0] |= 0x80
    if f2_lexi_largest(y):
        out[0] |= 0x20
    return bytes(out)


def g2_serialize(Pt):
    if Pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = Pt
    return _fp_to_be(x[1]) + _fp_to_be(x[0]) + _fp_to_be(y[1]) + _fp_to_be(y[0])


def _be_fp(b):
    """Parse 48 big-endian bytes with the top 3 bits cleared; return int or raise BAD_ENCODING if >= p."""
    v = int.from_bytes(b, "big") & ((1 << 381) - 1)
    if v >= P:
        raise BlstError(BLST_BAD_ENCODING)
    return v


def g1_uncompress(b):
    """blst POINTonE1_Uncompress_Z semantics."""
    in0 = b[0]
    if not in0 & 0x80:
        raise BlstError(BLST_BAD_ENCODING)
    if in0 & 0x40:
        if (in0 & 0x3F) == 0 and not any(b[1:48]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x = _be_fp(b[:48])
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if (y > (P - 1) // 2) != bool(in0 & 0x20):
        y = (-y) % P
    if x == 0:
        raise BlstError(BLST_POINT_NOT_IN_GROUP)  # blst: "(0,+-2) is not in group"
    return (x, y)


def g1_deserialize(b):
    """blst_p1_deserialize (96 bytes uncompressed or 48 compressed)."""
    in0 = b[0]
    if len(b) == 48 or (in0 & 0x80):
        if len(b) != 48:
            raise BlstError(BLST_BAD_ENCODING)
        return g1_uncompress(b)
    if len(b) != 96:
        raise BlstError(BLST_BAD_ENCODING)
    if in0 & 0x40:
        if (in0 & 0x3F) == 0 and not any(b[1:96]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    if in0 & 0x20:
        raise BlstError(BLST_BAD_ENCODING)
    x = _be_fp(b[:48])
    y = _be_fp(b[48:96])
    Pt = (x, y)
    if not E1.on_curve(Pt):
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if x == 0:
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return Pt


def g2_uncompress(b):
    """blst POINTonE2_Uncompress_Z semantics."""
    in0 = b[0]
    if not in0 & 0x80:
        raise BlstError(BLST_BAD_ENCODING)
    if in0 & 0x40:
        if (in0 & 0x3F) == 0 and not any(b[1:96]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x1 = _be_fp(b[:48])
    x0 = _be_fp(b[48:96])
    x = (x0, x1)
    rhs = f2_add(f2_mul(f2_sqr(x), x), B2)
    y = f2_sqrt(rhs)
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if f2_lexi_largest(y) != bool(in0 & 0x20):
        y = f2_neg(y)
    if f2_is_zero(x):
        # blst: "(0, +-2) is not in group"
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return (x, y)


def g2_deserialize(b):
    in0 = b[0]
    if in0 & 0x80:
        if len(b) != 96:
            raise BlstError(BLST_BAD_ENCODING)
        return g2_uncompress(b)
    if len(b) != 192:
        raise BlstError(BLST_BAD_ENCODING)
    if in0 & 0x40:
        if (in0 & 0x3F) == 0 and not any(b[1:192]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    if in0 & 0x20:
        raise BlstError(BLST_BAD_ENCODING)
    x = (_be_fp(b[48:96]), _be_fp(b[0:48]))
    y = (_be_fp(b[144:192]), _be_fp(b[96:144]))
    Pt = (x, y)
    if not E2.on_curve(Pt):
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if f2_is_zero(x):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return Pt
