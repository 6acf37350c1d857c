"""Test-data helpers built on the oracle (keys, messages, signatures, corruptions).

Keys follow the interop derivation (packages/state-transition/src/util/interop.ts:19-22);
messages are sha256(b"lodestar-mi355x" || tag || i) as SURVEY.md 8(d) prescribes.
"""
import functools
import hashlib

from oracle.curves import E1, E2, G1_GEN, g1_serialize, g1_compress, g2_compress, g2_serialize
from oracle.fields import P, R
from oracle.interop import interop_secret_key
from oracle.verifier import sign


@functools.lru_cache(maxsize=None)
def sk(i):
    return interop_secret_key(i)


@functools.lru_cache(maxsize=None)
def pk_point(i):
    return E1.mul(G1_GEN, sk(i))


def pk_bytes(i, compressed=False):
    return g1_compress(pk_point(i)) if compressed else g1_serialize(pk_point(i))


def msg(tag, i):
    return hashlib.sha256(b"lodestar-mi355x" + tag.encode() + i.to_bytes(8, "little")).digest()


@functools.lru_cache(maxsize=None)
def sig_point(key_idx_tuple, m):
    s = sum(sk(k) for k in key_idx_tuple) % R
    return sign(s, m)


def single_set(i, tag="t", key=None):
    k = i if key is None else key
    m = msg(tag, i)
    return ([pk_bytes(k)], m, g2_compress(sig_point((k,), m)))


def aggregate_set(i, keys, tag="agg"):
    m = msg(tag, i)
    return ([pk_bytes(k) for k in keys], m, g2_compress(sig_point(tuple(keys), m)))


# --- adversarial corruptions
def corrupt_wrong_message(s):
    pks, m, sig = s
    return (pks, hashlib.sha256(m).digest(), sig)


def corrupt_flip_x_bit(s, bit=7):
    pks, m, sig = s
    b = bytearray(sig)
    b[40] ^= 1 << (bit % 8)
    return (pks, m, bytes(b))


def corrupt_truncate(s):
    pks, m, sig = s
    return (pks, m, sig[:32])


def corrupt_not_in_group(s, seed=0):
    """Replace the signature by a point on E2 that is not in G2."""
    from oracle.curves import g2_uncompress, in_g2, BlstError
    pks, m, sig = s
    x0 = int.from_bytes(hashlib.sha256(b"nig" + m + bytes([seed])).digest(), "big") % P
    x1 = 0
    while True:
        b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
        b[0] |= 0x80
        try:
            pt = g2_uncompress(bytes(b))
            if pt is not None and not in_g2(pt):
                return (pks, m, bytes(b))
        except BlstError:
            pass
        x1 += 1


def corrupt_infinity(s):
    pks, m, sig = s
    return (pks, m, bytes([0xC0]) + bytes(95))


CORRUPTIONS = [corrupt_wrong_message, corrupt_flip_x_bit, corrupt_truncate, corrupt_not_in_group, corrupt_infinity]


def g1_not_in_group(seed=0):
    """An E1 point outside the r-torsion subgroup (affine, on the curve): KeyValidate must
    reject it with BLST_POINT_NOT_IN_GROUP (processDeposit.ts:57-65)."""
    from oracle.curves import in_g1
    from oracle.fields import fp_sqrt
    x = 5 + 7 * seed
    while True:
        y = fp_sqrt((x * x * x + 4) % P)
        if y is not None and not in_g1((x, y)):
            return (x, y)
        x += 1
