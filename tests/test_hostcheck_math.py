"""Stage-by-stage parity of the kernel math headers (lodestar_amd/csrc/lsg_*.hpp) with the
oracle, using a host (x86) build of those same headers (tests/native/hostcheck.hip).
This runs in the CPU container; the GPU parity tests (tests/test_gpu_parity.py) repeat
the end-to-end checks through the real HIP kernels.
"""
import ctypes
import os
import random
import subprocess

import pytest

from oracle.fields import (
    P, f2_mul, f2_sqr, f2_inv, f2_sqrt, f12_mul, f12_sqr, f12_inv, f12_frob, f12_frob2, f12_coeffs,
)
from oracle.curves import (
    E1, E2, G1_GEN, G2_GEN, g1_serialize, g2_serialize, g2_compress, in_g2, BlstError, g2_uncompress,
)
from oracle import hash_to_curve as h2c
from oracle.pairing import miller_loop_fast, final_exp_fast

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "hostcheck.hip")
# host builds of the generic math over two Fp backends: "elem" (12 x 32-bit limbs, fully
# reduced, lsg_fp_elem.hpp) and "pair" (the pair backend's lazy signed 14 x 29-bit limbs,
# lsg_fp_pair.hpp with all limbs in one lane)
LIBS = {"elem": (os.path.join(HERE, "native", "libhostcheck.so"), []),
        "pair": (os.path.join(HERE, "native", "libhostcheck_pair.so"), ["-DLSG_HOSTCHECK_PAIR"])}


def _build(backend):
    lib, defs = LIBS[backend]
    hdrs = [os.path.join(ROOT, "lodestar_amd", "csrc", f) for f in os.listdir(os.path.join(ROOT, "lodestar_amd", "csrc"))]
    newest = max(os.path.getmtime(p) for p in hdrs + [SRC])
    if os.path.exists(lib) and os.path.getmtime(lib) >= newest:
        return lib
    subprocess.check_call(["hipcc", "-x", "hip", "--cuda-host-only", "-O2", "-std=c++17", "-fPIC", "-shared"] + defs +
                          ["-I", os.path.join(ROOT, "lodestar_amd", "csrc"), SRC, "-o", lib])
    return lib


@pytest.fixture(scope="module", params=["elem", "pair"])
def hc(request):
    try:
        lib = _build(request.param)
    except (OSError, subprocess.CalledProcessError) as e:  # pragma: no cover
        pytest.skip(f"hipcc unavailable: {e}")
    h = ctypes.CDLL(lib)
    h.backend = request.param
    return h


def be(v):
    return int(v).to_bytes(48, "big")


def b2(a):
    return be(a[0]) + be(a[1])


def ub2(b):
    return (int.from_bytes(b[:48], "big"), int.from_bytes(b[48:96], "big"))


def b12(f):
    return b"".join(b2(c) for c in f12_coeffs(f))


def ub12(b):
    c = [ub2(b[96 * i:96 * i + 96]) for i in range(6)]
    return ((c[0], c[1], c[2]), (c[3], c[4], c[5]))


def buf(n):
    return ctypes.create_string_buffer(n)


rng = random.Random(1234)


def rfp():
    return rng.randrange(P)


def rf2():
    return (rfp(), rfp())


def rf12():
    return tuple(tuple(rf2() for _ in range(3)) for _ in range(2))


def test_fp_mul_inv(hc):
    for _ in range(200):
        a, b = rfp(), rfp()
        o = buf(48)
        hc.hc_fp_mul(be(a), be(b), o)
        assert int.from_bytes(o.raw, "big") == a * b % P
    for a in [0, 1, P - 1] + [rfp() for _ in range(20)]:
        o = buf(48)
        hc.hc_fp_inv(be(a), o)
        assert int.from_bytes(o.raw, "big") == (pow(a, -1, P) if a else 0)


def test_fp_from_be64(hc):
    for _ in range(100):
        v = rng.getrandbits(512)
        o = buf(48)
        hc.hc_fp_from_be64(v.to_bytes(64, "big"), o)
        assert int.from_bytes(o.raw, "big") == v % P
    for v in [0, (1 << 512) - 1, P, (1 << 384) - 1]:
        o = buf(48)
        hc.hc_fp_from_be64(v.to_bytes(64, "big"), o)
        assert int.from_bytes(o.raw, "big") == v % P


def test_fp2_ops(hc):
    for _ in range(50):
        a, b = rf2(), rf2()
        o = buf(96)
        hc.hc_fp2_mul(b2(a), b2(b), o)
        assert ub2(o.raw) == f2_mul(a, b)
        hc.hc_fp2_sqr(b2(a), o)
        assert ub2(o.raw) == f2_sqr(a)
        hc.hc_fp2_inv(b2(a), o)
        assert ub2(o.raw) == f2_inv(a)


def test_fp2_sqrt(hc):
    cases = [rf2() for _ in range(60)] + [(0, 0), (4, 0), (P - 4, 0), (0, 5), (rfp(), 0), (0, rfp())]
    for a in cases:
        o = buf(96)
        ok = hc.hc_fp2_sqrt(b2(a), o)
        exp = f2_sqrt(a)
        assert bool(ok) == (exp is not None), a
        if ok:
            r = ub2(o.raw)
            assert f2_sqr(r) == (a[0] % P, a[1] % P)


def test_fp12_ops(hc):
    for _ in range(5):
        a, b = rf12(), rf12()
        o = buf(576)
        hc.hc_fp12_mul(b12(a), b12(b), o)
        assert ub12(o.raw) == f12_mul(a, b)
        hc.hc_fp12_sqr(b12(a), o)
        assert ub12(o.raw) == f12_sqr(a)
        hc.hc_fp12_inv(b12(a), o)
        assert ub12(o.raw) == f12_inv(a)
        hc.hc_fp12_frob(b12(a), o)
        assert ub12(o.raw) == f12_frob(a)
        hc.hc_fp12_frob2(b12(a), o)
        assert ub12(o.raw) == f12_frob2(a)


def test_g2_uncompress_and_subgroup(hc):
    import json
    pts = json.load(open(os.path.join(HERE, "golden", "mainnet_g2_points.json")))
    for hx in pts:
        o = buf(192)
        assert hc.hc_g2_uncompress(bytes.fromhex(hx), o) == 0
        assert o.raw == g2_serialize(g2_uncompress(bytes.fromhex(hx)))
        assert hc.hc_g2_in_group(o.raw) == 1
    # random x: decompress where on curve; not in G2 w.h.p.
    hits = 0
    for _ in range(30):
        x = rf2()
        b = bytearray(be(x[1]) + be(x[0]))
        b[0] |= 0x80
        o = buf(192)
        e = hc.hc_g2_uncompress(bytes(b), o)
        try:
            exp = g2_uncompress(bytes(b))
            assert e == 0 and o.raw == g2_serialize(exp)
            assert hc.hc_g2_in_group(o.raw) == int(in_g2(exp))
            hits += 1
        except BlstError as err:
            assert e == err.code
    assert hits > 5
    bad = json.load(open(os.path.join(HERE, "golden", "mainnet_g2_points_bad.json")))
    for item in bad:
        o = buf(192)
        assert hc.hc_g2_uncompress(bytes.fromhex(item["sig"]), o) == 2


def test_hash_to_g2(hc):
    msgs = [b"", b"abc", bytes(32), bytes(range(32)), os.urandom(32), b"lodestar" * 20]
    for m in msgs:
        o = buf(192)
        hc.hc_hash_to_g2(m, len(m), h2c.DST_POP, len(h2c.DST_POP), o)
        assert o.raw == g2_serialize(h2c.hash_to_g2(m)), m


def test_expand_and_sswu(hc):
    m = b"sswu"
    o = buf(256)
    hc.hc_expand_xmd(m, len(m), h2c.DST_POP, len(h2c.DST_POP), o)
    assert o.raw == h2c.expand_message_xmd(m, h2c.DST_POP, 256)
    for _ in range(10):
        u = rf2()
        o = buf(192)
        hc.hc_sswu(b2(u), o)
        assert o.raw == g2_serialize(h2c.map_to_curve_sswu(u))


def test_scalar_mul(hc):
    pk = E1.mul(G1_GEN, 0xABCDEF)
    Q = E2.mul(G2_GEN, 12345)
    for k in [1, 2, 3, 4, 7, 8, 0x4924924924924924, 0xDB6DB6DB6DB6DB6D, 1 << 63, (1 << 63) - 1, (1 << 64) - 1,
              rng.getrandbits(64), rng.getrandbits(64) | (1 << 63)]:  # signed 3-bit windows: carries
        hc.hc_g1_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        hc.hc_g2_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        o = buf(96)
        hc.hc_g1_mul_u64(g1_serialize(pk), k, o)
        assert o.raw == g1_serialize(E1.mul(pk, k))
        o = buf(192)
        hc.hc_g2_mul_u64(g2_serialize(Q), k, o)
        assert o.raw == g2_serialize(E2.mul(Q, k))


def test_miller_loop_and_final_exp(hc):
    pk = E1.mul(G1_GEN, 777)
    Q = E2.mul(G2_GEN, 999)
    o = buf(576)
    hc.hc_miller(g1_serialize(pk), g2_serialize(Q), o)
    f = miller_loop_fast(pk, Q)
    assert ub12(o.raw) == f
    o2 = buf(576)
    hc.hc_final_exp(o.raw, o2)
    assert ub12(o2.raw) == final_exp_fast(f)


def test_miller_loop_multi_is_product_of_single_loops(hc):
    """lsg_pairing.hpp:miller_loop_multi (blst miller_loop_n form: shared f and squarings)
    equals the product of the per-pair Miller values; dropped pairs contribute 1."""
    from oracle.fields import f12_mul, F12_ONE
    pairs = [(E1.mul(G1_GEN, 11 + k), E2.mul(G2_GEN, 23 + 7 * k)) for k in range(4)]
    pb = b"".join(g1_serialize(p) for p, _ in pairs)
    qb = b"".join(g2_serialize(q) for _, q in pairs)
    singles = [miller_loop_fast(p, q) for p, q in pairs]
    for use in ([1, 1, 1, 1], [0, 1, 1, 1], [1, 0, 1, 0], [0, 0, 0, 1], [0, 0, 0, 0]):
        o = buf(576)
        hc.hc_miller_multi4(pb, qb, (ctypes.c_int32 * 4)(*use), o)
        exp = F12_ONE
        for u, f in zip(use, singles):
            if u:
                exp = f12_mul(exp, f)
        assert ub12(o.raw) == exp, use


def test_split_miller_loop_equals_multi_loop(hc):
    """lsg_pairing.hpp:miller_lines + miller_accum_multi (the device's k_miller_lines /
    k_miller_accum split) give the same field element as the product of single Miller loops
    (oracle/pairing.py:miller_loop_fast); dropped pairs contribute 1."""
    from oracle.fields import f12_mul, F12_ONE
    pairs = [(E1.mul(G1_GEN, 5 + 3 * k), E2.mul(G2_GEN, 17 + 11 * k)) for k in range(4)]
    pb = b"".join(g1_serialize(p) for p, _ in pairs)
    qb = b"".join(g2_serialize(q) for _, q in pairs)
    singles = [miller_loop_fast(p, q) for p, q in pairs]
    for use in ([1, 1, 1, 1], [0, 1, 1, 1], [1, 0, 0, 1], [0, 0, 0, 0]):
        o = buf(576)
        hc.hc_miller_split4(pb, qb, (ctypes.c_int32 * 4)(*use), o)
        exp = F12_ONE
        for u, f in zip(use, singles):
            if u:
                exp = f12_mul(exp, f)
        assert ub12(o.raw) == exp, use


def test_paired_line_miller_schedule(hc):
    """The fused kernel's schedule (lsg_k_miller.hip k_miller_fused: lines multiplied in pairs,
    then f * (l0 l1) * (l2 l3) with the kernel's product formulas), restated on the host,
    gives the product of single Miller loops (oracle/pairing.py:miller_loop_fast); dropped
    pairs contribute 1."""
    from oracle.fields import f12_mul, F12_ONE
    pairs = [(E1.mul(G1_GEN, 7 + 5 * k), E2.mul(G2_GEN, 13 + 9 * k)) for k in range(4)]
    pb = b"".join(g1_serialize(p) for p, _ in pairs)
    qb = b"".join(g2_serialize(q) for _, q in pairs)
    singles = [miller_loop_fast(p, q) for p, q in pairs]
    for use in ([1, 1, 1, 1], [0, 1, 1, 1], [1, 0, 0, 1], [1, 1, 0, 0], [0, 0, 0, 0]):
        o = buf(576)
        hc.hc_miller_paired4(pb, qb, (ctypes.c_int32 * 4)(*use), o)
        exp = F12_ONE
        for u, f in zip(use, singles):
            if u:
                exp = f12_mul(exp, f)
        assert ub12(o.raw) == exp, use


def test_g1_subgroup_check(hc):
    """lsg_curve.hpp:g1_in_group ([r]P == O, KeyValidate) against oracle/curves.py:in_g1 on
    subgroup points, the identity and on-curve points outside the subgroup."""
    from oracle.curves import in_g1
    from tests.blsdata import g1_not_in_group
    pts = [E1.mul(G1_GEN, k) for k in (1, 2, 12345)] + [g1_not_in_group(s) for s in range(3)]
    for pt in pts:
        assert hc.hc_g1_in_group(g1_serialize(pt)) == (1 if in_g1(pt) else 0)
    assert hc.hc_g1_in_group(g1_serialize(None)) == 1


def _g2_proj_blob(Q, z):
    """homogeneous projective blob (X, Y, Z) = (x z, y z, z) of an affine point; None -> (0, 1, 0)"""
    if Q is None:
        return b2((0, 0)) + b2((1, 0)) + b2((0, 0))
    x, y = Q
    return b2(f2_mul(x, z)) + b2(f2_mul(y, z)) + b2(z)


@pytest.mark.parametrize("waves", [1, 2])
def test_slp_programs_match_oracle(hc, waves):
    """The straight-line programs of the serial stages (tools/gen_slp.py), run op by op with
    the gfx950 interpreter's own operation code (lsg_slp_exec.hpp) in the host build of the
    pair backend, scheduled for one and two waves per item: final exponentiation, ML(-G1, S) and Horner + ML(-G1, S) against the
    oracle (oracle/pairing.py final_exp_fast, miller_loop_fast)."""
    if hc.backend != "pair":
        pytest.skip("programs run on the pair backend")
    from oracle.fields import f12_mul, F12_ONE
    neg_g1 = E1.neg(G1_GEN) if hasattr(E1, "neg") else (G1_GEN[0], (-G1_GEN[1]) % P)
    o = buf(48 * 14)
    # final exponentiation: a random element and a pairing product that is 1 after it
    pk = E1.mul(G1_GEN, 4242)
    Q = E2.mul(G2_GEN, 31337)
    prod = f12_mul(miller_loop_fast(pk, Q), miller_loop_fast(neg_g1, E2.mul(Q, 4242)))
    for f in (rf12(), prod):
        assert hc.hc_slp_run(0 + waves - 1, b12(f), o) == 12
        assert ub12(o.raw[:576]) == final_exp_fast(f)
    assert final_exp_fast(prod) == F12_ONE
    # ML(-G1, S) of a projective S, and S.Z
    for k in (1, 77, 123456789):
        S = E2.mul(G2_GEN, k)
        z = rf2()
        assert hc.hc_slp_run(2 + waves - 1, _g2_proj_blob(S, z), o) == 14
        assert ub12(o.raw[:576]) == miller_loop_fast(neg_g1, S)
        assert ub2(o.raw[576:672]) == z
    # Horner over 64 per-bit sums (some at infinity), then ML(-G1, S)
    Cs = [None if k % 5 == 3 else E2.mul(G2_GEN, 1000 + 17 * k) for k in range(64)]
    blob = b"".join(_g2_proj_blob(C, rf2()) for C in Cs)
    S = None
    for k in range(63, -1, -1):
        S = E2.add(E2.add(S, S), Cs[k])
    assert hc.hc_slp_run(4 + waves - 1, blob, o) == 14
    assert ub12(o.raw[:576]) == miller_loop_fast(neg_g1, S)
    # one-set Miller item (Montgomery lane-form in/out): a pair that takes part, and one that
    # does not (P = (0, 0), use 0) contributing exactly 1
    pk, Q = E1.mul(G1_GEN, 99), E2.mul(G2_GEN, 1234)
    (qx, qy) = Q
    assert hc.hc_slp_run(6 + waves - 1, be(pk[0]) + be(pk[1]) + b2(qx) + b2(qy) + be(1), o) == 12
    assert ub12(o.raw[:576]) == miller_loop_fast(pk, Q)
    assert hc.hc_slp_run(6 + waves - 1, be(0) + be(0) + b2(qx) + b2(qy) + be(0), o) == 12
    assert ub12(o.raw[:576]) == F12_ONE
    # cofactor clearing + affine of an SSWU-map sum (a point of E2 outside G2), projective in
    for k in range(2):
        u = (rng.randrange(P), rng.randrange(P))
        Qm = h2c.iso_map(h2c.map_to_curve_sswu(u))
        z = rf2()
        assert hc.hc_slp_run(8 + waves - 1, _g2_proj_blob(Qm, z), o) == 6
        Hc = h2c.clear_cofactor(Qm)
        assert (ub2(o.raw[:96]), ub2(o.raw[96:192])) == Hc
        assert ub2(o.raw[192:288]) != (0, 0)
    # G2 membership: a subgroup point passes, an E2 point outside G2 (the map's raw output)
    # and a small-order point fail
    Sg = E2.mul(G2_GEN, 4321)
    R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5
    small = None  # a point of small prime order l | h2 (the complete formulas meet O on the way)
    for t in range(20):
        Qt = h2c.iso_map(h2c.map_to_curve_sswu((7 + t, 11 * t)))
        for l in (13, 23, 2713):
            cand = E2.mul(Qt, R_ORDER * (H2 // l))
            if cand is not None:
                small, order = cand, l
                break
        if small is not None:
            break
    assert small is not None and E2.mul(small, order) is None
    for pt, member in ((Sg, True), (Qm, False), (small, False)):
        assert hc.hc_slp_run(10 + waves - 1, b2(pt[0]) + b2(pt[1]), o) == 4
        zero = all(ub2(o.raw[96 * i:96 * i + 96]) == (0, 0) for i in range(2))
        assert zero == member
    # [r] P for a 64-bit r, bits least significant first (0 / 1 in Montgomery form)
    for r in (1, 2, 3, 0xDEADBEEFCAFEF00D, (1 << 64) - 1):
        bits = b"".join(be((r >> k) & 1) for k in range(64))
        assert hc.hc_slp_run(12 + waves - 1, b2(Sg[0]) + b2(Sg[1]) + bits, o) == 6
        X, Y, Z = ub2(o.raw[:96]), ub2(o.raw[96:192]), ub2(o.raw[192:288])
        zi = f2_inv(Z)
        assert (f2_mul(X, zi), f2_mul(Y, zi)) == E2.mul(Sg, r)


def test_inv_gcd_matches_pow(hc):
    """lsg_inv.hpp (divstep GCD inversion of the programs' INV operation) against pow(x, -1, p),
    including 0 (-> 0), 1, p - 1 and values near 2^k"""
    if hc.backend != "pair":
        pytest.skip("pair backend only")
    vals = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, 1 << 380, (1 << 200) + 1] + [rng.randrange(P) for _ in range(300)]
    o = buf(48)
    for x in vals:
        hc.hc_inv_gcd(be(x), o)
        assert int.from_bytes(o.raw, "big") == (pow(x, -1, P) if x else 0), x


def _limbs_value(limbs):
    return sum(int(v) << (29 * k) for k, v in enumerate(limbs))


def test_fp2_sop_bound_limits(hc):
    """The Fp2 product as two sums of products (lsg_fp_pair.hpp pair_fp2_mul_sop) at the lazy
    bounds of its inputs: limbs at the edges of [-8, 2^29 + 8), signed top limbs with
    |v| < 2^12.6 p, against the exact integers: out = (a0 b0 - a1 b1, a0 b1 + a1 b0) / R mod p,
    |out| < 3p, limbs 0..12 normalised.  (Host build: one lane holds every column for 14 steps
    and carries at mid-loop; on gfx950 a column lives 7 steps per lane)"""
    if hc.backend != "pair":
        pytest.skip("pair backend only")
    import itertools
    R = 1 << 406
    Rinv = pow(R, -1, P)
    top_max = (int(2 ** 12.6 * P) >> (29 * 13))  # the largest top limb of a value < 2^12.6 p
    lo_hi, lo_lo = (1 << 29) + 7, -8
    bound = int(2 ** 12.6 * P)

    def clamp(limbs):  # the top limb's magnitude lowered until |value| < 2^12.6 p
        while abs(_limbs_value(limbs)) >= bound:
            limbs[13] += -1 if limbs[13] > 0 else 1
        return limbs
    patterns = []
    for lo, top in itertools.product((lo_hi, lo_lo, 0, (1 << 29) - 1), (top_max, -top_max, 0, 1)):
        patterns.append(clamp([lo] * 13 + [top]))
    r = random.Random(77)
    for _ in range(40):  # random limbs anywhere in the lazy range
        patterns.append(clamp([r.randrange(-8, (1 << 29) + 8) for _ in range(13)] + [r.randrange(-top_max, top_max + 1)]))
    I32 = ctypes.c_int32 * 28
    for k in range(len(patterns) * 2):
        a0, a1 = patterns[k % len(patterns)], patterns[(3 * k + 1) % len(patterns)]
        b0, b1 = patterns[(5 * k + 2) % len(patterns)], patterns[(7 * k + 3) % len(patterns)]
        va0, va1, vb0, vb1 = map(_limbs_value, (a0, a1, b0, b1))
        assert max(abs(v) for v in (va0, va1, vb0, vb1)) < 2 ** 12.6 * P
        out = I32()
        hc.hc_pair_fp2_mul_raw(I32(*(a0 + a1)), I32(*(b0 + b1)), out)
        c0, c1 = list(out[:14]), list(out[14:])
        v0, v1 = _limbs_value(c0), _limbs_value(c1)
        assert (v0 - (va0 * vb0 - va1 * vb1) * Rinv) % P == 0
        assert (v1 - (va0 * vb1 + va1 * vb0) * Rinv) % P == 0
        assert abs(v0) < 3 * P and abs(v1) < 3 * P
        assert all(0 <= c < (1 << 29) for c in c0[:13] + c1[:13])
