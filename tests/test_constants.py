"""The kernels' Montgomery constants (lodestar_amd/csrc/lsg_constants.hpp, 12 x 32-bit limbs,
R = 2^384; lsg_constants_r29.hpp, 14 x 29-bit limbs, R = 2^406) against the oracle, CPU only.

tools/gen_constants.py writes both headers without importing oracle/ (it is product build
tooling); here every emitted value is decoded back to an integer and checked against the
oracle's own definition of the same quantity (oracle/fields.py, curves.py, hash_to_curve.py,
whose 3-isogeny coefficients and psi constants are pinned by the genesis KAT,
tests/test_oracle_kat.py).  The committed headers must also be what the generator writes now.
"""
import os
import re
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.curves import G1_GEN, PSI_CX, PSI_CY, psi, E2, G2_GEN  # noqa: E402
from oracle.fields import GAMMA1, GAMMA2, P, X_ABS, f2_inv, f2_mul, f2_neg  # noqa: E402
from oracle.hash_to_curve import SSWU_A, SSWU_B, SSWU_Z, XDEN, XNUM, YDEN, YNUM  # noqa: E402

CSRC = os.path.join(ROOT, "lodestar_amd", "csrc")
LAYOUTS = {"lsg_constants.hpp": (32, 12), "lsg_constants_r29.hpp": (29, 14)}

DECL = re.compile(r"LSG_CONST (fpc_t|fp2c_t|uint32_t) (\w+)(?:\[\d+\])? = (\{.*?\});", re.S)


def parse(path):
    """name -> list of u32 words (fp2c_t: both halves in order); also the scalar words of
    the `uint32_t A = x, B = y;` declaration of LSG_X_ABS_*"""
    text = open(path).read()
    out = {}
    for _, name, body in DECL.findall(text):
        out[name] = [int(w, 16) for w in re.findall(r"0x([0-9a-f]+)u", body)]
    for name, v in re.findall(r"(LSG_X_ABS_(?:LO|HI)) = 0x([0-9a-f]+)u", text):
        out[name] = [int(v, 16)]
    for name, v in re.findall(r"LSG_CONST uint32_t (LSG_N0P) = 0x([0-9a-f]+)u;", text):
        out[name] = [int(v, 16)]
    return out


def to_int(words, bits):
    return sum(w << (bits * i) for i, w in enumerate(words))


@pytest.fixture(scope="module", params=sorted(LAYOUTS))
def layout(request):
    bits, nl = LAYOUTS[request.param]
    consts = parse(os.path.join(CSRC, request.param))
    rm = 1 << (bits * nl)
    rinv = pow(rm, -1, P)

    def fp(name, mont=True):
        w = consts[name]
        assert len(w) == nl, name
        assert all(x < (1 << bits) for x in w), f"{name}: a limb wider than {bits} bits"
        v = to_int(w, bits)
        assert v < P, name
        return v * rinv % P if mont else v

    def fp2(name):
        w = consts[name]
        assert len(w) == 2 * nl, name
        lo, hi = to_int(w[:nl], bits), to_int(w[nl:], bits)
        assert lo < P and hi < P, name
        return (lo * rinv % P, hi * rinv % P)

    return {"bits": bits, "nl": nl, "rm": rm, "c": consts, "fp": fp, "fp2": fp2}


def test_generator_reproduces_committed_headers():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "lsg_constants.hpp")
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_constants.py"), out], check=True, timeout=120)
        for name in LAYOUTS:
            assert open(os.path.join(d, name)).read() == open(os.path.join(CSRC, name)).read(), name


def test_modulus_and_reduction_constants(layout):
    L = layout
    bits = L["bits"]
    assert to_int(L["c"]["LSG_P"], bits) == P
    n0p = L["c"]["LSG_N0P"][0]
    assert (P * n0p + 1) % (1 << bits) == 0  # -p^-1 mod 2^bits
    assert L["fp"]("FP_ONE") == 1
    assert L["fp"]("FP_R2") == L["rm"] % P  # mont(R) = R^2 mod p
    assert L["fp"]("FP_RCUBE") == L["rm"] * L["rm"] % P
    assert L["fp"]("FP_R3") == (1 << 384) * L["rm"] % P
    assert L["fp"]("FP_R2_SHL256") == (1 << 256) * L["rm"] % P
    assert L["fp"]("FP_ONE_CANON", mont=False) == 1
    assert L["fp"]("FP_HALF") * 2 % P == 1
    assert L["fp"]("LSG_HALF_P_CANON", mont=False) == (P - 1) // 2
    if bits != 32:  # conversions between this layout and the 12 x 32-bit one
        assert L["fp"]("FP_FROM_R384", mont=False) == (1 << (2 * bits * L["nl"] - 384)) % P
        assert L["fp"]("FP_TO_R384", mont=False) == (1 << 384) % P


def test_exponents_and_curve_parameter(layout):
    c = layout["c"]
    assert to_int(c["LSG_EXP_P_MINUS_2"], 32) == P - 2
    assert to_int(c["LSG_EXP_P_PLUS_1_DIV_4"], 32) == (P + 1) // 4
    assert to_int(c["LSG_EXP_P_MINUS_3_DIV_4"], 32) == (P - 3) // 4
    assert c["LSG_X_ABS_LO"][0] | (c["LSG_X_ABS_HI"][0] << 32) == X_ABS


def test_curve_constants(layout):
    fp, fp2 = layout["fp"], layout["fp2"]
    assert fp("FP_B_G1") == 4 and fp("FP_B3_G1") == 12
    assert fp2("FP2_B_G2") == (4, 4)
    assert (fp("G1_GEN_X"), fp("G1_GEN_Y")) == G1_GEN
    assert fp("G1_GEN_NEG_Y") == (-G1_GEN[1]) % P


def test_frobenius_and_psi_constants(layout):
    fp, fp2 = layout["fp"], layout["fp2"]
    for i in range(6):
        assert fp2(f"FROB1_G{i}") == GAMMA1[i], i
        assert fp2(f"FROB2_G{i}") == GAMMA2[i], i
    assert fp2("PSI_CX") == PSI_CX and fp2("PSI_CY") == PSI_CY
    # psi^2(x, y) = (x * PSI2_CX, y * PSI2_CY), both in Fp: checked on the G2 generator
    q2 = psi(psi(G2_GEN))
    assert q2 == (f2_mul(G2_GEN[0], (fp("PSI2_CX"), 0)), f2_mul(G2_GEN[1], (fp("PSI2_CY"), 0)))
    assert E2.on_curve(q2)


def test_hash_to_curve_constants(layout):
    fp, fp2 = layout["fp"], layout["fp2"]
    assert fp2("SSWU_A") == SSWU_A and fp2("SSWU_B") == SSWU_B and fp2("SSWU_Z") == SSWU_Z
    assert fp2("SSWU_MINUS_B_OVER_A") == f2_mul(f2_neg(SSWU_B), f2_inv(SSWU_A))
    assert fp2("SSWU_B_OVER_ZA") == f2_mul(SSWU_B, f2_inv(f2_mul(SSWU_Z, SSWU_A)))
    nz = (SSWU_Z[0] ** 2 + SSWU_Z[1] ** 2) % P
    assert fp("SSWU_NZ_POW_P1D4") == pow(nz, (P + 1) // 4, P)
    for name, poly in (("ISO_XNUM", XNUM), ("ISO_XDEN", XDEN), ("ISO_YNUM", YNUM), ("ISO_YDEN", YDEN)):
        for k, coef in enumerate(poly):
            assert fp2(f"{name}_{k}") == coef, (name, k)
        assert f"{name}_{len(poly)}" not in layout["c"]


def test_every_declared_constant_is_checked(layout):
    checked = {"LSG_P", "LSG_N0P", "FP_ONE", "FP_R2", "FP_RCUBE", "FP_R3", "FP_R2_SHL256", "FP_ONE_CANON", "FP_HALF",
               "LSG_HALF_P_CANON", "FP_FROM_R384", "FP_TO_R384", "LSG_EXP_P_MINUS_2", "LSG_EXP_P_PLUS_1_DIV_4",
               "LSG_EXP_P_MINUS_3_DIV_4", "LSG_X_ABS_LO", "LSG_X_ABS_HI", "FP_B_G1", "FP_B3_G1", "FP2_B_G2", "G1_GEN_X",
               "G1_GEN_Y", "G1_GEN_NEG_Y", "PSI_CX", "PSI_CY", "PSI2_CX", "PSI2_CY", "SSWU_A", "SSWU_B", "SSWU_Z",
               "SSWU_MINUS_B_OVER_A", "SSWU_B_OVER_ZA", "SSWU_NZ_POW_P1D4"}
    checked |= {f"FROB{k}_G{i}" for k in (1, 2) for i in range(6)}
    checked |= {f"ISO_{n}_{k}" for n, m in (("XNUM", 4), ("XDEN", 3), ("YNUM", 4), ("YDEN", 4)) for k in range(m)}
    assert set(layout["c"]) <= checked, set(layout["c"]) - checked
