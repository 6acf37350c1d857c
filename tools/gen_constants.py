#!/usr/bin/env python3
"""Build tool: emits the Montgomery-form constants of the gfx950 kernels for the two limb
layouts:
  lodestar_amd/csrc/lsg_constants.hpp      12 x 32-bit little-endian limbs, R = 2^384
                                           (quad and row backends, host element backend)
  lodestar_amd/csrc/lsg_constants_r29.hpp  14 x 29-bit little-endian limbs, R = 2^406
                                           (radix-2^29 thread-per-set backend)

Standalone on purpose -- it does not import oracle/ (the checker); tests/test_constants.py
cross-checks every emitted value against the oracle.  The 3-isogeny coefficients are the
RFC 9380 section 8.8.2 / appendix E.3 values (the same ones oracle/iso3_derive.py derives
by Velu's formulas and the genesis KAT selects).
"""
import os
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000
# limb layout (set by main): bits per limb, limbs, Montgomery radix R = 2^(bits*limbs)
BITS, NL = 32, 12
RM = 1 << 384
N0P = (-pow(P, -1, 1 << 32)) % (1 << 32)


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(r, a)
        a = f2mul(a, a)
        e >>= 1
    return r


def f2inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
    return (a[0] * n % P, -a[1] * n % P)


def limbs(v, n=12, bits=32):
    return [(v >> (bits * i)) & ((1 << bits) - 1) for i in range(n)]


def mont(v):
    return v * RM % P


def arr(v, n=12):
    """a 32-bit-word array (exponents: bit-scanned by fp_pow_fixed in every layout)"""
    return "{" + ", ".join("0x%08xu" % x for x in limbs(v, n)) + "}"


def arrl(v):
    """a field element in the current limb layout"""
    return "{" + ", ".join("0x%08xu" % x for x in limbs(v, NL, BITS)) + "}"


XI = (1, 1)
GAMMA1 = [f2pow(XI, i * (P - 1) // 6) for i in range(6)]
GAMMA2 = [f2pow(XI, i * (P * P - 1) // 6) for i in range(6)]
PSI_CX = f2inv(f2pow(XI, (P - 1) // 3))
PSI_CY = f2inv(f2pow(XI, (P - 1) // 2))
# psi^2(x, y) = (x * c2x, y * c2y) with c2 = c * conj(c) in Fp
PSI2_CX = f2mul(PSI_CX, (PSI_CX[0], -PSI_CX[1] % P))
PSI2_CY = f2mul(PSI_CY, (PSI_CY[0], -PSI_CY[1] % P))
assert PSI2_CX[1] == 0 and PSI2_CY[1] == 0

SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = (-2 % P, -1 % P)
MINUS_B_OVER_A = f2mul((-SSWU_B[0] % P, -SSWU_B[1] % P), f2inv(SSWU_A))
B_OVER_ZA = f2mul(SSWU_B, f2inv(f2mul(SSWU_Z, SSWU_A)))

H = lambda s: int(s, 16)
ISO_XNUM = [
    (H("05c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     H("05c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, H("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (H("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     H("08ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (H("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO_XDEN = [
    (0, H("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63")),
    (0xC, H("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f")),
    (1, 0),
]
ISO_YNUM = [
    (H("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     H("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, H("05c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (H("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     H("08ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (H("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO_YDEN = [
    (H("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb"),
     H("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb")),
    (0, H("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3")),
    (0x12, H("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99")),
    (1, 0),
]

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1


def fp_decl(name, v):
    return f"LSG_CONST fpc_t {name} = {{{arrl(mont(v))}}};\n"


def fp2_decl(name, v):
    return f"LSG_CONST fp2c_t {name} = {{{{{arrl(mont(v[0]))}}}, {{{arrl(mont(v[1]))}}}}};\n"


def main(out, bits=32):
    global BITS, NL, RM, N0P
    BITS, NL = bits, (12 if bits == 32 else 14)
    RM = 1 << (BITS * NL)
    N0P = (-pow(P, -1, 1 << BITS)) % (1 << BITS)
    s = []
    s.append("// GENERATED by tools/gen_constants.py -- do not edit.\n")
    s.append(f"// Montgomery form (R = 2^{BITS * NL}), {NL} x {BITS}-bit little-endian limbs"
             f"{'' if BITS == 32 else ' (one u32 word each)'}.\n#pragma once\n")
    if BITS != 32:
        s.append(f"#define LSG_NLIMBS {NL}\n")
    s.append("#include \"lsg_types.hpp\"\n\n")
    s.append(f"LSG_CONST uint32_t LSG_P[{NL}] = {arrl(P)};\n")
    s.append(f"LSG_CONST uint32_t LSG_N0P = 0x{N0P:08x}u;\n")
    s.append(f"LSG_CONST uint32_t LSG_EXP_P_MINUS_2[12] = {arr(P - 2)};\n")
    s.append(f"LSG_CONST uint32_t LSG_EXP_P_PLUS_1_DIV_4[12] = {arr((P + 1) // 4)};\n")
    s.append(f"LSG_CONST uint32_t LSG_EXP_P_MINUS_3_DIV_4[12] = {arr((P - 3) // 4)};\n")
    s.append(f"LSG_CONST uint32_t LSG_HALF_P_CANON[{NL}] = {arrl((P - 1) // 2)};  // (p-1)/2, canonical\n")
    s.append(f"LSG_CONST uint32_t LSG_X_ABS_LO = 0x{X_ABS & 0xFFFFFFFF:08x}u, LSG_X_ABS_HI = 0x{X_ABS >> 32:08x}u;\n\n")
    s.append(fp_decl("FP_ONE", 1))
    s.append(fp_decl("FP_R2", RM % P))  # mont(R) = R^2
    s.append(fp_decl("FP_R3", (1 << 384) * RM % P))  # mont(2^384 R) (= R^3 for R = 2^384)
    s.append(fp_decl("FP_RCUBE", RM * RM % P))  # R^3: mont(y, R^3) = y R^2 (an integer inverse to Montgomery)
    s.append(fp_decl("FP_R2_SHL256", (1 << 256) * RM % P))  # mont(2^256 R) = 2^256 R^2 mod p
    s.append(f"LSG_CONST fpc_t FP_ONE_CANON = {{{arrl(1)}}};  // plain 1 (for from_mont)\n")
    if BITS != 32:  # plain multipliers between this layout and the 12 x 32-bit (R = 2^384) one
        s.append(f"LSG_CONST fpc_t FP_FROM_R384 = {{{arrl((1 << (2 * BITS * NL - 384)) % P)}}};  // x R^2 / 2^384\n")
        s.append(f"LSG_CONST fpc_t FP_TO_R384 = {{{arrl((1 << 384) % P)}}};  // x 2^384 / R\n")
    s.append(fp_decl("FP_HALF", pow(2, -1, P)))
    s.append(fp_decl("FP_B_G1", 4))
    s.append(fp_decl("FP_B3_G1", 12))
    s.append(fp2_decl("FP2_B_G2", (4, 4)))
    s.append(fp_decl("G1_GEN_X", G1_X))
    s.append(fp_decl("G1_GEN_Y", G1_Y))
    s.append(fp_decl("G1_GEN_NEG_Y", (-G1_Y) % P))
    s.append("\n")
    for i in range(6):
        s.append(fp2_decl(f"FROB1_G{i}", GAMMA1[i]))
    for i in range(6):
        s.append(fp2_decl(f"FROB2_G{i}", GAMMA2[i]))
    s.append(fp2_decl("PSI_CX", PSI_CX))
    s.append(fp2_decl("PSI_CY", PSI_CY))
    s.append(fp_decl("PSI2_CX", PSI2_CX[0]))
    s.append(fp_decl("PSI2_CY", PSI2_CY[0]))
    s.append("\n")
    s.append(fp2_decl("SSWU_A", SSWU_A))
    s.append(fp2_decl("SSWU_B", SSWU_B))
    s.append(fp2_decl("SSWU_Z", SSWU_Z))
    s.append(fp2_decl("SSWU_MINUS_B_OVER_A", MINUS_B_OVER_A))
    s.append(fp2_decl("SSWU_B_OVER_ZA", B_OVER_ZA))
    # N(Z)^((p+1)/4) with N(Z) = 5 a non-square: sqrt(N(gx2)) from sqrt-candidate of N(gx1) (lsg_h2c.hpp)
    s.append(fp_decl("SSWU_NZ_POW_P1D4", pow((SSWU_Z[0] ** 2 + SSWU_Z[1] ** 2) % P, (P + 1) // 4, P)))
    for name, poly in (("ISO_XNUM", ISO_XNUM), ("ISO_XDEN", ISO_XDEN), ("ISO_YNUM", ISO_YNUM), ("ISO_YDEN", ISO_YDEN)):
        for k, c in enumerate(poly):
            s.append(fp2_decl(f"{name}_{k}", c))
    with open(out, "w") as f:
        f.write("".join(s))


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "..", "lodestar_amd", "csrc", "lsg_constants.hpp")
    main(out)
    main(os.path.join(os.path.dirname(out), "lsg_constants_r29.hpp"), bits=29)
