#!/usr/bin/env python3
"""Build tool: straight-line programs (SLPs) for the per-group serial stages.

A final exponentiation (blst finalverify under packages/beacon-node/src/chain/bls/
maybeBatch.ts:18,37) or the signature-side Miller loop ML(-G1, sum r_i sig_i) of one RLC
group is a single dependency chain of ~10^4 Fp products.  Run as ordinary code it leaves a
wave64 waiting on one product at a time.  Here the chain is traced ONCE, at build time, into
a data-independent program of Fp operations over numbered value slots:

    MUL      dst = mont(sum_k a_k slot_k, sum_k b_k slot_k)      (Montgomery product)
    LIN      dst = sum_k c_k slot_k                              (small signed coefficients)
    LOADMUL  dst = mont(input Fp #j of the item, sum_k b_k slot_k)  (input conversion)

list-scheduled into steps of at most 32*W independent operations (critical path first) and
register-allocated into LDS slots.  lodestar_amd/csrc/lsg_slp.hip interprets the program
with one item per workgroup: in every step each lane PAIR of the W waves takes one operation
(pair backend: 14 limbs of 29 bits, lsg_fp_pair.hpp), gathers its operand forms from LDS,
multiplies and writes the result back.  A batch of 18 independent products then costs about
what one product costs, so a chain of 10^4 products runs in ~10^3 steps.

Linear combinations never get a step of their own when they can ride along: an operand of a
MUL is a form of up to 7 slots with coefficients in [-32, 31], gathered with 64-bit
accumulation and one carry round.  Value bounds are tracked (|v| < B p with B <= 2^12, the
pair backend's lazy range); a form that would exceed the limits is materialised by a LIN op,
a value that grows too large is tamed by a product with Montgomery one.

The algorithms below restate lodestar_amd/csrc/lsg_pairing.hpp (itself the mirror of
oracle/pairing.py): the Miller loop uses exactly the same projective doubling/addition steps
and line scalings, so Miller values are bit-identical to the other kernels'; field
arithmetic formulas (Karatsuba towers, Granger-Scott squaring) only have to be correct.
Every program is checked here, at generation time, by running the emitted op list
(scheduling and slot allocation included) on random inputs against a direct evaluation of the
same algorithm with Python integers.  Standalone: does not import oracle/ (the checker).

usage: gen_slp.py OUT.h [--check N]
"""
import heapq
import os
import random
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
X_ABS = 0xD201000000010000
NLIMB, LBITS = 14, 29
R = 1 << (NLIMB * LBITS)  # Montgomery radix of the pair backend (2^406)
RINV = pow(R, -1, P)
# Bounds (|v| < B p).  The pair backend's product w = (a b + m p) / R, 0 <= m < R = 2^406,
# satisfies -p < w < 2p whenever B_a B_b <= 2^25 (p / R < 2^-25); stored values stay below
# 2^20 p (the signed top limb then holds < 2^24, the 64-bit accumulators never overflow).
MUL_BB = 1 << 24  # B_a * B_b of a product's operands
MAXB = 1 << 12  # operand bound when both operands are large
LIN_MAX = 1 << 20  # any stored value
MAX_TERMS = 7  # terms per operand form (A and B each)
COEF_MIN, COEF_MAX = -32, 31
SLOT_BITS = 10
MAX_SLOTS = 1 << SLOT_BITS
W_LAT = {"mul": 1.0, "loadmul": 1.0, "lin": 0.25, "inv": 20.0}  # step costs relative to one product
COMBINE_TERMS = int(os.environ.get("LSG_SLP_COMBINE", "12"))  # a form built by +/- keeps up to this many terms
COMBINE_KEEP = int(os.environ.get("LSG_SLP_KEEP", "7"))  # ... and is cut back to this many
# Per program: the Miller-loop programs keep wider forms before cutting them back (their
# line and point formulas then collapse fewer fresh terms into LIN chains on the critical
# path: two-wave steps 330 -> 270 for a Miller item, 331 -> 273 for ML(-G1), 709 -> 651 for
# Horner + ML); the final exponentiation's Granger-Scott chain is shortest at 12 (630 steps;
# 643 at 14, 663 at 20, 1059 at 28).
COMBINE_BY_PROGRAM = {"miller_neg_g1": 28, "horner_miller": 28, "miller_item1": 28}
SPLIT_COLLAPSE = os.environ.get("LSG_SLP_SPLIT", "1") == "1"


def _n_enc(items):
    """encoded terms of a LIN over items (a coefficient outside [-32, 31] repeats its term)"""
    return sum(-(-c // COEF_MAX) if c > 0 else -(c // -COEF_MIN) for _, c in items)


# ----------------------------------------------------------------------------- engines
class IntF:
    """concrete Fp element (standard representation) -- the generator's reference evaluator"""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v % P

    def __add__(self, o):
        return IntF(self.v + o.v)

    def __sub__(self, o):
        return IntF(self.v - o.v)

    def __neg__(self):
        return IntF(-self.v)

    def __mul__(self, o):
        if isinstance(o, int):
            return IntF(self.v * o)
        return IntF(self.v * o.v)

    __rmul__ = __mul__


class IntEngine:
    def const(self, v):
        return IntF(v)

    def inv(self, a):
        return IntF(pow(a.v, -1, P) if a.v else 0)

    def zero(self):
        return IntF(0)


class Sym:
    """a linear form sum_k c_k * value_k over the program's values (Montgomery domain)"""
    __slots__ = ("cx", "t")

    def __init__(self, cx, t):
        self.cx = cx
        self.t = t

    def _combine(self, o, sign):
        t = dict(self.t)
        for v, c in o.t.items():
            t[v] = t.get(v, 0) + sign * c
        return Sym(self.cx, self.cx.shape({v: c for v, c in t.items() if c}))

    def __add__(self, o):
        return self._combine(o, 1)

    def __sub__(self, o):
        return self._combine(o, -1)

    def __neg__(self):
        return Sym(self.cx, {k: -c for k, c in self.t.items()})

    def __mul__(self, o):
        if isinstance(o, int):
            t = self.t
            if self.cx._fbound(t.items()) * abs(o) > LIN_MAX // 64:
                t = dict(self.cx.fit(t, MAX_TERMS, max(2, LIN_MAX // (64 * abs(o)))))
            return Sym(self.cx, self.cx.shape({k: c * o for k, c in t.items() if c * o}))
        return self.cx.mul(self, o)

    def __rmul__(self, o):
        assert isinstance(o, int)
        return self.__mul__(o)


class Ctx:
    """records a program: values are inputs, constants or op results.  Forms are kept
    expanded over op results as long as they stay small; when one must shrink, its OLDEST
    terms (earliest ready-time estimate) are collapsed into one LIN value -- that value is
    ready long before the recent terms (the products just made), so the LIN stays off the
    critical path of the chain"""

    def __init__(self, name, n_inputs, load_inputs=False):
        self.name = name
        self.ops = []  # [kind, dst, A terms, B terms, input index]
        self.bound = []  # per value: |v| < bound * p
        self.est = []  # per value: ready time estimate (products = 1, LIN = 0.25)
        self.prod = []  # per value: producing op index, or -1 (input/constant)
        self.consts = {}  # raw slot content -> value id
        self.const_list = []  # (value id, raw content)
        self.inputs = []  # value ids of raw inputs (non-LOADMUL programs)
        self.outputs = []
        self.memo = {}  # materialised term tuples -> value id
        self.n_inputs = n_inputs
        self.load_inputs = load_inputs
        self.one = self._raw_const(R % P)  # Montgomery one (taming)
        self.combine = COMBINE_TERMS if "LSG_SLP_COMBINE" in os.environ else COMBINE_BY_PROGRAM.get(name, COMBINE_TERMS)

    def _new(self, bound, prod, est=0.0):
        self.bound.append(bound)
        self.prod.append(prod)
        self.est.append(est)
        return len(self.bound) - 1

    def _raw_const(self, raw):
        if raw not in self.consts:
            v = self._new(1, -1)
            self.consts[raw] = v
            self.const_list.append((v, raw))
        return self.consts[raw]

    def form_est(self, vs):
        return max((self.est[v] for v in vs), default=0.0)

    # ---- engine interface
    def const(self, value):
        return Sym(self, {self._raw_const(value * R % P): 1})

    def zero(self):
        return Sym(self, {})

    def input(self, j):
        """input Fp #j of the item in Montgomery form"""
        if self.load_inputs == "mont":  # already Montgomery (lane-form values, < 2p)
            raw = self._new(2, -1)
            self.inputs.append(raw)
            return Sym(self, {raw: 1})
        if self.load_inputs:
            v = self._new(2, len(self.ops), 1.0)
            self.ops.append(["loadmul", v, [], [(self._raw_const(R * R % P), 1)], j])
            return Sym(self, {v: 1})
        raw = self._new(1, -1)
        self.inputs.append(raw)
        return self._mul_forms([(raw, 1)], [(self._raw_const(R * R % P), 1)])

    # ---- forms
    def _fbound(self, terms):
        return sum(abs(c) * self.bound[v] for v, c in terms)

    def _lin(self, terms):
        d = self._new(self._fbound(terms), len(self.ops), self.form_est(v for v, _ in terms) + W_LAT["lin"])
        assert self.bound[d] <= LIN_MAX, self.bound[d]
        self.ops.append(["lin", d, terms[:MAX_TERMS], terms[MAX_TERMS:], -1])
        return d

    def _tame_id(self, v):
        d = self._new(2, len(self.ops), self.est[v] + 1)
        self.ops.append(["mul", d, [(v, 1)], [(self.one, 1)], -1])
        return d

    def mat_terms(self, items, tame=False):
        """one value id holding sum c v over items (memoised); tame: reduced below 2p by a
        product with Montgomery one"""
        items = [(v, c) for v, c in items if c]
        if not items:
            return self._raw_const(0)
        if len(items) == 1 and items[0][1] == 1 and (not tame or self.bound[items[0][0]] <= 2):
            return items[0][0]
        key = (tuple(sorted(items)), tame)
        if key in self.memo:
            return self.memo[key]
        terms = []
        for v, c in items:  # coefficients outside the encodable range: repeat the term
            while c > COEF_MAX or c < COEF_MIN:
                step = COEF_MAX if c > 0 else COEF_MIN
                terms.append((v, step))
                c -= step
            if c:
                terms.append((v, c))
        while self._fbound(terms) > LIN_MAX:  # tame the largest contributions until it fits
            k = max(range(len(terms)), key=lambda i: abs(terms[i][1]) * self.bound[terms[i][0]])
            v, c = terms[k]
            if self.bound[v] <= 2:
                raise ValueError("form too large even with tamed terms")
            terms[k] = (self._tame_id(v), c)
        while len(terms) > 2 * MAX_TERMS:
            head = self._lin(terms[:2 * MAX_TERMS])
            terms = [(head, 1)] + terms[2 * MAX_TERMS:]
        d = self._lin(terms) if not (len(terms) == 1 and terms[0][1] == 1) else terms[0][0]
        if tame and self.bound[d] > 2:
            d = self._tame_id(d)
        self.memo[key] = d
        return d

    def fit(self, t, max_terms, max_bound):
        """the form t as <= max_terms encodable terms of bound <= max_bound: its oldest terms
        collapsed into one value (tamed when the bound needs it) when necessary"""
        items = [(v, c) for v, c in t.items() if c]

        def enc(it):
            return all(COEF_MIN <= c <= COEF_MAX for _, c in it)

        if len(items) <= max_terms and enc(items) and self._fbound(items) <= max_bound:
            return items
        # out-of-range coefficients first, then oldest first
        items.sort(key=lambda vc: (COEF_MIN <= vc[1] <= COEF_MAX, self.est[vc[0]], vc[0]))
        for m in range(1, len(items) + 1):
            old, rest = items[:m], items[m:]
            if len(rest) + 1 > max_terms or not enc(rest):
                continue
            b_rest, b_old = self._fbound(rest), self._fbound(old)
            if b_rest + min(b_old, 2) > max_bound:
                continue
            tame = b_rest + b_old > max_bound or b_old > LIN_MAX
            if m == 1 and not tame and enc(old):
                continue
            if not tame and SPLIT_COLLAPSE and _n_enc(old) > 2 * MAX_TERMS:
                split = self._split_collapse(items, m, max_terms, max_bound)
                if split is not None:
                    return split
            return [(self.mat_terms(old, tame), 1)] + rest
        return [(self.mat_terms(items, True), 1)]

    def _split_collapse(self, items, m0, max_terms, max_bound):
        """the oldest terms as several LIN values of <= 14 encoded terms each, computed side by
        side, where one value would need a chain (a LIN of 14 terms, then a LIN over it and the
        rest): the consumer takes the partial sums as separate terms.  None if no split fits."""
        for m in range(m0, len(items) + 1):
            old, rest = items[:m], items[m:]
            chunks, cur = [], []
            for it in old:
                if cur and _n_enc(cur + [it]) > 2 * MAX_TERMS:
                    chunks.append(cur)
                    cur = []
                cur.append(it)
            chunks.append(cur)
            if len(rest) + len(chunks) > max_terms:
                continue
            if self._fbound(rest) + self._fbound(old) > max_bound or self._fbound(old) > LIN_MAX:
                return None
            return [(self.mat_terms(ch, False), 1) for ch in chunks] + rest
        return None

    def shape(self, t):
        """keep a combined form within the working size"""
        if len(t) <= self.combine and self._fbound(t.items()) <= LIN_MAX // 64:
            return t
        return dict(self.fit(t, COMBINE_KEEP, LIN_MAX // 64))

    def _mul_forms(self, A, B):
        d = self._new(2, len(self.ops), self.form_est(v for v, _ in A + B) + 1)
        self.ops.append(["mul", d, A, B, -1])
        return Sym(self, {d: 1})

    def mul(self, a, b):
        if not a.t or not b.t:
            return self.zero()
        # the smaller operand first; the other may then be as large as the product allows
        if self._fbound(a.t.items()) < self._fbound(b.t.items()):
            a, b = b, a
        B = self.fit(b.t, MAX_TERMS, MAXB)
        A = self.fit(a.t, MAX_TERMS, min(LIN_MAX, MUL_BB // max(1, self._fbound(B))))
        return self._mul_forms(A, B)

    def inv(self, s):
        """s^-1: the INV operation inverts a value in (-p, 2p) (a product output) and
        multiplies the integer inverse by R^3 (Montgomery form of the inverse)"""
        t = self.mul(s, Sym(self, {self.one: 1}))
        (tv,) = t.t
        A = [(tv, 1)]
        B = [(self._raw_const(R * R * R % P), 1)]
        d = self._new(2, len(self.ops), self.est[tv] + W_LAT["inv"])
        self.ops.append(["inv", d, A, B, -1])
        return Sym(self, {d: 1})

    def output(self, s):
        """an output Fp: converted out of Montgomery form (in (-p, 2p), canonicalised by the
        kernel)"""
        A = self.fit(s.t, MAX_TERMS, LIN_MAX) if s.t else [(self._raw_const(0), 1)]
        # Montgomery-form outputs (lane-form consumers) are tamed below 2p; the others leave
        # Montgomery form for the canonical blobs
        B = [(self.one if self.load_inputs == "mont" else self._raw_const(1), 1)]
        d = self._new(2, len(self.ops))
        self.ops.append(["mul", d, A, B, -1])
        self.outputs.append(d)


# ----------------------------------------------------------------------------- tower
# Fp2 = Fp[u]/(u^2 + 1), Fp6 = Fp2[v]/(v^3 - xi), xi = 1 + u, Fp12 = Fp6[w]/(w^2 - v)
# (lsg_tower.hpp); elements are tuples of engine values.
def f2_add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def f2_sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def f2_neg(a):
    return (-a[0], -a[1])


def f2_conj(a):
    return (a[0], -a[1])


def f2_muls(a, k):
    return (a[0] * k, a[1] * k)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    t2 = (a[0] + a[1]) * (b[0] + b[1])
    return (t0 - t1, t2 - t0 - t1)


def f2_sqr(a):
    return ((a[0] + a[1]) * (a[0] - a[1]), 2 * (a[0] * a[1]))


def f2_mul_fp(a, s):
    return (a[0] * s, a[1] * s)


def f2_mul_xi(a):
    return (a[0] - a[1], a[0] + a[1])


def f2_zero(E):
    return (E.zero(), E.zero())


def f2_one(E):
    return (E.const(1), E.zero())


def f2_const(E, c):
    return (E.const(c[0]), E.const(c[1]))


def fp_pow(E, a, e):
    """a^e, sliding window of 4 (fixed public exponent)"""
    a2 = a * a
    T = [a]
    for _ in range(7):
        T.append(T[-1] * a2)
    bits = bin(e)[2:]
    i = 0
    r = None
    while i < len(bits):
        if bits[i] == "0":
            r = r * r
            i += 1
            continue
        j = min(i + 4, len(bits))
        while bits[j - 1] == "0":
            j -= 1
        val = int(bits[i:j], 2)
        if r is not None:
            for _ in range(j - i):
                r = r * r
            r = r * T[val >> 1]
        else:
            r = T[val >> 1]
        i = j
    return r


def fp_inv(E, a):
    """a^-1 (0 -> 0): one INV operation (divstep GCD, lsg_inv.hpp) in a program"""
    return E.inv(a)


def f2_inv(E, a):
    n = a[0] * a[0] + a[1] * a[1]
    ni = fp_inv(E, n)
    return (a[0] * ni, -(a[1] * ni))


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul_v(a):
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_mul(a, b):
    v0 = f2_mul(a[0], b[0])
    v1 = f2_mul(a[1], b[1])
    v2 = f2_mul(a[2], b[2])
    c0 = f2_add(v0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a[1], a[2]), f2_add(b[1], b[2])), v1), v2)))
    c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a[0], a[1]), f2_add(b[0], b[1])), v0), v1), f2_mul_xi(v2))
    c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a[0], a[2]), f2_add(b[0], b[2])), v0), v2), v1)
    return (c0, c1, c2)


def f6_mul_01(a, b0, b1):
    v0 = f2_mul(a[0], b0)
    v1 = f2_mul(a[1], b1)
    c0 = f2_add(f2_mul_xi(f2_mul(a[2], b1)), v0)
    c1 = f2_sub(f2_sub(f2_mul(f2_add(a[0], a[1]), f2_add(b0, b1)), v0), v1)
    c2 = f2_add(f2_mul(a[2], b0), v1)
    return (c0, c1, c2)


def f6_mul_1(a, b1):
    return (f2_mul_xi(f2_mul(a[2], b1)), f2_mul(a[0], b1), f2_mul(a[1], b1))


def f6_inv(E, a):
    t0 = f2_sub(f2_sqr(a[0]), f2_mul_xi(f2_mul(a[1], a[2])))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a[2])), f2_mul(a[0], a[1]))
    t2 = f2_sub(f2_sqr(a[1]), f2_mul(a[0], a[2]))
    den = f2_add(f2_mul(a[0], t0), f2_mul_xi(f2_add(f2_mul(a[2], t1), f2_mul(a[1], t2))))
    di = f2_inv(E, den)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


def f12_mul(a, b):
    t0 = f6_mul(a[0], b[0])
    t1 = f6_mul(a[1], b[1])
    t2 = f6_mul(f6_add(a[0], a[1]), f6_add(b[0], b[1]))
    return (f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(t2, t0), t1))


def f12_sqr(a):
    t = f6_mul(a[0], a[1])
    u = f6_mul(f6_add(a[0], a[1]), f6_add(a[0], f6_mul_v(a[1])))
    return (f6_sub(f6_sub(u, t), f6_mul_v(t)), f6_add(t, t))


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(E, a):
    t = f6_sub(f6_mul(a[0], a[0]), f6_mul_v(f6_mul(a[1], a[1])))
    ti = f6_inv(E, t)
    return (f6_mul(a[0], ti), f6_neg(f6_mul(a[1], ti)))


def f12_one(E):
    z = f2_zero(E)
    return ((f2_one(E), z, z), (z, z, z))


def f12_mul_line(f, l00, l01, l11):
    t0 = f6_mul_01(f[0], l00, l01)
    u = f6_mul_01(f6_add(f[0], f[1]), l00, f2_add(l01, l11))
    t1 = f6_mul_1(f[1], l11)
    return (f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(u, t0), t1))


def _f2pow(a, e):
    def m(x, y):
        return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)
    r = (1, 0)
    while e:
        if e & 1:
            r = m(r, a)
        a = m(a, a)
        e >>= 1
    return r


XI = (1, 1)
G1C = [_f2pow(XI, j * (P - 1) // 6) for j in range(6)]  # frobenius: coefficient of w^j
G2C = [_f2pow(XI, j * (P * P - 1) // 6) for j in range(6)]


def f12_frob(E, a):
    # w^j order: c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2
    c = [a[0][0], a[1][0], a[0][1], a[1][1], a[0][2], a[1][2]]
    r = [f2_conj(c[0])] + [f2_mul(f2_conj(c[j]), f2_const(E, G1C[j])) for j in range(1, 6)]
    return ((r[0], r[2], r[4]), (r[1], r[3], r[5]))


def f12_frob2(E, a):
    c = [a[0][0], a[1][0], a[0][1], a[1][1], a[0][2], a[1][2]]
    r = [c[0]] + [f2_mul_fp(c[j], E.const(G2C[j][0])) for j in range(1, 6)]
    assert all(G2C[j][1] == 0 for j in range(6))
    return ((r[0], r[2], r[4]), (r[1], r[3], r[5]))


def fp4_square(a, b):
    t0 = f2_sqr(a)
    t1 = f2_sqr(b)
    c0 = f2_add(f2_mul_xi(t1), t0)
    c1 = f2_sub(f2_sub(f2_sqr(f2_add(a, b)), t0), t1)
    return c0, c1


def f12_cyc_sqr(f):
    """Granger-Scott squaring (f in the cyclotomic subgroup), lsg_tower.hpp:412"""
    z0, z4, z3 = f[0]
    z2, z1, z5 = f[1]
    t0, t1 = fp4_square(z0, z1)
    u0, u1 = fp4_square(z2, z3)
    t2, t3 = fp4_square(z4, z5)
    z0 = f2_add(f2_muls(f2_sub(t0, z0), 2), t0)
    z1 = f2_add(f2_muls(f2_add(t1, z1), 2), t1)
    z4 = f2_add(f2_muls(f2_sub(u0, z4), 2), u0)
    z5 = f2_add(f2_muls(f2_add(u1, z5), 2), u1)
    t0 = f2_mul_xi(t3)
    z2 = f2_add(f2_muls(f2_add(t0, z2), 2), t0)
    z3 = f2_add(f2_muls(f2_sub(t2, z3), 2), t2)
    return ((z0, z4, z3), (z2, z1, z5))


def f12_exp_by_x(g):
    r = g
    for b in range(62, -1, -1):
        r = f12_cyc_sqr(r)
        if (X_ABS >> b) & 1:
            r = f12_mul(r, g)
    return f12_conj(r)


def final_exp(E, f):
    """f^(3 (p^12 - 1)/r), lsg_pairing.hpp:318"""
    f1 = f12_mul(f12_conj(f), f12_inv(E, f))
    g = f12_mul(f12_frob2(E, f1), f1)
    t0 = f12_mul(f12_exp_by_x(g), f12_conj(g))
    t0 = f12_mul(f12_exp_by_x(t0), f12_conj(t0))
    t1 = f12_mul(f12_exp_by_x(t0), f12_frob(E, t0))
    t2 = f12_mul(f12_mul(f12_exp_by_x(f12_exp_by_x(t1)), f12_frob2(E, t1)), f12_conj(t1))
    return f12_mul(t2, f12_mul(f12_sqr(g), g))


# ----------------------------------------------------------------------------- curve
B3 = 12  # 3 b' with b' = 4 (1 + u): fp2_mul_b3(a) = 12 xi a


def f2_mul_b3(a):
    return f2_muls(f2_mul_xi(a), B3)


def g2_add(p, q):
    """RCB 2016 algorithm 7 (complete addition, a = 0), lsg_curve.hpp:82"""
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    t0 = f2_mul(X1, X2)
    t1 = f2_mul(Y1, Y2)
    t2 = f2_mul(Z1, Z2)
    t3 = f2_sub(f2_mul(f2_add(X1, Y1), f2_add(X2, Y2)), f2_add(t0, t1))
    t4 = f2_sub(f2_mul(f2_add(Y1, Z1), f2_add(Y2, Z2)), f2_add(t1, t2))
    Y3 = f2_sub(f2_mul(f2_add(X1, Z1), f2_add(X2, Z2)), f2_add(t0, t2))
    t0 = f2_muls(t0, 3)
    t2 = f2_mul_b3(t2)
    Z3 = f2_add(t1, t2)
    t1 = f2_sub(t1, t2)
    Y3 = f2_mul_b3(Y3)
    X3 = f2_sub(f2_mul(t3, t1), f2_mul(t4, Y3))
    Y3 = f2_add(f2_mul(t1, Z3), f2_mul(Y3, t0))
    Z3 = f2_add(f2_mul(Z3, t4), f2_mul(t0, t3))
    return (X3, Y3, Z3)


def g2_dbl(p):
    """RCB 2016 algorithm 9 (doubling, a = 0), lsg_curve.hpp:151"""
    X, Y, Z = p
    t0 = f2_sqr(Y)
    Z3 = f2_muls(t0, 8)
    t1 = f2_mul(Y, Z)
    t2 = f2_mul_b3(f2_sqr(Z))
    X3 = f2_mul(t2, Z3)
    Y3 = f2_add(t0, t2)
    Z3 = f2_mul(t1, Z3)
    t0 = f2_sub(t0, f2_muls(t2, 3))
    Y3 = f2_add(X3, f2_mul(t0, Y3))
    X3 = f2_muls(f2_mul(t0, f2_mul(X, Y)), 2)
    return (X3, Y3, Z3)


def ml_dbl_step(T):
    """T <- 2T and its unevaluated line, lsg_pairing.hpp:17 (same representatives)"""
    X, Y, Z = T
    t0 = f2_sqr(Y)
    t1 = f2_mul(Y, Z)
    t2 = f2_mul_b3(f2_sqr(Z))
    XX = f2_sqr(X)
    l00 = f2_sub(t2, t0)
    l01 = f2_muls(XX, 3)
    l11 = f2_neg(f2_muls(t1, 2))
    Z3 = f2_muls(t0, 8)
    X3 = f2_mul(t2, Z3)
    Y3 = f2_add(t0, t2)
    Z3 = f2_mul(t1, Z3)
    s0 = f2_sub(t0, f2_muls(t2, 3))
    Y3 = f2_add(X3, f2_mul(s0, Y3))
    X3 = f2_muls(f2_mul(s0, f2_mul(X, Y)), 2)
    return (X3, Y3, Z3), (l00, l01, l11)


def ml_add_step(T, Q):
    """T <- T + Q (Q affine) and its unevaluated line, lsg_pairing.hpp:48"""
    X, Y, Z = T
    qx, qy = Q
    theta = f2_sub(Y, f2_mul(qy, Z))
    delta = f2_sub(X, f2_mul(qx, Z))
    l00 = f2_sub(f2_mul(delta, qy), f2_mul(theta, qx))
    l01 = theta
    l11 = f2_neg(delta)
    C = f2_sqr(theta)
    D = f2_sqr(delta)
    Ee = f2_mul(D, delta)
    F = f2_mul(Z, C)
    G = f2_mul(X, D)
    H = f2_sub(f2_add(Ee, F), f2_muls(G, 2))
    X3 = f2_mul(delta, H)
    Y3 = f2_sub(f2_mul(theta, f2_sub(G, H)), f2_mul(Ee, Y))
    Z3 = f2_mul(Ee, Z)
    return (X3, Y3, Z3), (l00, l01, l11)


def miller_loop(E, Pxy, Q):
    """f_{|x|,Q}(P) conjugated, lsg_pairing.hpp:173 (P affine G1, Q affine G2)"""
    xP, yP = Pxy

    def ev(L):
        return (L[0], f2_mul_fp(L[1], xP), f2_mul_fp(L[2], yP))

    T = (Q[0], Q[1], f2_one(E))
    T, L = ml_dbl_step(T)
    L = ev(L)
    z = f2_zero(E)
    f = ((L[0], L[1], z), (z, L[2], z))
    T, L = ml_add_step(T, Q)
    f = f12_mul_line(f, *ev(L))
    for b in range(61, -1, -1):
        f = f12_sqr(f)
        T, L = ml_dbl_step(T)
        f = f12_mul_line(f, *ev(L))
        if (X_ABS >> b) & 1:
            T, L = ml_add_step(T, Q)
            f = f12_mul_line(f, *ev(L))
    return f12_conj(f)


G1X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1


def proj_to_aff(E, p):
    zi = f2_inv(E, p[2])
    return (f2_mul(p[0], zi), f2_mul(p[1], zi))


def ml_neg_g1(E, S):
    """ML(-G1, S) for S projective (lsg_serial.hip:44); the caller substitutes 1 when S = O"""
    return miller_loop(E, (E.const(G1X), E.const(P - G1Y)), proj_to_aff(E, S))


def horner(Cs):
    """S = sum_k 2^k C_k by Horner over the 64 per-bit sums (lsg_serial.hip:63)"""
    s = Cs[63]
    for k in range(62, -1, -1):
        s = g2_add(g2_dbl(s), Cs[k])
    return s


# ----------------------------------------------------------------------------- programs
def flat12(f):
    return [x for c6 in f for c2 in c6 for x in c2]


def unflat12(v):
    return tuple(tuple((v[6 * a + 2 * b], v[6 * a + 2 * b + 1]) for b in range(3)) for a in range(2))


def g2p_from(v, o=0):
    return ((v[o], v[o + 1]), (v[o + 2], v[o + 3]), (v[o + 4], v[o + 5]))


def prog_final_exp(E, inp):
    """in: F (12 Fp, tower order); out: FE(F) (12 Fp) -- the kernel compares with one"""
    return flat12(final_exp(E, unflat12(inp(12))))


def prog_miller_neg_g1(E, inp):
    """in: S projective (6 Fp); out: ML(-G1, S) (12 Fp) and S.Z (2 Fp: S = O test)"""
    v = inp(6)
    S = g2p_from(v)
    return flat12(ml_neg_g1(E, S)) + list(S[2])


def prog_horner_miller(E, inp):
    """in: 64 per-bit sums C_k (64 x 6 Fp); out: ML(-G1, S) (12 Fp) and S.Z (2 Fp)"""
    v = inp(384)
    S = horner([g2p_from(v, 6 * k) for k in range(64)])
    return flat12(ml_neg_g1(E, S)) + list(S[2])


def miller_loop_masked(E, Pxy, Q, u):
    """f_{|x|,Q}(P) conjugated for one pair of a Miller item (lsg_pairing.hpp:173), with the
    pair's use flag u (Montgomery 1 or 0) folded into every line: a pair that does not take
    part (P = (0, 0), u = 0) contributes the line (1, 0, 0) at every step, i.e. exactly 1 --
    the same identity lines k_miller_fused uses for such pairs"""
    xP, yP = Pxy
    one = E.const(1)

    def ev(L):
        l00 = (u * (L[0][0] - one) + one, u * L[0][1])
        return (l00, f2_mul_fp(L[1], xP), f2_mul_fp(L[2], yP))

    T = (Q[0], Q[1], f2_one(E))
    T, L = ml_dbl_step(T)
    L = ev(L)
    z = f2_zero(E)
    f = ((L[0], L[1], z), (z, L[2], z))
    T, L = ml_add_step(T, Q)
    f = f12_mul_line(f, *ev(L))
    for b in range(61, -1, -1):
        f = f12_sqr(f)
        T, L = ml_dbl_step(T)
        f = f12_mul_line(f, *ev(L))
        if (X_ABS >> b) & 1:
            T, L = ml_add_step(T, Q)
            f = f12_mul_line(f, *ev(L))
    return f12_conj(f)


def prog_miller_item1(E, inp):
    """in (Montgomery lane-form values): P (x, y; 0 when the pair is unused), Q = H(m)
    (x.c0, x.c1, y.c0, y.c1), u (1 or 0); out: the item's Miller value (12 Fp, Montgomery)"""
    v = inp(7)
    return flat12(miller_loop_masked(E, (v[0], v[1]), ((v[2], v[3]), (v[4], v[5])), v[6]))


def _f2inv_int(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
    return (a[0] * n % P, -a[1] * n % P)


def _f2mul_int(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


PSI_CX = _f2inv_int(_f2pow(XI, (P - 1) // 3))  # psi(x, y) = (conj(x) cx, conj(y) cy)
PSI_CY = _f2inv_int(_f2pow(XI, (P - 1) // 2))
PSI2_CX = _f2mul_int(PSI_CX, (PSI_CX[0], -PSI_CX[1] % P))[0]  # psi^2 = psi o psi: the norms
PSI2_CY = _f2mul_int(PSI_CY, (PSI_CY[0], -PSI_CY[1] % P))[0]


def g2_psi(E, p):
    return (f2_mul(f2_conj(p[0]), f2_const(E, PSI_CX)), f2_mul(f2_conj(p[1]), f2_const(E, PSI_CY)), f2_conj(p[2]))


def g2_psi2(E, p):
    return (f2_mul_fp(p[0], E.const(PSI2_CX)), f2_mul_fp(p[1], E.const(PSI2_CY)), p[2])


def g2_neg(p):
    return (p[0], f2_neg(p[1]), p[2])


def jac_dbl(p):
    """Jacobian doubling, a = 0 (lsg_curve.hpp jac_dbl_t)"""
    X, Y, Z = p
    A = f2_sqr(X)
    B = f2_sqr(Y)
    C = f2_sqr(B)
    D = f2_muls(f2_sub(f2_sqr(f2_add(X, B)), f2_add(A, C)), 2)
    Ee = f2_muls(A, 3)
    X3 = f2_sub(f2_sqr(Ee), f2_muls(D, 2))
    Y3 = f2_sub(f2_mul(Ee, f2_sub(D, X3)), f2_muls(C, 8))
    Z3 = f2_muls(f2_mul(Y, Z), 2)
    return (X3, Y3, Z3)


def jac_from_proj(p):
    """homogeneous (X:Y:Z) -> Jacobian (XZ : YZ^2 : Z) (lsg_curve.hpp; the infinity select of
    the kernels is left out: a hashed point at infinity has probability < 2^-380)"""
    return (f2_mul(p[0], p[2]), f2_mul(p[1], f2_sqr(p[2])), p[2])


def jac_to_proj(p):
    return (f2_mul(p[0], p[2]), p[1], f2_mul(f2_sqr(p[2]), p[2]))


def proj_mul_xabs(p):
    """[|x|]P: 63 Jacobian doublings, 5 complete additions (lsg_curve.hpp proj_mul_xabs)"""
    acc = jac_from_proj(p)
    for b in range(62, -1, -1):
        acc = jac_dbl(acc)
        if (X_ABS >> b) & 1:
            acc = jac_from_proj(g2_add(jac_to_proj(acc), p))
    return jac_to_proj(acc)


def clear_cofactor(E, p):
    """h_eff P = c + [x]([x]P + psi(P)), c = psi^2(2P) - psi(P) - P - [x]P (lsg_h2c.hpp:228)"""
    u = g2_psi(E, p)
    c = g2_add(g2_psi2(E, g2_dbl(p)), g2_neg(u))
    c = g2_add(c, g2_neg(p))
    t1 = g2_neg(proj_mul_xabs(p))
    c = g2_add(c, g2_neg(t1))
    t2 = g2_neg(proj_mul_xabs(g2_add(t1, u)))
    return g2_add(c, t2)


def prog_h2c_clear(E, inp):
    """in (Montgomery lane form): Q0 + Q1 of the SSWU map, projective (6 Fp); out: H = h_eff Q
    affine (4 Fp, Montgomery) and its projective Z (2 Fp: the H = O test)"""
    v = inp(6)
    q = clear_cofactor(E, g2p_from(v))
    zi = f2_inv(E, q[2])
    return list(f2_mul(q[0], zi)) + list(f2_mul(q[1], zi)) + list(q[2])


def g2_mul_xabs_complete(p):
    """[|x|]P with the complete formulas only (RCB doubling and addition): exact for every
    point of E2, small-order ones included -- the subgroup check's inputs are adversarial"""
    acc = p
    for b in range(62, -1, -1):
        acc = g2_dbl(acc)
        if (X_ABS >> b) & 1:
            acc = g2_add(acc, p)
    return acc


def prog_g2_subgroup(E, inp):
    """Scott's test psi(P) == [x]P (x < 0; lsg_curve.hpp g2_in_group) for an affine signature
    point (4 Fp, Montgomery lane form); out: X1 Z2 - X2 Z1, Y1 Z2 - Y2 Z1 of psi(P) and -[|x|]P
    (4 Fp): both zero iff P is in G2 (the kernel reads them)"""
    v = inp(4)
    P = ((v[0], v[1]), (v[2], v[3]), f2_one(E))
    X1, Y1, Z1 = g2_psi(E, P)
    X2, Y2, Z2 = g2_neg(g2_mul_xabs_complete(P))
    return list(f2_sub(f2_mul(X1, Z2), f2_mul(X2, Z1))) + list(f2_sub(f2_mul(Y1, Z2), f2_mul(Y2, Z1)))


def prog_g2_scale(E, inp):
    """[r] sig for the RLC (lsg_k_sig.hip k_sig_scale): in the affine point (4 Fp, Montgomery
    lane form) and the 64 bits of r as 0 / 1 (Montgomery) values, least significant first; out:
    [r] P projective (6 Fp).  2-bit windows: the window's point (O, P, 2P or 3P) is a linear
    combination of the precomputed multiples with the window's indicator values -- selected
    off the critical path -- added with the complete formulas (exact for O)"""
    v = inp(4 + 64)
    one = E.const(1)
    P = ((v[0], v[1]), (v[2], v[3]), f2_one(E))
    bits = v[4:]
    P2 = g2_dbl(P)
    P3 = g2_add(P2, P)
    T = None
    for w in range(31, -1, -1):
        b1, b0 = bits[2 * w + 1], bits[2 * w]
        c3 = b1 * b0
        c2 = b1 - c3
        c1 = b0 - c3
        pick = []
        for k in range(3):  # X, Y, Z
            comp = []
            for i in range(2):
                t = c1 * P[k][i] if not (k == 2) else (c1 if i == 0 else E.zero())
                t = t + c2 * P2[k][i] + c3 * P3[k][i]
                if k == 1 and i == 0:
                    t = t + (one - c1 - c2 - c3)  # O = (0 : 1 : 0)
                comp.append(t)
            pick.append(tuple(comp))
        D = tuple(pick)
        T = D if T is None else g2_add(g2_dbl(g2_dbl(T)), D)
    return [c for pt in T for c in pt]


PROGRAMS = {
    # name: (builder, n_inputs, inputs: False = canonical blob bytes, True = loaded by LOADMUL
    #        ops inside the program, "mont" = Montgomery lane-form values, outputs likewise)
    "final_exp": (prog_final_exp, 12, False),
    "miller_neg_g1": (prog_miller_neg_g1, 6, False),
    "horner_miller": (prog_horner_miller, 384, True),
    "miller_item1": (prog_miller_item1, 7, "mont"),
    "h2c_clear": (prog_h2c_clear, 6, "mont"),
    "g2_subgroup": (prog_g2_subgroup, 4, "mont"),
    "g2_scale": (prog_g2_scale, 68, "mont"),
}


def trace(name):
    fn, n_in, load = PROGRAMS[name]
    cx = Ctx(name, n_in, load)
    ins = [None]

    def inp(n):
        assert n == n_in
        ins[0] = [cx.input(j) for j in range(n)]
        return ins[0]

    outs = fn(cx, inp)
    for o in outs:
        cx.output(o)
    return cx


# ----------------------------------------------------------------------------- schedule
def dce(cx):
    live = [False] * len(cx.ops)
    stack = [cx.prod[v] for v in cx.outputs if cx.prod[v] >= 0]
    while stack:
        i = stack.pop()
        if live[i]:
            continue
        live[i] = True
        for v, _ in cx.ops[i][2] + cx.ops[i][3]:
            if cx.prod[v] >= 0 and not live[cx.prod[v]]:
                stack.append(cx.prod[v])
    return [i for i in range(len(cx.ops)) if live[i]]


# One-wave programs run where a launch holds hundreds of groups (throughput): a step costs its
# slowest lane, so a step with any product costs a product, while a step of linear combinations
# alone skips the product (~1/3 of the cost).  Their steps are typed: a product step when at
# least TYPED_ALPHA * 32 products are ready (its spare lanes take linear combinations), a
# step of linear combinations otherwise.  Final exponentiation: 766 -> ~650 product-step
# equivalents; ML(-G1) 437 -> ~340; a Miller item 436 -> ~345.
# (The cofactor-clearing and [r] sig programs are product chains: typed steps only lengthen
# them, and the clearing runs one wave per set for a lone set too.)
TYPED_ALPHA = float(os.environ.get("LSG_SLP_TYPED", "0.5"))
TYPED_PROGRAMS = ("final_exp", "miller_neg_g1", "miller_item1", "horner_miller", "g2_subgroup")


def schedule(cx, W, earliest=None, typed=None):
    """list scheduling: steps of <= 32 W ops, longest remaining path first (typed: see
    TYPED_ALPHA)"""
    if typed == "crit":
        return _schedule_crit(cx, W, earliest)
    if typed:
        return _schedule_typed(cx, W, typed, earliest)
    cap = 32 * W
    ops = dce(cx)
    idx = {o: k for k, o in enumerate(ops)}
    n = len(ops)
    preds = [[] for _ in range(n)]
    succs = [[] for _ in range(n)]
    for k, o in enumerate(ops):
        seen = set()
        for v, _ in cx.ops[o][2] + cx.ops[o][3]:
            p = cx.prod[v]
            if p >= 0 and p not in seen:
                seen.add(p)
                preds[k].append(idx[p])
                succs[idx[p]].append(k)
    lat = [W_LAT[cx.ops[o][0]] for o in ops]
    prio = [0.0] * n
    for k in range(n - 1, -1, -1):  # ops are recorded in a topological order
        prio[k] = lat[k] + max((prio[s] for s in succs[k]), default=0.0)
    npred = [len(p) for p in preds]
    ready_at = [0] * n
    heap = [(-prio[k], k) for k in range(n) if npred[k] == 0]
    heapq.heapify(heap)
    steps = []
    waiting = []  # (step, k): ready only from that step on
    t = 0
    done = 0
    while done < n:
        cur = []
        deferred = []
        while heap and len(cur) < cap:
            pr, k = heapq.heappop(heap)
            if ready_at[k] > t or (earliest and earliest.get(ops[k], 0) > t):
                deferred.append((pr, k))
                continue
            cur.append(k)
        for x in deferred:
            heapq.heappush(heap, x)
        if not cur:
            t += 1
            steps.append([])
            continue
        steps.append([ops[k] for k in cur])
        done += len(cur)
        for k in cur:
            for s in succs[k]:
                npred[s] -= 1
                ready_at[s] = max(ready_at[s], t + 1)
                if npred[s] == 0:
                    heapq.heappush(heap, (-prio[s], s))
        t += 1
    return [s for s in steps if s]


def _schedule_typed(cx, W, alpha, earliest=None):
    cap = 32 * W
    ops = dce(cx)
    idx = {o: k for k, o in enumerate(ops)}
    n = len(ops)
    preds = [[] for _ in range(n)]
    succs = [[] for _ in range(n)]
    for k, o in enumerate(ops):
        seen = set()
        for v, _ in cx.ops[o][2] + cx.ops[o][3]:
            p = cx.prod[v]
            if p >= 0 and p not in seen:
                seen.add(p)
                preds[k].append(idx[p])
                succs[idx[p]].append(k)
    islin = [cx.ops[o][0] == "lin" for o in ops]
    lat = [W_LAT[cx.ops[o][0]] for o in ops]
    prio = [0.0] * n
    for k in range(n - 1, -1, -1):
        prio[k] = lat[k] + max((prio[s] for s in succs[k]), default=0.0)
    npred = [len(p) for p in preds]
    hm, hl = [], []  # ready products, ready linear combinations
    for k in range(n):
        if npred[k] == 0:
            heapq.heappush(hl if islin[k] else hm, (-prio[k], k))
    steps = []
    done = 0
    t = 0

    def take(h, cur):
        deferred = []
        while h and len(cur) < cap:
            pr, k = heapq.heappop(h)
            if earliest and earliest.get(ops[k], 0) > t:
                deferred.append((pr, k))
                continue
            cur.append(k)
        for x in deferred:
            heapq.heappush(h, x)

    while done < n:
        cur = []
        n_mul = sum(1 for _, k in hm if not (earliest and earliest.get(ops[k], 0) > t))
        n_lin = sum(1 for _, k in hl if not (earliest and earliest.get(ops[k], 0) > t))
        if n_mul >= alpha * cap or (n_mul and not n_lin):
            take(hm, cur)
        take(hl, cur)
        if cur:
            steps.append([ops[k] for k in cur])
            done += len(cur)
            for k in cur:
                for s in succs[k]:
                    npred[s] -= 1
                    if npred[s] == 0:
                        heapq.heappush(hl if islin[s] else hm, (-prio[s], s))
        t += 1
    return steps


# Two-wave programs run where a launch holds few groups (latency): a step of linear
# combinations alone still skips the product, so a linear combination on the critical path is
# cheaper in a step of its own than riding in a product step.  Priorities are remaining
# critical-path costs with a LIN at CRIT_LIN of a product step; a step takes only linear
# combinations when the most critical ready one outranks every ready product.  Final
# exponentiation: 612 -> ~550 product-step equivalents (618 -> 636 steps, ~130 of them cheap).
CRIT_LIN = 0.5


def _schedule_crit(cx, W, earliest=None):
    cap = 32 * W
    ops = dce(cx)
    idx = {o: k for k, o in enumerate(ops)}
    n = len(ops)
    preds = [[] for _ in range(n)]
    succs = [[] for _ in range(n)]
    for k, o in enumerate(ops):
        seen = set()
        for v, _ in cx.ops[o][2] + cx.ops[o][3]:
            p = cx.prod[v]
            if p >= 0 and p not in seen:
                seen.add(p)
                preds[k].append(idx[p])
                succs[idx[p]].append(k)
    islin = [cx.ops[o][0] == "lin" for o in ops]
    lat = [CRIT_LIN if islin[k] else W_LAT[cx.ops[ops[k]][0]] for k in range(n)]
    prio = [0.0] * n
    for k in range(n - 1, -1, -1):
        prio[k] = lat[k] + max((prio[s] for s in succs[k]), default=0.0)
    npred = [len(p) for p in preds]
    hm, hl = [], []
    for k in range(n):
        if npred[k] == 0:
            heapq.heappush(hl if islin[k] else hm, (-prio[k], k))
    steps = []
    done = 0
    t = 0

    def ready(k):
        return not (earliest and earliest.get(ops[k], 0) > t)

    def top(h):
        return max((-pr for pr, k in h if ready(k)), default=None)

    def take(h, cur):
        deferred = []
        while h and len(cur) < cap:
            pr, k = heapq.heappop(h)
            if not ready(k):
                deferred.append((pr, k))
                continue
            cur.append(k)
        for x in deferred:
            heapq.heappush(h, x)

    while done < n:
        cur = []
        tm, tl = top(hm), top(hl)
        if tm is not None and (tl is None or tl <= tm):
            take(hm, cur)
        take(hl, cur)
        if cur:
            steps.append([ops[k] for k in cur])
            done += len(cur)
            for k in cur:
                for s2 in succs[k]:
                    npred[s2] -= 1
                    if npred[s2] == 0:
                        heapq.heappush(hl if islin[s2] else hm, (-prio[s2], s2))
        t += 1
    return steps


def _hold_back(cx, steps, pred, lead):
    """earliest steps holding every op selected by pred back to `lead` steps before its first
    consumer in `steps` (ops scheduled early only because capacity was free hold their results
    in LDS for nothing)"""
    first_use = {}
    for t, st in enumerate(steps):
        for o in st:
            for v, _ in cx.ops[o][2] + cx.ops[o][3]:
                p = cx.prod[v]
                if p >= 0 and pred(p):
                    first_use[p] = min(first_use.get(p, 1 << 30), t)
    return {p: max(0, u - lead) for p, u in first_use.items()}


def schedule_loads(cx, W, passes=3, lead=4):
    """list schedule, then hold LOADMUL inputs and off-critical-path work back towards their
    consumers: a few passes, each kept only if it does not lengthen the program"""
    typed = None
    if cx.name in TYPED_PROGRAMS:
        if W == 1 and TYPED_ALPHA > 0:
            typed = TYPED_ALPHA
        elif W == 2 and CRIT_LIN > 0 and os.environ.get("LSG_SLP_CRIT", "1") == "1":
            typed = "crit"
    steps = schedule(cx, W, typed=typed)
    if cx.load_inputs is True:
        steps = schedule(cx, W, _hold_back(cx, steps, lambda p: cx.ops[p][0] == "loadmul", 3), typed=typed)
    best = steps
    _, best_slots = allocate(cx, best)
    for _ in range(passes):
        cand = schedule(cx, W, _hold_back(cx, steps, lambda p: True, lead), typed=typed)
        if len(cand) > len(best) * 1.01:
            break
        _, ns = allocate(cx, cand)
        steps = cand
        if ns < best_slots:
            best, best_slots = cand, ns
    return best


def allocate(cx, steps):
    """LDS slots: constants first (kept), then values by their lifetime in steps"""
    n_val = len(cx.bound)
    slot = [-1] * n_val
    for k, (v, _) in enumerate(cx.const_list):
        slot[v] = k
    base = len(cx.const_list)
    last = [-1] * n_val
    for t, s in enumerate(steps):
        for o in s:
            for v, _ in cx.ops[o][2] + cx.ops[o][3]:
                last[v] = max(last[v], t)
    for v in cx.outputs:
        last[v] = 1 << 30
    free = []
    nxt = base
    expire = {}  # step -> slots freed after it
    for v in cx.inputs:
        if nxt >= MAX_SLOTS:
            raise ValueError("slots")
        slot[v] = nxt
        nxt += 1
        expire.setdefault(last[v], []).append(slot[v])
    for t, s in enumerate(steps):
        # slots last read before step t are free for writes in step t
        for sl in expire.pop(t - 1, []):
            heapq.heappush(free, sl)
        for o in s:
            d = cx.ops[o][1]
            if free:
                sl = heapq.heappop(free)
            else:
                sl = nxt
                nxt += 1
            slot[d] = sl
            if last[d] < 0:
                last[d] = t  # dead value (cannot happen after dce except outputs)
            expire.setdefault(max(last[d], t), []).append(sl)
    if nxt > MAX_SLOTS:
        raise ValueError("%s: %d slots > %d" % (cx.name, nxt, MAX_SLOTS))
    return slot, nxt


# ----------------------------------------------------------------------------- check
def run_program(cx, steps, slot, n_slots, raw_inputs):
    """execute the scheduled, allocated program (values mod p, Montgomery semantics)"""
    mem = [None] * n_slots
    for v, raw in cx.const_list:
        mem[slot[v]] = raw % P
    for v, x in zip(cx.inputs, raw_inputs):
        mem[slot[v]] = x % P

    def form(terms):
        s = 0
        for v, c in terms:
            x = mem[slot[v]]
            assert x is not None, "read of an unwritten slot"
            s += c * x
        return s % P

    for s in steps:
        res = []
        for o in s:
            kind, d, A, B, j = cx.ops[o]
            if kind == "lin":
                r = (form(A) + form(B)) % P
            elif kind == "mul":
                r = form(A) * form(B) * RINV % P
            elif kind == "inv":
                x = form(A)
                r = (pow(x, -1, P) if x else 0) * form(B) * RINV % P
            else:
                r = raw_inputs[j] * form(B) * RINV % P
            res.append((slot[d], r))
        for sl, r in res:  # writes after every read of the step
            mem[sl] = r
    return [mem[slot[v]] for v in cx.outputs]


def reference(name, raw_inputs):
    fn, n_in, _ = PROGRAMS[name]
    E = IntEngine()
    outs = fn(E, lambda n: [IntF(x) for x in raw_inputs])
    return [o.v for o in outs]


def rand_inputs(name, rng):
    """inputs for which the program's algorithm is meaningful (points on the curve, nonzero
    field elements); the check is an identity of the op list anyway"""
    _, n_in, _ = PROGRAMS[name]
    return [rng.randrange(1, P) for _ in range(n_in)]


# ----------------------------------------------------------------------------- emit
def limbs29(v):
    return [(v >> (LBITS * i)) & ((1 << LBITS) - 1) for i in range(NLIMB)]


def enc_term(sl, c):
    assert 0 <= sl < MAX_SLOTS and COEF_MIN <= c <= COEF_MAX
    return sl | ((c & 63) << SLOT_BITS)


def encode(cx, steps, slot):
    """8 words per op: w0 = dst | kind << 10 | nA << 12 | nB << 16 | input << 20; w1..w7 = 14
    16-bit terms (slot | coef << 10), the A terms at positions 0..6, the B terms at 7..13
    (unused terms are 0: slot 0 with coefficient 0).  Step descriptor: ops | max nA << 8 |
    max nB << 11 | has LIN << 14 | has MUL/LOADMUL << 15 | first op << 16."""
    kinds = {"lin": 0, "mul": 1, "loadmul": 2, "inv": 3}
    words = []
    desc = []
    for s in steps:
        assert len(s) < 256 and len(words) // 8 < 1 << 16
        na = max(len(cx.ops[o][2]) for o in s)
        nb = max(len(cx.ops[o][3]) for o in s)
        has_lin = any(cx.ops[o][0] == "lin" for o in s)
        has_mul = any(cx.ops[o][0] != "lin" for o in s)
        desc.append(len(s) | na << 8 | nb << 11 | has_lin << 14 | has_mul << 15 | (len(words) // 8) << 16)
        for o in s:
            kind, d, A, B, j = cx.ops[o]
            assert len(A) <= MAX_TERMS and len(B) <= MAX_TERMS
            ta = [enc_term(slot[v], c) for v, c in A]
            tb = [enc_term(slot[v], c) for v, c in B]
            terms = ta + [0] * (7 - len(ta)) + tb + [0] * (7 - len(tb))
            assert 0 <= j < 4096 or kind != "loadmul"
            w0 = slot[d] | kinds[kind] << 10 | len(A) << 12 | len(B) << 16 | (max(j, 0) << 20)
            words.append(w0)
            for k in range(7):
                words.append(terms[2 * k] | terms[2 * k + 1] << 16)
    desc.append(0)  # sentinel: the interpreter prefetches one step ahead
    return words, desc


def stats(cx, steps):
    nm = sum(1 for s in steps for o in s if cx.ops[o][0] != "lin")
    nl = sum(1 for s in steps for o in s if cx.ops[o][0] == "lin")
    sm = sum(1 for s in steps if any(cx.ops[o][0] != "lin" for o in s))
    cost = sum(max((W_LAT[cx.ops[o][0]] for o in s), default=0) + (0.25 if any(cx.ops[o][0] == "lin" for o in s) and
               any(cx.ops[o][0] != "lin" for o in s) else 0) for s in steps)
    return nm, nl, len(steps), sm, cost


def build(name, W):
    cx = trace(name)
    steps = schedule_loads(cx, W)
    slot, n_slots = allocate(cx, steps)
    return cx, steps, slot, n_slots


WAVES = (1, 2)  # programs are scheduled for one and for two waves per item


def emit(out_path, n_check=1, verbose=True):
    rng = random.Random(20261017)
    lines = ["// GENERATED by tools/gen_slp.py -- do not edit.",
             "// Straight-line programs of the per-group serial stages (lsg_slp.hip), each scheduled",
             "// for W = 1 and 2 waves per item (steps of <= 32 W operations): lsg_slp_<name>_w<W>.",
             "#pragma once", "#include <stdint.h>",
             "#ifndef LSG_SLP_ARRAY", "#define LSG_SLP_ARRAY static const", "#endif", ""]
    for name in PROGRAMS:
        cx = trace(name)
        for W in WAVES:
            steps = schedule_loads(cx, W)
            slot, n_slots = allocate(cx, steps)
            for _ in range(n_check):
                x = rand_inputs(name, rng)
                got = run_program(cx, steps, slot, n_slots, x)
                if cx.load_inputs == "mont":  # Montgomery in and out
                    want = reference(name, [v * RINV % P for v in x])
                    got = [v * RINV % P for v in got]
                else:
                    want = reference(name, x)
                if got != want:
                    raise SystemExit("gen_slp: program %s (W=%d) does not reproduce its algorithm" % (name, W))
            words, desc = encode(cx, steps, slot)
            nm, nl, ns, sm, cost = stats(cx, steps)
            if verbose:
                print("[gen_slp] %-14s W=%d ops %6d (mul %6d lin %5d) steps %5d (with mul %5d) cost %.0f slots %d" %
                      (name, W, nm + nl, nm, nl, ns, sm, cost, n_slots), flush=True)
            cn = "lsg_slp_%s_w%d" % (name, W)
            lines.append("// %s: %d ops (%d products), %d steps, %d LDS slots" % (cn, nm + nl, nm, ns, n_slots))
            lines.append("LSG_SLP_ARRAY uint32_t %s_ops[%d] __attribute__((aligned(32))) = {" % (cn, len(words)))
            for i in range(0, len(words), 8):
                lines.append("  " + ", ".join("0x%08xu" % w for w in words[i:i + 8]) + ",")
            lines.append("};")
            lines.append("LSG_SLP_ARRAY uint32_t %s_steps[%d] = {" % (cn, len(desc)))
            for i in range(0, len(desc), 12):
                lines.append("  " + ", ".join("0x%08xu" % w for w in desc[i:i + 12]) + ",")
            lines.append("};")
            consts = [c for _, c in cx.const_list]
            lines.append("LSG_SLP_ARRAY uint32_t %s_consts[%d] = {" % (cn, 14 * len(consts)))
            for c in consts:
                lines.append("  " + ", ".join("0x%08xu" % w for w in limbs29(c)) + ",")
            lines.append("};")
            ins = [slot[v] for v in cx.inputs] or [0]
            outs = [slot[v] for v in cx.outputs]
            lines.append("LSG_SLP_ARRAY uint16_t %s_in[%d] = {%s};" % (cn, len(ins), ", ".join(map(str, ins))))
            lines.append("LSG_SLP_ARRAY uint16_t %s_out[%d] = {%s};" % (cn, len(outs), ", ".join(map(str, outs))))
            lines.append("#define %s_N_STEPS %d" % (cn.upper(), ns))
            lines.append("#define %s_N_SLOTS %d" % (cn.upper(), n_slots))
            lines.append("#define %s_N_CONSTS %d" % (cn.upper(), len(consts)))
            lines.append("#define %s_N_IN %d" % (cn.upper(), len(cx.inputs)))
            lines.append("#define %s_N_LOAD %d" % (cn.upper(), cx.n_inputs if cx.load_inputs else 0))
            lines.append("#define %s_N_OUT %d" % (cn.upper(), len(outs)))
            lines.append("")
    tmp = out_path + ".tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, out_path)


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "lodestar_amd", "csrc",
                                                                  "lsg_slp_progs.h")
    nc = int(sys.argv[sys.argv.index("--check") + 1]) if "--check" in sys.argv else 1
    emit(out, nc)
