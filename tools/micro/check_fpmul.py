"""Checks the SAMPLE lines of tools/micro/fpmul_probe against Python big integers."""
import sys

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab


def val(hexs, limbs):
    words = [int(hexs[8 * i:8 * i + 8], 16) for i in range(limbs)][::-1]  # printed most significant first
    bits = 32 if limbs == 12 else 29
    return sum(w << (bits * k) for k, w in enumerate(words))


ok = True
for line in open(sys.argv[1]):
    if not line.startswith("SAMPLE"):
        continue
    f = line.split()
    name, limbs = f[1], int(f[2])
    ins = [val(h, limbs) for h in f[3:7]]
    outs = [val(h, limbs) for h in f[7:11]]
    rinv = pow(2, -(384 if limbs == 12 else 406), P)
    a, b, c, d = ins
    exp = [a * b * rinv % P, b * c * rinv % P, c * d * rinv % P]
    exp.append(d * exp[0] * rinv % P)
    for o, e in zip(outs, exp):
        good = (o == e) if limbs == 12 else (o % P == e and o < 2 * P)
        ok &= good
    print(name, "ok" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
