"""Generates the committed golden fixtures from the oracle (whose hash_to_G2, keygen,
serialization and signing are pinned by the reference's genesis KAT,
packages/beacon-node/test/e2e/interop/genesisState.test.ts:49-56).

  hash_to_g2.json         msg -> uncompressed H(msg) with the POP DST
  sig_decode.json         96/192/other-byte signatures -> point or blst error code
  aggregate_pubkeys.json  pubkey lists -> uncompressed aggregate or error
  verdict_jobs.json       work packages -> per-job verdicts (worker.ts semantics)
  aggregate_signatures.json  op-pool signature lists -> compressed aggregate or error (8f(4))

Run: python tests/golden/gen_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.curves import (  # noqa: E402
    E1, E2, g1_serialize, g1_compress, g2_serialize, g2_compress, g2_uncompress, g2_deserialize, in_g2, BlstError,
    BLST_INVALID_SIZE, BLST_POINT_NOT_IN_GROUP,
)
from oracle.fields import P  # noqa: E402
from oracle import hash_to_curve as h2c  # noqa: E402
from oracle import verifier as ov  # noqa: E402
from tests import blsdata as bd  # noqa: E402


def sig_case(b):
    try:
        pt = ov.signature_from_bytes(b, True)
        return {"sig": b.hex(), "err": 0, "point": g2_serialize(pt).hex()}
    except BlstError as e:
        return {"sig": b.hex(), "err": e.code}


def main():
    rng = random.Random(2024)
    # hash_to_g2
    msgs = [b"", b"abc", bytes(32), bytes([0xFF]) * 32] + [bd.msg("golden", i) for i in range(12)]
    h = {"dst": h2c.DST_POP.decode(), "cases": [{"msg": m.hex(), "out": g2_serialize(h2c.hash_to_g2(m)).hex()}
                                                 for m in msgs if len(m) == 32]}
    json.dump(h, open(os.path.join(HERE, "hash_to_g2.json"), "w"), indent=1)

    # signature decoding
    cases = []
    mainnet = json.load(open(os.path.join(HERE, "mainnet_g2_points.json")))
    for hx in mainnet:
        cases.append(sig_case(bytes.fromhex(hx)))
    base = bd.single_set(0)[2]
    cases.append(sig_case(base))
    cases.append(sig_case(bytes([0xC0]) + bytes(95)))            # infinity
    cases.append(sig_case(bytes([0xE0]) + bytes(95)))            # infinity + sign bit -> bad encoding
    cases.append(sig_case(bytes([0xC0]) + bytes(94) + b"\x01"))  # infinity with junk
    cases.append(sig_case(bytes([base[0] & 0x7F]) + base[1:]))  # compression bit cleared
    pbytes = bytearray((P).to_bytes(48, "big") + bytes(48))      # x.c1 = p  -> bad encoding
    pbytes[0] |= 0x80
    cases.append(sig_case(bytes(pbytes)))
    for i in range(40):                                          # random x: off-curve / not in group
        x0 = rng.randrange(P)
        x1 = rng.randrange(P)
        b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
        b[0] |= 0x80 | (0x20 if i & 1 else 0)
        cases.append(sig_case(bytes(b)))
    for i in range(4):
        cases.append(sig_case(bd.corrupt_flip_x_bit(bd.single_set(i), bit=i)[2]))
        cases.append(sig_case(bd.corrupt_not_in_group(bd.single_set(i), seed=i)[2]))
    for i in range(3):                                           # uncompressed 192-byte encodings
        pt = g2_uncompress(bd.single_set(i)[2])
        cases.append(sig_case(g2_serialize(pt)))
    cases.append(sig_case(bytes([0x40]) + bytes(191)))
    json.dump({"cases": cases}, open(os.path.join(HERE, "sig_decode.json"), "w"), indent=1)

    # pubkey aggregation
    agg = []
    for n in (1, 2, 3, 17, 64, 512):
        keys = [rng.randrange(1024) for _ in range(n)]
        pks = [bd.pk_bytes(k) for k in keys]
        s = ov.aggregate_pubkeys([bd.pk_point(k) for k in keys])
        agg.append({"pks": [p.hex() for p in pks], "err": 0, "out": g1_serialize(s).hex()})
    keys = [3, 5, 9]
    agg.append({"pks": [bd.pk_bytes(k, compressed=True).hex() for k in keys], "err": 0,
                "out": g1_serialize(ov.aggregate_pubkeys([bd.pk_point(k) for k in keys])).hex()})
    pk = bd.pk_point(7)
    neg = g1_serialize(E1.neg(pk))
    agg.append({"pks": [g1_serialize(pk).hex(), neg.hex()], "err": 0, "out": g1_serialize(None).hex()})
    bad = bytearray(g1_serialize(pk))
    bad[95] ^= 1
    agg.append({"pks": [g1_serialize(pk).hex(), bytes(bad).hex()], "err": 2})
    json.dump({"cases": agg}, open(os.path.join(HERE, "aggregate_pubkeys.json"), "w"), indent=1)

    # op-pool signature aggregation (Signature.aggregate of signatureFromBytesNoCheck)
    json.dump({"cases": aggregate_signature_cases(rng, mainnet)},
              open(os.path.join(HERE, "aggregate_signatures.json"), "w"), indent=1)


def sig_agg_case(sigs):
    try:
        return {"sigs": [b.hex() for b in sigs], "err": 0, "out": ov.aggregate_signatures(sigs).hex()}
    except BlstError as e:
        return {"sigs": [b.hex() for b in sigs], "err": e.code}


def aggregate_signature_cases(rng, mainnet):
    cases = []
    sigs = [bd.single_set(i)[2] for i in range(128)]
    for n in (1, 2, 3, 16, 128):                                  # committee-shaped aggregates
        cases.append(sig_agg_case(sigs[:n]))
    real = []
    for hx in mainnet:                                            # the reference's mainnet G2 points
        b = bytes.fromhex(hx)
        try:
            ov.signature_from_bytes(b, False)
            real.append(b)
        except BlstError:
            pass
    cases.append(sig_agg_case(real))
    inf = bytes([0xC0]) + bytes(95)
    cases.append(sig_agg_case([sigs[0], inf, sigs[1]]))          # infinity contributes nothing
    cases.append(sig_agg_case([inf]))
    pt = g2_uncompress(sigs[5])
    cases.append(sig_agg_case([sigs[5], g2_compress(E2.neg(pt))]))  # P + (-P) = identity
    cases.append(sig_agg_case([sigs[2], sigs[2]]))                # doubling inside the tree
    cases.append(sig_agg_case([sigs[3], bd.corrupt_not_in_group(bd.single_set(3), seed=3)[2]]))  # no subgroup check
    cases.append(sig_agg_case([sigs[4], bd.corrupt_flip_x_bit(bd.single_set(4), bit=4)[2], sigs[6]]))
    cases.append(sig_agg_case([sigs[7], bytes([0xE0]) + bytes(95)]))  # bad encoding
    cases.append(sig_agg_case([g2_serialize(g2_uncompress(s)) for s in sigs[:5]]))  # 192-byte inputs
    rng.shuffle(cases)
    return cases


if __name__ == "__main__":
    main()
