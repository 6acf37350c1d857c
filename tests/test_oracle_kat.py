"""Pins the CPU oracle against the reference's own known answers.

- packages/beacon-node/test/e2e/interop/genesisState.test.ts:49-56 (genesis deposit KAT:
  interop sk #0 -> pubkey, withdrawal credentials, deposit signature under the minimal
  preset's GENESIS_FORK_VERSION) -- pins keygen, G1/G2 compression, hash_to_G2 with the
  POP DST and G2 scalar multiplication bit-exactly.
- packages/beacon-node/test/unit/chain/bls/utils.test.ts:7-25 (chunkify outputs).
- real mainnet G2 points held in the reference's fixtures
  (packages/beacon-node/test/unit/sync/backfill/blocks.json: block signatures and randao
  reveals) must decompress and pass the G2 subgroup check.
"""
import json
import os

import pytest

from oracle.curves import (
    E1, E2, G1_GEN, G2_GEN, g1_compress, g2_compress, g2_uncompress, in_g2, in_g2_psi, psi, BlstError,
)
from oracle.fields import R, X
from oracle.interop import GENESIS_KAT, interop_secret_key, genesis_deposit_signing_root
from oracle import hash_to_curve as h2c
from oracle.verifier import sign, sk_to_pk, verify_signature_sets_maybe_batch, chunkify_maximize_chunk_size

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_genesis_pubkey():
    sk = interop_secret_key(0)
    assert g1_compress(sk_to_pk(sk)).hex() == GENESIS_KAT["pubkey"]


def test_genesis_withdrawal_credentials_and_signature():
    sk = interop_secret_key(0)
    pk = g1_compress(sk_to_pk(sk))
    wc, root = genesis_deposit_signing_root(pk)
    assert wc.hex() == GENESIS_KAT["withdrawal_credentials"]
    sig = g2_compress(sign(sk, root))
    assert sig.hex() == GENESIS_KAT["signature"]


def test_genesis_signature_verifies_and_tamper_fails():
    sk = interop_secret_key(0)
    pk = sk_to_pk(sk)
    _, root = genesis_deposit_signing_root(g1_compress(pk))
    sig = bytes.fromhex(GENESIS_KAT["signature"])
    assert verify_signature_sets_maybe_batch([{"publicKey": pk, "message": root, "signature": sig}])
    bad_root = bytes([root[0] ^ 1]) + root[1:]
    assert not verify_signature_sets_maybe_batch([{"publicKey": pk, "message": bad_root, "signature": sig}])


def test_iso3_derivation_selects_committed_constants():
    from oracle.iso3_derive import derive_iso3_candidates
    cands = derive_iso3_candidates()
    assert h2c.ISO3 in cands
    # Exactly one candidate reproduces the KAT signature
    sk = interop_secret_key(0)
    _, root = genesis_deposit_signing_root(g1_compress(sk_to_pk(sk)))
    u0, u1 = h2c.hash_to_field_fp2(root, h2c.DST_POP)
    hits = 0
    for c in cands:
        def m(u):
            x, y = h2c.map_to_curve_sswu(u)
            xn, xd, yn, yd = c
            ev = h2c._peval
            from oracle.fields import f2_mul, f2_inv
            return (f2_mul(ev(xn, x), f2_inv(ev(xd, x))), f2_mul(y, f2_mul(ev(yn, x), f2_inv(ev(yd, x)))))
        Hm = h2c.clear_cofactor(E2.add(m(u0), m(u1)))
        if g2_compress(E2.mul(Hm, sk)).hex() == GENESIS_KAT["signature"]:
            hits += 1
            assert c == h2c.ISO3
    assert hits == 1


def test_h_eff_matches_psi_form():
    u0, u1 = h2c.hash_to_field_fp2(b"lodestar", h2c.DST_POP)
    Q = E2.add(h2c.map_to_curve_g2(u0), h2c.map_to_curve_g2(u1))
    assert not in_g2(Q)
    Hq = h2c.clear_cofactor(Q)
    assert E2.eq(Hq, E2.mul(Q, h2c.H_EFF_G2))
    assert in_g2(Hq) and in_g2_psi(Hq) and not in_g2_psi(Q)


def test_chunkify_reference_cases():
    # packages/beacon-node/test/unit/chain/bls/utils.test.ts:7-25
    expected = [
        [[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
        [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]],
    ]
    for i, exp in enumerate(expected):
        assert chunkify_maximize_chunk_size(list(range(i + 1)), 3) == exp


def test_mainnet_block_signatures_are_g2_points():
    path = os.path.join(GOLDEN, "mainnet_g2_points.json")
    pts = json.load(open(path))
    assert len(pts) >= 8
    for hx in pts:
        Pt = g2_uncompress(bytes.fromhex(hx))
        assert in_g2_psi(Pt)
        assert g2_compress(Pt).hex() == hx


def test_aggregate_signatures_oracle_and_golden():
    """Op-pool aggregation: the golden fixture is the oracle's output, and
    the oracle is pinned by a property independent of it: the aggregate of sk_i-signatures
    over one message is the signature of sum(sk_i) (BLS linearity), as the sync-committee
    contribution pool relies on (syncContributionAndProofPool.ts:169-186)."""
    from oracle.curves import g2_compress
    from oracle.verifier import aggregate_signatures
    from tests import blsdata as bd
    m = bd.msg("oppool", 0)
    keys = [interop_secret_key(i) for i in range(5)]
    sigs = [g2_compress(sign(k, m)) for k in keys]
    assert aggregate_signatures(sigs) == g2_compress(sign(sum(keys) % R, m))
    with pytest.raises(ValueError, match="EMPTY_AGGREGATE_ARRAY"):
        aggregate_signatures([])
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "aggregate_signatures.json")))
    for c in gold["cases"]:
        sg = [bytes.fromhex(x) for x in c["sigs"]]
        if c["err"]:
            with pytest.raises(BlstError) as e:
                aggregate_signatures(sg)
            assert e.value.code == c["err"]
        else:
            assert aggregate_signatures(sg).hex() == c["out"]


def test_attestation_signing_root_oracle():
    """AttestationData.hashTreeRoot restated against the tree written out
    node by node; SigningData is the helper the genesis KAT pins."""
    import hashlib
    from oracle import interop as oi
    h = lambda a, b: hashlib.sha256(a + b).digest()  # noqa: E731
    d = bytes(range(128))
    dom = bytes(range(100, 132))
    u = lambda b: b + bytes(24)  # noqa: E731
    z = bytes(32)
    src, tgt = h(u(d[48:56]), d[56:88]), h(u(d[88:96]), d[96:128])
    root = h(h(h(u(d[0:8]), u(d[8:16])), h(d[16:48], src)), h(h(tgt, z), h(z, z)))
    assert oi.attestation_data_root(d) == root
    assert oi.attestation_signing_root(d, dom) == h(root, dom)
