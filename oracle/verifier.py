"""ORACLE (test infrastructure only) -- verdict semantics of Lodestar's BLS verifier path.

Follows, line by line:
- packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39   verify_signature_sets_maybe_batch
- packages/beacon-node/src/chain/bls/multithread/worker.ts:30-114   verify_many_signature_sets
- packages/beacon-node/src/chain/bls/multithread/utils.ts:4-19  chunkify_maximize_chunk_size
- packages/beacon-node/src/chain/bls/utils.ts:5-26   get_aggregated_pubkey(s_count)
and, for the math below maybeBatch, the un-vendored @chainsafe/bls@7.1.1 /
@chainsafe/blst@0.2.8 / blst behaviour:
- Signature.fromBytes(bytes, affine, validate=true): size 96|192 else BLST_INVALID_SIZE,
  blst deserialization errors, then the G2 subgroup check (BLST_POINT_NOT_IN_GROUP).
- verifyMultipleSignatures: blst Pairing.mul_n_aggregate with non-zero 64-bit random
  scalars r_i; infinite signatures are skipped; infinite pubkeys -> BLST_PK_IS_INFINITY;
  verdict = FE(prod ML([r_i]PK_i, H(m_i)) * conj(ML(G1, sum r_i sig_i))) == 1.
- verify (1 set): e(PK, H(m)) == e(G1, sig), infinite sig -> false (unpinned).
Randomizers are injectable so verdicts are deterministic in tests.
"""
import os

from .fields import F12_ONE, f12_mul, f12_conj, f12_is_one
from .curves import (
    E1, E2, G1_GEN, BlstError, BLST_INVALID_SIZE, BLST_PK_IS_INFINITY, BLST_POINT_NOT_IN_GROUP,
    g1_deserialize, g2_deserialize, in_g1, in_g2, g1_serialize, g1_compress, g2_compress,
)
from .hash_to_curve import hash_to_g2
from .pairing import miller_loop_fast, final_exp_fast


class EmptySetError(Exception):
    pass


def signature_from_bytes(b, validate=True):
    if len(b) not in (96, 192):
        raise BlstError(BLST_INVALID_SIZE)
    pt = g2_deserialize(bytes(b))
    if validate and pt is not None and not in_g2(pt):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


def public_key_from_bytes(b):
    if len(b) not in (48, 96):
        raise BlstError(BLST_INVALID_SIZE)
    return g1_deserialize(bytes(b))


def public_key_validate(b):
    """PublicKey.fromBytes(bytes, CoordType.affine, validate=true) as processDeposit.ts:57-65
    calls it (KeyValidate): decode, then blst rejects the identity (BLST_PK_IS_INFINITY) and
    points outside the r-torsion subgroup (BLST_POINT_NOT_IN_GROUP).  SURVEY.md 8f(2)."""
    pt = public_key_from_bytes(b)
    if pt is None:
        raise BlstError(BLST_PK_IS_INFINITY)
    if not in_g1(pt):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


def aggregate_pubkeys(points):
    """@chainsafe/bls PublicKey.aggregate (utils.ts:11).  Empty -> EMPTY_AGGREGATE_ARRAY."""
    if len(points) == 0:
        raise ValueError("EMPTY_AGGREGATE_ARRAY")
    acc = None
    for pt in points:
        acc = E1.add(acc, pt)
    return acc


def aggregate_signatures(sigs):
    """Op-pool aggregation: bls.Signature.aggregate(sigs.map(
    signatureFromBytesNoCheck)).toBytes() -- opPools/utils.ts:32-34 decodes with validate=false
    (size/encoding/on-curve only), aggregatedAttestationPool.ts:322 and
    syncContributionAndProofPool.ts:185 sum and compress.  Empty -> EMPTY_AGGREGATE_ARRAY;
    the first undecodable signature raises its BlstError."""
    if len(sigs) == 0:
        raise ValueError("EMPTY_AGGREGATE_ARRAY")
    acc = None
    for b in sigs:
        acc = E2.add(acc, signature_from_bytes(b, validate=False))
    return g2_compress(acc)


def default_rand():
    while True:
        r = int.from_bytes(os.urandom(8), "little")
        if r:
            return r


def verify_single(pk, msg, sig):
    if pk is None:
        raise BlstError(BLST_PK_IS_INFINITY)
    if sig is None:
        return False
    f = f12_mul(miller_loop_fast(pk, hash_to_g2(msg)), f12_conj(miller_loop_fast(G1_GEN, sig)))
    return f12_is_one(final_exp_fast(f))


def verify_multiple(sets, rands=None):
    """sets: list of (pk_point, msg_bytes, sig_point).  rands: list of non-zero ints < 2^64."""
    gt = F12_ONE
    S = None
    for i, (pk, msg, sig) in enumerate(sets):
        r = rands[i] if rands is not None else default_rand()
        if sig is not None:
            S = E2.add(S, E2.mul(sig, r))
        if pk is None:
            raise BlstError(BLST_PK_IS_INFINITY)
        gt = f12_mul(gt, miller_loop_fast(E1.mul(pk, r), hash_to_g2(msg)))
    if S is not None:
        gt = f12_mul(gt, f12_conj(miller_loop_fast(G1_GEN, S)))
    return f12_is_one(final_exp_fast(gt))


def verify_signature_sets_maybe_batch(sets, rands=None):
    """maybeBatch.ts:16-39.  sets: list of dicts {publicKey: point, message: bytes, signature: bytes}."""
    if len(sets) >= 2:
        des = [(s["publicKey"], s["message"], signature_from_bytes(s["signature"], True)) for s in sets]
        return verify_multiple(des, rands)
    if len(sets) == 0:
        raise EmptySetError("Empty signature set")
    s = sets[0]
    sig = signature_from_bytes(s["signature"], True)
    return verify_single(s["publicKey"], s["message"], sig)


def chunkify_maximize_chunk_size(arr, min_per_chunk):
    """multithread/utils.ts:4-19."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i:i + per_chunk]) for i in range(0, len(arr), per_chunk)]


BATCHABLE_MIN_PER_CHUNK = 16


def verify_many_signature_sets(work_reqs, rand_fn=None):
    """multithread/worker.ts:30-106.  work_reqs: list of {"opts": {"batchable": bool},
    "sets": [{"publicKey": bytes(96|48), "message": bytes32, "signature": bytes}]}.
    Returns dict(batch_retries, batch_sigs_success, results=[("success", bool) | ("error", str)])."""
    rand_fn = rand_fn or default_rand
    results = [None] * len(work_reqs)
    batch_retries = 0
    batch_sigs_success = 0
    batchable, non_batchable = [], []
    for i, req in enumerate(work_reqs):
        sets = [{"publicKey": public_key_from_bytes(s["publicKey"]), "message": s["message"],
                 "signature": s["signature"]} for s in req["sets"]]
        (batchable if req["opts"].get("batchable") else non_batchable).append((i, sets))
    if batchable:
        for chunk in chunkify_maximize_chunk_size(batchable, BATCHABLE_MIN_PER_CHUNK):
            all_sets = [s for _, sets in chunk for s in sets]
            try:
                ok = verify_signature_sets_maybe_batch(all_sets, [rand_fn() for _ in all_sets])
                if ok:
                    for idx, sets in chunk:
                        batch_sigs_success += len(sets)
                        results[idx] = ("success", True)
                else:
                    batch_retries += 1
                    non_batchable.extend(chunk)
            except Exception:  # worker.ts:79-85 swallows batch errors
                batch_retries += 1
                non_batchable.extend(chunk)
    for idx, sets in non_batchable:
        try:
            results[idx] = ("success", verify_signature_sets_maybe_batch(sets, [rand_fn() for _ in sets]))
        except Exception as e:  # noqa: BLE001
            results[idx] = ("error", str(e))
    return {"batch_retries": batch_retries, "batch_sigs_success": batch_sigs_success, "results": results}


def sign(sk, msg):
    return E2.mul(hash_to_g2(msg), sk)


def sk_to_pk(sk):
    return E1.mul(G1_GEN, sk)


def batch_partial(sets, rands):
    """Per-shard half of verify_multiple for the node-sharded path, with the
    device's conventions (lodestar_amd/csrc/lsg_host.hip: the package group excludes such sets): sets whose signature
    does not decode (or whose key is infinite) contribute 1 and are reported by error code.
    sets: list of (pk_bytes, msg, sig_bytes).  Returns (partial Fp12, [error codes])."""
    from .curves import BlstError as _BE
    gt = F12_ONE
    S = None
    errs = []
    for (pkb, msg, sigb), r in zip(sets, rands):
        try:
            sig = signature_from_bytes(sigb, True)
            pk = public_key_from_bytes(pkb)
            if pk is None:
                raise _BE(BLST_PK_IS_INFINITY)
        except _BE as e:
            errs.append(e.code)
            continue
        errs.append(0)
        if sig is not None:
            S = E2.add(S, E2.mul(sig, r))
        gt = f12_mul(gt, miller_loop_fast(E1.mul(pk, r), hash_to_g2(msg)))
    if S is not None:
        gt = f12_mul(gt, f12_conj(miller_loop_fast(G1_GEN, S)))
    return gt, errs


def final_verify_partials(partials):
    """prod(partials) -> final exponentiation == 1 (one FE for the whole node)."""
    gt = F12_ONE
    for p in partials:
        gt = f12_mul(gt, p)
    return bool(partials) and f12_is_one(final_exp_fast(gt))
