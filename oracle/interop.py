"""ORACLE (test infrastructure only) -- interop key derivation and the signing roots
needed by the genesis known-answer test.

Restates:
- packages/state-transition/src/util/interop.ts:19-22  (interop secret key i:
  sk = int_le(sha256(int_to_bytes_le(i, 32))) mod r)
- packages/state-transition/src/util/signingRoot.ts:7-13, util/domain.ts:7-31
  (compute_domain / compute_signing_root)
- packages/beacon-node/src/node/utils/interop/deposits.ts:28-44 (DepositMessage root)
"""
import hashlib

from .fields import R


def sha256(b):
    return hashlib.sha256(b).digest()


def interop_secret_key(index):
    return int.from_bytes(sha256(index.to_bytes(32, "little")), "little") % R


def _merkleize(chunks):
    n = 1
    while n < len(chunks):
        n *= 2
    layer = list(chunks) + [bytes(32)] * (n - len(chunks))
    while len(layer) > 1:
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def _pack_bytes(b):
    chunks = [b[i:i + 32] for i in range(0, len(b), 32)]
    chunks[-1] = chunks[-1] + bytes(32 - len(chunks[-1]))
    return chunks


def htr_bytes_vector(b):
    return _merkleize(_pack_bytes(b))


def htr_uint64(v):
    return v.to_bytes(8, "little") + bytes(24)


def compute_fork_data_root(current_version, genesis_validators_root):
    return _merkleize([htr_bytes_vector(current_version), genesis_validators_root])


def compute_domain(domain_type, fork_version, genesis_validators_root):
    return domain_type + compute_fork_data_root(fork_version, genesis_validators_root)[:28]


def compute_signing_root(object_root, domain):
    return _merkleize([object_root, domain])


def deposit_message_root(pubkey, withdrawal_credentials, amount):
    return _merkleize([htr_bytes_vector(pubkey), withdrawal_credentials, htr_uint64(amount)])


DOMAIN_DEPOSIT = bytes.fromhex("03000000")
# The beacon-node test suite runs under the minimal preset (test/setupPreset.ts:3-5),
# whose GENESIS_FORK_VERSION is 0x00000001 (config/src/chainConfig/presets/minimal.ts:24).
GENESIS_FORK_VERSION_MINIMAL = bytes.fromhex("00000001")
MAX_EFFECTIVE_BALANCE = 32_000_000_000

# packages/beacon-node/test/e2e/interop/genesisState.test.ts:51-55
GENESIS_KAT = {
    "pubkey": "a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c",
    "withdrawal_credentials": "00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b",
    "amount": 32000000000,
    "signature": "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446",
}


def genesis_deposit_signing_root(pubkey_bytes):
    wc = bytearray(sha256(pubkey_bytes))
    wc[0] = 0  # BLS_WITHDRAWAL_PREFIX
    domain = compute_domain(DOMAIN_DEPOSIT, GENESIS_FORK_VERSION_MINIMAL, bytes(32))
    return bytes(wc), compute_signing_root(deposit_message_root(pubkey_bytes, bytes(wc), MAX_EFFECTIVE_BALANCE), domain)


def attestation_data_root(data128):
    """ssz.phase0.AttestationData.hashTreeRoot over its 128-byte SSZ serialization (slot u64,
    index u64, beaconBlockRoot, source Checkpoint{epoch u64, root}, target Checkpoint) -- the
    objectRoot of getAttestationDataSigningRoot (state-transition/src/signatureSets/
    indexedAttestation.ts:11-19).  SURVEY.md 8f(3)."""
    assert len(data128) == 128
    d = bytes(data128)

    def u64(b):
        return b + bytes(24)

    def checkpoint(b):
        return _merkleize([u64(b[:8]), b[8:40]])
    return _merkleize([u64(d[0:8]), u64(d[8:16]), d[16:48], checkpoint(d[48:88]), checkpoint(d[88:128])])


def attestation_signing_root(data128, domain):
    return compute_signing_root(attestation_data_root(data128), domain)
