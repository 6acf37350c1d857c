"""ORACLE -- test infrastructure only.

A pure-Python (big int + hashlib) CPU restatement of the BLS12-381 signature-set
verification path under Lodestar's IBlsVerifier (packages/beacon-node/src/chain/bls/).
It is the *checker* for the HIP implementation in lodestar_amd/: only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.  The product
path never imports, calls or links anything under oracle/.

Parity pin: the genesis known-answer test (packages/beacon-node/test/e2e/interop/
genesisState.test.ts:49-56: interop sk #0 -> pubkey, deposit signature) pins keygen,
G1/G2 serialization, hash_to_G2 with the POP DST and G2 scalar multiplication
bit-exactly; see tests/test_oracle_kat.py.  The arithmetic's reference
implementation (@chainsafe/blst@0.2.8 -> supranational blst) is un-vendored and
absent from this container, so edge-case error precedence is restated from blst's
published behaviour and is marked "unpinned" where no in-tree fixture covers it.
"""
