"""lodestar_amd -- MI355X-native BLS12-381 signature-set verifier behind Lodestar's IBlsVerifier.

Host mirror of packages/beacon-node/src/chain/bls/ over the C ABI in include/lodestar_bls.h,
whose HIP kernels (lodestar_amd/csrc/) run on gfx950.
"""
__version__ = "0.1.0"
