"""The C restatement of the oracle (oracle/c/bls_cpu.c: bench.py's multi-threaded CPU
baseline) against the Python oracle and the committed golden vectors.

It must agree with the oracle before its timing means anything: hash_to_G2 outputs
(tests/golden/hash_to_g2.json, pinned by the genesis KAT of
packages/beacon-node/test/e2e/interop/genesisState.test.ts:49-56), signature decoding and
error codes for 96-byte compressed encodings (tests/golden/sig_decode.json), and
maybeBatch verdicts (packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39) on valid and
corrupted sets.
"""
import ctypes
import json
import os
import subprocess

import pytest

from tests import blsdata as bd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "oracle", "c")
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def lib():
    subprocess.check_call(["make", "-s", "-C", CDIR])
    L = ctypes.CDLL(os.path.join(CDIR, "libbls_cpu.so"))
    L.cpu_verify_sets.restype = ctypes.c_int
    L.cpu_verify_sets.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint64]
    L.cpu_verify_chunks.restype = ctypes.c_int
    L.cpu_verify_chunks.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
    L.cpu_sig_decode.restype = ctypes.c_int
    L.cpu_sig_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    L.cpu_hash_to_g2.restype = None
    L.cpu_hash_to_g2.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                 ctypes.c_char_p]
    return L


def test_hash_to_g2_golden(lib):
    g = json.load(open(os.path.join(GOLDEN, "hash_to_g2.json")))
    dst = g["dst"].encode()
    for c in g["cases"]:
        m = bytes.fromhex(c["msg"])
        out = ctypes.create_string_buffer(192)
        lib.cpu_hash_to_g2(m, len(m), dst, len(dst), out)
        assert out.raw.hex() == c["out"], c["msg"]


def test_sig_decode_golden(lib):
    g = json.load(open(os.path.join(GOLDEN, "sig_decode.json")))
    n = 0
    for c in g["cases"]:
        b = bytes.fromhex(c["sig"])
        if len(b) != 96:  # the baseline takes compressed signatures only (the workload's form)
            continue
        out = ctypes.create_string_buffer(192)
        err = lib.cpu_sig_decode(b, len(b), out)
        assert err == c["err"], c["sig"]
        if err == 0:
            assert out.raw.hex() == c["point"], c["sig"]
        n += 1
    assert n >= 50


def _pack(sets):
    return (b"".join(s[0][0] for s in sets), b"".join(s[1] for s in sets), b"".join(s[2] for s in sets))


@pytest.mark.parametrize("n", [1, 2, 5])
def test_verdicts_match_oracle(lib, n):
    sets = [bd.single_set(i, tag="oc") for i in range(n)]
    assert lib.cpu_verify_sets(*_pack(sets), n, 7) == 1
    bad = list(sets)
    bad[n // 2] = bd.corrupt_wrong_message(bad[n // 2])
    assert lib.cpu_verify_sets(*_pack(bad), n, 7) == 0
    inf = list(sets)
    inf[0] = bd.corrupt_infinity(inf[0])
    assert lib.cpu_verify_sets(*_pack(inf), n, 7) == 0  # infinite signature skipped -> false (M10)
    nig = list(sets)
    nig[-1] = bd.corrupt_not_in_group(nig[-1])
    assert lib.cpu_verify_sets(*_pack(nig), n, 7) == -3  # BLST_POINT_NOT_IN_GROUP


@pytest.mark.parametrize("chunk", [8, 16])
def test_threaded_chunks(lib, chunk):
    """worker.ts:17,54 batches of 16 sets (17 Miller pairs with the signature term)."""
    sets = [bd.single_set(i, tag="oc") for i in range(2 * chunk + 4)]
    sets[chunk + 5] = bd.corrupt_wrong_message(sets[chunk + 5])
    pk, m, s = _pack(sets)
    verdicts = (ctypes.c_int * 3)()
    ok = lib.cpu_verify_chunks(pk, m, s, len(sets), chunk, 3, 99, verdicts)
    assert list(verdicts) == [1, 0, 1] and ok == 2
