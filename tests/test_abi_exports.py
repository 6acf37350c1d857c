"""The C-ABI library loads without a GPU and exports every entry point that
include/lodestar_bls.h declares (no compute calls: those need an MI355X)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "lodestar_bls.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(lsg_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("lsg_init", "lsg_submit_jobs", "lsg_wait_jobs", "lsg_verify_jobs", "lsg_aggregate_pubkeys",
              "lsg_hash_to_g2", "lsg_sig_decode", "lsg_final_submit", "lsg_init_devices", "lsg_reserve",
              "lsg_jobs_partial", "lsg_wait_jobs_node", "lsg_assign_jobs"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from lodestar_amd import _native
    lib = _native.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert set(declared_symbols()) == set(_native.EXPORTS)


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    from lodestar_amd import _native
    lib = _native.load_library()
    h = ctypes.c_void_p()
    assert lib.lsg_init(0, ctypes.byref(h)) == _native.LSG_ERR_NO_DEVICE
    try:
        _native.Context(0)
    except _native.NativeUnavailable:
        pass
    else:
        raise AssertionError("Context() must raise without a gfx950 device")


def test_assign_jobs_matches_the_host_rule():
    """lsg_assign_jobs (the whole-job split of lsg_init_devices, host code, no GPU) equals the
    rule of lodestar_amd.sharded.assign_jobs on ragged and empty inputs."""
    import random
    from lodestar_amd import _native
    from lodestar_amd.sharded import assign_jobs
    rng = random.Random(3)
    cases = [[], [0], [1], [5, 0, 0, 7], [1] * 33, [128] * 9 + [1] * 40]
    cases += [[rng.choice([0, 1, 1, 2, 3, 128]) for _ in range(rng.randrange(1, 300))] for _ in range(50)]
    for sizes in cases:
        for n in (1, 2, 3, 8):
            got = _native.assign_jobs(sizes, n)
            assert got == assign_jobs(sizes, n), (sizes, n)
            assert got == sorted(got) and all(0 <= g < n for g in got)
