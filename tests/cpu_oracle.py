"""ctypes access to the C restatement of the oracle (oracle/c/libbls_cpu.so; checked against
the Python oracle and the golden vectors by tests/test_oracle_c.py) for parity tests at the
BASELINE configs' sizes, where the pure-Python oracle would take minutes.  Test
infrastructure only.

Per-set expectations follow maybeBatch.ts:16-39 for one set (verify; decode errors throw) and
the job rules of worker.ts:30-106 are derived from them in ``expected_jobs``: a batchable
16-job chunk passes iff every set in it decodes and verifies; otherwise each job is
re-verified alone (an RLC batch over a job's sets has the same verdict as the AND of its
sets' single verifications up to the 2^-64 randomizer bound the reference accepts).
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "oracle", "c")
_lib = None


def lib():
    global _lib
    if _lib is None:
        so = os.path.join(CDIR, "libbls_cpu.so")
        if not os.path.exists(so):
            subprocess.check_call(["make", "-s", "-C", CDIR])
        L = ctypes.CDLL(so)
        L.cpu_verify_chunks.restype = ctypes.c_int
        L.cpu_verify_chunks.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
        L.cpu_verify_sets.restype = ctypes.c_int
        L.cpu_verify_sets.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint64]
        _lib = L
    return _lib


def threads():
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return min(int(env), 32)
    return max(1, min(len(os.sched_getaffinity(0)), 32))


def verify_each(pks96, msgs, sigs):
    """Per set: 1 valid, 0 invalid, -BLST code when the 96-byte signature (or the key) does
    not decode; a signature of another length gives -10 (BLST_INVALID_SIZE)."""
    n = len(sigs)
    fixed = [s if len(s) == 96 else bytes(96) for s in sigs]
    out = (ctypes.c_int * max(n, 1))()
    lib().cpu_verify_chunks(b"".join(pks96), b"".join(msgs), b"".join(fixed), n, 1, threads(), 0x5EED, out)
    res = list(out[:n])
    for i, s in enumerate(sigs):
        if len(s) != 96:
            res[i] = -10
    return res


def expected_jobs(jobs_sets, batchable, per_set):
    """worker.ts:30-106 from per-set outcomes.  jobs_sets: per job the list of its set indices;
    batchable: per job flag; per_set: verify_each output.  Returns (per-job (status, code),
    batch_retries, batch_sigs_success) with status 1 valid, 0 invalid, 2 error."""
    def job_result(idx):
        if not idx:
            return (2, 100)
        for i in idx:
            if per_set[i] < 0:
                return (2, -per_set[i])
        return (1 if all(per_set[i] == 1 for i in idx) else 0, 0)

    res = [None] * len(jobs_sets)
    retries = success = 0
    bj = [j for j in range(len(jobs_sets)) if batchable[j]]
    count = len(bj) // 16
    if count <= 1:
        chunks = [bj] if bj else []
    else:
        per = -(-len(bj) // count)
        chunks = [bj[i:i + per] for i in range(0, len(bj), per)]
    for ch in chunks:
        sets = [i for j in ch for i in jobs_sets[j]]
        if sets and all(per_set[i] == 1 for i in sets):
            success += len(sets)
            for j in ch:
                res[j] = (1, 0)
        else:
            retries += 1
            for j in ch:
                res[j] = job_result(jobs_sets[j])
    for j in range(len(jobs_sets)):
        if not batchable[j]:
            res[j] = job_result(jobs_sets[j])
    return res, retries, success
