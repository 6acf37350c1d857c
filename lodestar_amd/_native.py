"""ctypes binding of the C ABI in include/lodestar_bls.h (lodestar_amd/liblodestar_bls.so).

The library is built in-tree by ``lodestar_amd.build`` (hipcc --offload-arch=gfx950).
There is no fallback: if the library or a gfx950 device is missing, every entry point
raises ``NativeUnavailable``.
"""
import ctypes
import os
import struct
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSG_LIB", os.path.join(HERE, "liblodestar_bls.so"))  # LSG_LIB: A/B builds
# the A/B and test build (lodestar_amd/build.py build_ab, csrc/lsg_ab.h): the same C ABI with
# the stage switches read from the environment -- tests that compare two forms of a stage
AB_LIB_PATH = os.path.join(HERE, "liblodestar_bls_ab.so")

LSG_OK = 0
LSG_ERR_NO_DEVICE = 2
LSG_ERR_BUSY = 6
LSG_ERR_ENTROPY = 7

LSG_INVALID = 0
LSG_VALID = 1
LSG_ERROR = 2

LSG_JOB_BATCHABLE = 1
LSG_JOB_PRIORITY = 2

BLST_NAMES = {
    0: "BLST_SUCCESS", 1: "BLST_BAD_ENCODING", 2: "BLST_POINT_NOT_ON_CURVE", 3: "BLST_POINT_NOT_IN_GROUP",
    4: "BLST_AGGR_TYPE_MISMATCH", 5: "BLST_VERIFY_FAIL", 6: "BLST_PK_IS_INFINITY", 7: "BLST_BAD_SCALAR",
    10: "BLST_INVALID_SIZE",
}
LSG_ERR_EMPTY_SET = 100
LSG_ERR_EMPTY_AGGREGATE = 101
LSG_ERR_BAD_INDEX = 102
LSG_PK_INDEX = 4  # lsg_set.pk_len for keys named by pubkey-table index


def error_message(code):
    """Error text in the form the reference's callers match on: the BLST code name is a
    substring (multithread.test.ts:97 'BLST_INVALID_SIZE'; spec harness 'BLST_ERROR')."""
    if code == LSG_ERR_EMPTY_SET:
        return "Empty signature set"
    if code == LSG_ERR_EMPTY_AGGREGATE:
        return "EMPTY_AGGREGATE_ARRAY"
    if code == LSG_ERR_BAD_INDEX:
        return "Unknown pubkey index"
    return "BLST_ERROR: " + BLST_NAMES.get(code, f"BLST_UNKNOWN_{code}")


class NativeUnavailable(RuntimeError):
    pass


class PkIndices(list):
    """A set's pubkeys given as validator indices into the context's pubkey table
    (Context.pubkey_table_set; lsg_set.pk_len = LSG_PK_INDEX) instead of encoded bytes."""

    def tobytes(self):
        import array
        a = array.array("I", self)
        assert a.itemsize == 4
        return a.tobytes()


class LsgSet(ctypes.Structure):
    _fields_ = [
        ("pks", ctypes.c_void_p), ("pk_len", ctypes.c_uint32), ("n_pks", ctypes.c_uint32),
        ("msg", ctypes.c_void_p), ("msg_len", ctypes.c_uint32),
        ("sig", ctypes.c_void_p), ("sig_len", ctypes.c_uint32),
    ]


class LsgJob(ctypes.Structure):
    _fields_ = [("sets", ctypes.POINTER(LsgSet)), ("n_sets", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class LsgJobResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("err_code", ctypes.c_int32)]


class LsgStats(ctypes.Structure):
    _fields_ = [
        ("batch_retries", ctypes.c_uint32), ("batch_sigs_success", ctypes.c_uint32),
        ("start_ns", ctypes.c_uint64), ("end_ns", ctypes.c_uint64),
        ("n_final_exps", ctypes.c_uint32), ("submit_us", ctypes.c_uint32),
        ("key_error", ctypes.c_int32), ("key_error_job", ctypes.c_uint32),
    ]


_lib = None
_lib_lock = threading.Lock()

EXPORTS = [
    "lsg_init", "lsg_init_devices", "lsg_destroy", "lsg_device_count", "lsg_last_error", "lsg_device_name",
    "lsg_reserve", "lsg_allocation_count", "lsg_verify_jobs", "lsg_verify_sets",
    "lsg_aggregate_pubkeys", "lsg_hash_to_g2", "lsg_sig_decode", "lsg_batch_partial", "lsg_final_verify",
    "lsg_probe_fp_mul_rate", "lsg_last_kernel_times", "lsg_sign", "lsg_sk_to_pk",
    "lsg_submit_jobs", "lsg_wait_jobs", "lsg_wait_jobs_node", "lsg_jobs_partial", "lsg_assign_jobs", "lsg_poll",
    "lsg_final_submit", "lsg_final_wait", "lsg_pipeline_slots", "lsg_probe_mad_peak",
    "lsg_pubkey_table_set", "lsg_pubkey_table_size", "lsg_pubkey_validate",
    "lsg_final_submit_groups", "lsg_final_wait_groups", "lsg_aggregate_signatures",
    "lsg_signing_roots", "lsg_attestation_signing_roots", "lsg_jobs_partial_device", "lsg_final_submit_device",
    "lsg_set_coalesce", "lsg_aggregate_pubkeys_multi", "lsg_check_fp2_mul",
]


def load_library(path=LIB_PATH):
    """Load the shared library and declare prototypes (works without a GPU)."""
    global _lib
    with _lib_lock:
        if _lib is not None and path == LIB_PATH:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(f"{path} not built (run python -c 'import __graft_entry__; __graft_entry__.build()')")
        lib = ctypes.CDLL(path)
        vp, u32, u64, i32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_size_t
        pi32 = ctypes.POINTER(ctypes.c_int32)
        lib.lsg_init.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        lib.lsg_init_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(vp)]
        lib.lsg_device_count.argtypes = [vp, pi32]
        lib.lsg_reserve.argtypes = [vp, sz, sz, sz, i32]
        lib.lsg_allocation_count.argtypes = [vp, ctypes.POINTER(u64)]
        lib.lsg_wait_jobs_node.argtypes = [vp, u64, i32, ctypes.POINTER(LsgJobResult), ctypes.POINTER(LsgStats)]
        lib.lsg_jobs_partial.argtypes = [vp, u64, ctypes.c_char_p, pi32]
        lib.lsg_jobs_partial_device.argtypes = [vp, u64, vp, pi32]
        lib.lsg_final_submit_device.argtypes = [vp, vp, sz, ctypes.POINTER(u64)]
        lib.lsg_assign_jobs.argtypes = [ctypes.POINTER(u32), sz, i32, pi32]
        lib.lsg_destroy.argtypes = [vp]
        lib.lsg_last_error.argtypes = [vp]
        lib.lsg_last_error.restype = ctypes.c_char_p
        lib.lsg_device_name.argtypes = [vp, ctypes.c_char_p, sz]
        lib.lsg_verify_jobs.argtypes = [vp, ctypes.POINTER(LsgJob), sz, u64, ctypes.POINTER(LsgJobResult),
                                        ctypes.POINTER(LsgStats)]
        lib.lsg_verify_sets.argtypes = [vp, ctypes.POINTER(LsgSet), sz, u64, ctypes.POINTER(LsgJobResult)]
        lib.lsg_aggregate_pubkeys.argtypes = [vp, ctypes.c_char_p, u32, sz, ctypes.c_char_p, pi32]
        lib.lsg_aggregate_pubkeys_multi.argtypes = [vp, ctypes.POINTER(LsgSet), sz, ctypes.c_char_p, pi32]
        lib.lsg_hash_to_g2.argtypes = [vp, ctypes.c_char_p, u32, sz, ctypes.c_char_p, u32, ctypes.c_char_p]
        lib.lsg_sig_decode.argtypes = [vp, ctypes.c_char_p, u32, sz, ctypes.c_char_p, pi32]
        lib.lsg_batch_partial.argtypes = [vp, ctypes.POINTER(LsgSet), sz, u64, ctypes.c_char_p, pi32, pi32]
        lib.lsg_final_verify.argtypes = [vp, ctypes.c_char_p, sz, pi32]
        lib.lsg_probe_fp_mul_rate.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        lib.lsg_last_kernel_times.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                              ctypes.c_int]
        lib.lsg_sign.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, u32, sz, ctypes.c_char_p]
        lib.lsg_sk_to_pk.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p]
        pu64 = ctypes.POINTER(u64)
        lib.lsg_submit_jobs.argtypes = [vp, ctypes.POINTER(LsgJob), sz, u64, pu64]
        lib.lsg_wait_jobs.argtypes = [vp, u64, ctypes.POINTER(LsgJobResult), ctypes.POINTER(LsgStats)]
        lib.lsg_poll.argtypes = [vp, u64, pi32]
        lib.lsg_pubkey_table_set.argtypes = [vp, sz, ctypes.c_char_p, u32, sz, pi32]
        lib.lsg_pubkey_table_size.argtypes = [vp, ctypes.POINTER(sz)]
        lib.lsg_final_submit_groups.argtypes = [vp, ctypes.c_char_p, sz, sz, pu64]
        lib.lsg_final_wait_groups.argtypes = [vp, u64, pi32]
        lib.lsg_pubkey_validate.argtypes = [vp, ctypes.c_char_p, u32, sz, ctypes.c_char_p, pi32]
        lib.lsg_signing_roots.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, u32, ctypes.c_char_p]
        lib.lsg_attestation_signing_roots.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, u32, ctypes.c_char_p]
        lib.lsg_aggregate_signatures.argtypes = [vp, ctypes.c_char_p, u32, ctypes.POINTER(u32), sz,
                                                 ctypes.c_char_p, pi32]
        lib.lsg_final_submit.argtypes = [vp, ctypes.c_char_p, sz, pu64]
        lib.lsg_final_wait.argtypes = [vp, u64, pi32]
        lib.lsg_pipeline_slots.argtypes = [vp, pi32]
        lib.lsg_set_coalesce.argtypes = [vp, u32, i32]
        lib.lsg_check_fp2_mul.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p]
        lib.lsg_probe_mad_peak.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        for name in EXPORTS:
            if name != "lsg_last_error":
                getattr(lib, name).restype = ctypes.c_int
        if path == LIB_PATH:
            _lib = lib
        return lib


class SetBuffer:
    """Keeps the bytes of a list of sets alive while the C call runs."""

    def __init__(self, sets):
        # sets: iterable of (pks: list[bytes], msg: bytes, sig: bytes)
        self._keep = []
        sets = list(sets)
        self.arr = (LsgSet * max(len(sets), 1))()
        for i, (pks, msg, sig) in enumerate(sets):
            if isinstance(pks, PkIndices):
                pk_len, pkb = LSG_PK_INDEX, pks.tobytes()
            else:
                pk_len = len(pks[0]) if pks else 96
                if any(len(p) != pk_len for p in pks):
                    raise ValueError("all pubkeys of one set must share one encoding length")
                pkb = b"".join(pks)
            for b in (pkb, msg, sig):
                self._keep.append(b)
            s = self.arr[i]
            s.pks = ctypes.cast(ctypes.c_char_p(pkb), ctypes.c_void_p) if pkb else None
            s.pk_len = pk_len
            s.n_pks = len(pks)
            s.msg = ctypes.cast(ctypes.c_char_p(msg), ctypes.c_void_p) if msg else None
            s.msg_len = len(msg)
            s.sig = ctypes.cast(ctypes.c_char_p(sig), ctypes.c_void_p) if sig else None
            s.sig_len = len(sig)
        self.n = len(sets)


def assign_jobs(job_sizes, n_devices):
    """lsg_assign_jobs (host only): the device of every job for lsg_init_devices."""
    lib = load_library()
    n = len(job_sizes)
    sizes = (ctypes.c_uint32 * max(n, 1))(*job_sizes)
    owner = (ctypes.c_int32 * max(n, 1))()
    rc = lib.lsg_assign_jobs(sizes, n, int(n_devices), owner)
    if rc != LSG_OK:
        raise ValueError(f"lsg_assign_jobs failed ({rc})")
    return list(owner[:n])


class PreparedJobs:
    """A package of jobs laid out once as lsg_job / lsg_set arrays (numpy-filled), so that it
    can be submitted repeatedly without per-set Python work: every lsg_submit_jobs still copies
    all its bytes from host memory and draws fresh randomizers.  jobs: list of (sets, flags),
    sets = list of (pks, msg, sig) as for Context.verify_jobs."""

    def __init__(self, jobs):
        import numpy as np
        flat = [st for sets, _ in jobs for st in sets]
        n = len(flat)
        pk_parts, pk_len, n_pks = [], np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint32)
        for i, (pks, _m, _s) in enumerate(flat):
            if isinstance(pks, PkIndices):
                pk_len[i], b = LSG_PK_INDEX, pks.tobytes()
            else:
                pk_len[i] = len(pks[0]) if pks else 96
                if any(len(p) != pk_len[i] for p in pks):
                    raise ValueError("all pubkeys of one set must share one encoding length")
                b = b"".join(pks)
            n_pks[i] = len(pks)
            pk_parts.append(b)

        def pack(parts):
            lens = np.array([len(p) for p in parts] or [0], np.uint64)
            offs = np.zeros_like(lens)
            if len(parts) > 1:
                offs[1:] = np.cumsum(lens)[:-1]
            buf = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8).copy()
            return buf, offs, lens

        self._pk, pk_off, _ = pack(pk_parts)
        self._msg, msg_off, msg_len = pack([m for _, m, _ in flat])
        self._sig, sig_off, sig_len = pack([s for _, _, s in flat])
        self.sets = (LsgSet * max(n, 1))()
        dt = np.dtype({"names": ["pks", "pk_len", "n_pks", "msg", "msg_len", "sig", "sig_len"],
                       "formats": [np.uint64, np.uint32, np.uint32, np.uint64, np.uint32, np.uint64, np.uint32],
                       "offsets": [LsgSet.pks.offset, LsgSet.pk_len.offset, LsgSet.n_pks.offset, LsgSet.msg.offset,
                                   LsgSet.msg_len.offset, LsgSet.sig.offset, LsgSet.sig_len.offset],
                       "itemsize": ctypes.sizeof(LsgSet)})
        v = np.frombuffer(self.sets, dtype=dt)
        if n:
            v["pks"][:n] = np.where(n_pks[:n] > 0, self._pk.ctypes.data + pk_off[:n], 0)
            v["pk_len"][:n] = pk_len[:n]
            v["n_pks"][:n] = n_pks[:n]
            v["msg"][:n] = np.where(msg_len[:n] > 0, self._msg.ctypes.data + msg_off[:n], 0)
            v["msg_len"][:n] = msg_len[:n]
            v["sig"][:n] = np.where(sig_len[:n] > 0, self._sig.ctypes.data + sig_off[:n], 0)
            v["sig_len"][:n] = sig_len[:n]
        self.n_jobs = len(jobs)
        self.n_sets = n
        self.jobs = (LsgJob * max(len(jobs), 1))()
        jd = np.dtype({"names": ["sets", "n_sets", "flags"], "formats": [np.uint64, np.uint32, np.uint32],
                       "offsets": [LsgJob.sets.offset, LsgJob.n_sets.offset, LsgJob.flags.offset],
                       "itemsize": ctypes.sizeof(LsgJob)})
        jv = np.frombuffer(self.jobs, dtype=jd)
        counts = np.array([len(sets) for sets, _ in jobs] or [0], np.uint64)
        firsts = np.zeros_like(counts)
        if len(jobs) > 1:
            firsts[1:] = np.cumsum(counts)[:-1]
        if jobs:
            jv["sets"][:len(jobs)] = ctypes.addressof(self.sets) + firsts * ctypes.sizeof(LsgSet)
            jv["n_sets"][:len(jobs)] = counts
            jv["flags"][:len(jobs)] = [f for _, f in jobs]


class Context:
    """A device context (lsg_ctx) over `device`, or over the list `devices` (lsg_init_devices).
    Raises NativeUnavailable without a gfx950 GPU."""

    def __init__(self, device=0, devices=None, lib=None):
        self.lib = load_library(lib or LIB_PATH)
        h = ctypes.c_void_p()
        if devices is None:
            rc = self.lib.lsg_init(int(device), ctypes.byref(h))
        else:
            ids = (ctypes.c_int * len(devices))(*devices)
            rc = self.lib.lsg_init_devices(ids, len(devices), ctypes.byref(h))
        if rc != LSG_OK:
            raise NativeUnavailable(f"lsg_init({devices if devices is not None else device}) failed with status {rc} "
                                    f"(no gfx950 device?)")
        self.h = h
        self.device = device if devices is None else devices[0]
        self.devices = [self.device] if devices is None else list(devices)

    def reserve(self, max_sets, max_pks=None, max_msg_bytes=None, n_slots=0):
        """lsg_reserve: preallocate the first n_slots pipeline slots (0 = all) for packages of up
        to max_sets sets (so that steady-state submissions allocate nothing)."""
        max_pks = max_sets if max_pks is None else max_pks
        max_msg_bytes = 32 * max_sets if max_msg_bytes is None else max_msg_bytes
        self._check(self.lib.lsg_reserve(self.h, max_sets, max_pks, max_msg_bytes, n_slots), "lsg_reserve")

    def set_coalesce(self, max_sets, max_inflight=2):
        """lsg_set_coalesce: packages of <= max_sets sets are held while max_inflight launches
        are on the device and go out together (0 turns it off)"""
        self._check(self.lib.lsg_set_coalesce(self.h, int(max_sets), int(max_inflight)), "lsg_set_coalesce")

    def allocation_count(self):
        v = ctypes.c_uint64()
        self._check(self.lib.lsg_allocation_count(self.h, ctypes.byref(v)), "lsg_allocation_count")
        return v.value

    def device_count(self):
        v = ctypes.c_int32()
        self._check(self.lib.lsg_device_count(self.h, ctypes.byref(v)), "lsg_device_count")
        return v.value

    def close(self):
        if getattr(self, "h", None):
            self.lib.lsg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _check(self, rc, what):
        if rc != LSG_OK:
            raise RuntimeError(f"{what} failed ({rc}): {self.lib.lsg_last_error(self.h).decode(errors='replace')}")

    def device_name(self):
        b = ctypes.create_string_buffer(256)
        self._check(self.lib.lsg_device_name(self.h, b, 256), "lsg_device_name")
        return b.value.decode()

    def verify_jobs(self, jobs, seed=0):
        """jobs: list of (sets, flags) with sets = list of (pks, msg, sig), or PreparedJobs.
        Returns (results list of (status, err_code), stats dict)."""
        t = self.submit_jobs(jobs, seed=seed)
        if t is None:
            raise RuntimeError("lsg_submit_jobs: every pipeline slot is busy")
        return self.wait_jobs(t)

    def submit_jobs(self, jobs, seed=0):
        """Asynchronous verify_jobs: returns a ticket for wait_jobs, or None when every
        pipeline slot is busy (LSG_ERR_BUSY).  The inputs are copied before returning."""
        p = jobs if isinstance(jobs, PreparedJobs) else PreparedJobs(jobs)
        t = ctypes.c_uint64()
        rc = self.lib.lsg_submit_jobs(self.h, p.jobs, p.n_jobs, seed, ctypes.byref(t))
        if rc == LSG_ERR_BUSY:
            return None
        self._check(rc, "lsg_submit_jobs")
        return (t.value, p.n_jobs)

    @staticmethod
    def _results(res, st, n):
        out = [(res[i].status, res[i].err_code) for i in range(n)]
        stats = {k: getattr(st, k) for k, _ in LsgStats._fields_ }
        return out, stats

    def wait_jobs(self, ticket, raw=False):
        """-> (per-job (status, err_code), stats); raw=True returns the ctypes result array."""
        return self.wait_jobs_node(ticket, -1, raw=raw)

    def wait_jobs_node(self, ticket, node_valid, raw=False):
        """lsg_wait_jobs_node: resolve a ticket with the node verdict of the all-gathered
        partials (1 passed, 0 failed; -1 = this GPU's own check, i.e. wait_jobs)."""
        t, n = ticket
        res = (LsgJobResult * max(n, 1))()
        st = LsgStats()
        self._check(self.lib.lsg_wait_jobs_node(self.h, t, int(node_valid), res, ctypes.byref(st)),
                    "lsg_wait_jobs_node")
        if raw:
            return res, {k: getattr(st, k) for k, _ in LsgStats._fields_ }
        return self._results(res, st, n)

    def jobs_partial_device(self, ticket, dev_ptr):
        """lsg_jobs_partial_device: the package partial copied device-to-device to dev_ptr (576
        bytes on this context's device, e.g. a torch tensor's data_ptr()); -> has_batch"""
        hb = ctypes.c_int32()
        self._check(self.lib.lsg_jobs_partial_device(self.h, ticket[0], ctypes.c_void_p(dev_ptr), ctypes.byref(hb)),
                    "lsg_jobs_partial_device")
        return bool(hb.value)

    def final_submit_device(self, dev_ptr, n):
        """lsg_final_submit_device over n partials in device memory -> final ticket (None if busy)"""
        t = ctypes.c_uint64()
        rc = self.lib.lsg_final_submit_device(self.h, ctypes.c_void_p(dev_ptr), n, ctypes.byref(t))
        if rc == LSG_ERR_BUSY:
            return None
        self._check(rc, "lsg_final_submit_device")
        return t.value

    def jobs_partial(self, ticket):
        """lsg_jobs_partial: (576-byte Miller product of the package group, has_batch)."""
        out = ctypes.create_string_buffer(576)
        hb = ctypes.c_int32()
        self._check(self.lib.lsg_jobs_partial(self.h, ticket[0], out, ctypes.byref(hb)), "lsg_jobs_partial")
        return out.raw, bool(hb.value)

    def probe_mad_peak(self):
        v = ctypes.c_double()
        self._check(self.lib.lsg_probe_mad_peak(self.h, ctypes.byref(v)), "lsg_probe_mad_peak")
        return v.value

    def pipeline_slots(self):
        n = ctypes.c_int32()
        self._check(self.lib.lsg_pipeline_slots(self.h, ctypes.byref(n)), "lsg_pipeline_slots")
        return n.value

    def poll(self, ticket):
        t = ticket[0] if isinstance(ticket, tuple) else ticket
        d = ctypes.c_int32()
        self._check(self.lib.lsg_poll(self.h, t, ctypes.byref(d)), "lsg_poll")
        return bool(d.value)

    def verify_sets(self, sets, seed=0):
        b = SetBuffer(sets)
        res = LsgJobResult()
        self._check(self.lib.lsg_verify_sets(self.h, b.arr, b.n, seed, ctypes.byref(res)), "lsg_verify_sets")
        return res.status, res.err_code

    def aggregate_pubkeys(self, pks):
        """pks: list of encoded keys, or PkIndices into the pubkey table."""
        if isinstance(pks, PkIndices):
            pk_len, pkb = LSG_PK_INDEX, pks.tobytes()
        else:
            pk_len, pkb = (len(pks[0]) if pks else 96), b"".join(pks)
        out = ctypes.create_string_buffer(96)
        err = ctypes.c_int32()
        self._check(self.lib.lsg_aggregate_pubkeys(self.h, pkb, pk_len, len(pks), out, ctypes.byref(err)),
                    "lsg_aggregate_pubkeys")
        return out.raw, err.value

    def aggregate_pubkeys_multi(self, key_lists):
        """PublicKey.aggregate for every list of keys (encoded bytes, or PkIndices) in one device
        pass: [(uncompressed 96 B, BLST / LSG error code)] per list."""
        n = len(key_lists)
        if n == 0:
            return []
        b = SetBuffer([(k, b"", b"") for k in key_lists])
        out = ctypes.create_string_buffer(96 * n)
        err = (ctypes.c_int32 * n)()
        self._check(self.lib.lsg_aggregate_pubkeys_multi(self.h, b.arr, n, out, err), "lsg_aggregate_pubkeys_multi")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [(raw[96 * i:96 * i + 96], err[i]) for i in range(n)]

    def pubkey_table_set(self, first_index, pks):
        """index2pubkey[first_index + k] = pks[k] on the device; returns per-key BLST codes."""
        n = len(pks)
        pk_len = len(pks[0]) if pks else 96
        err = (ctypes.c_int32 * max(n, 1))()
        self._check(self.lib.lsg_pubkey_table_set(self.h, first_index, b"".join(pks), pk_len, n, err),
                    "lsg_pubkey_table_set")
        return list(err[:n])

    def pubkey_table_size(self):
        n = ctypes.c_size_t()
        self._check(self.lib.lsg_pubkey_table_size(self.h, ctypes.byref(n)), "lsg_pubkey_table_size")
        return n.value

    def pubkey_validate(self, pks):
        """Batched KeyValidate: [(uncompressed 96 B, BLST code)] per key."""
        n = len(pks)
        if n == 0:
            return []
        pk_len = len(pks[0])
        out = ctypes.create_string_buffer(96 * n)
        err = (ctypes.c_int32 * n)()
        self._check(self.lib.lsg_pubkey_validate(self.h, b"".join(pks), pk_len, n, out, err), "lsg_pubkey_validate")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [(raw[96 * k:96 * k + 96], err[k]) for k in range(n)]

    def aggregate_signatures(self, groups):
        """Op-pool Signature.aggregate over each list of signatures in `groups` (one device
        pass for all): [(compressed 96 B, BLST code or LSG_ERR_EMPTY_AGGREGATE)] per group."""
        ng = len(groups)
        if ng == 0:
            return []
        flat = [sg for g in groups for sg in g]
        sl = len(flat[0]) if flat else 96
        assert all(len(sg) == sl for sg in flat)
        offs = (ctypes.c_uint32 * (ng + 1))()
        for g in range(ng):
            offs[g + 1] = offs[g] + len(groups[g])
        out = ctypes.create_string_buffer(96 * ng)
        err = (ctypes.c_int32 * ng)()
        self._check(self.lib.lsg_aggregate_signatures(self.h, b"".join(flat), sl, offs, ng, out, err),
                    "lsg_aggregate_signatures")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [(raw[96 * g:96 * g + 96], err[g]) for g in range(ng)]

    def _signing_roots(self, fn, objs, size, domains):
        n = len(objs)
        if n == 0:
            return []
        assert all(len(o) == size for o in objs)
        if isinstance(domains, (bytes, bytearray)):
            dom, stride = bytes(domains), 0
        else:
            assert len(domains) == n
            dom, stride = b"".join(domains), 32
        assert len(dom) == (32 if stride == 0 else 32 * n)
        out = ctypes.create_string_buffer(32 * n)
        self._check(getattr(self.lib, fn)(self.h, b"".join(objs), n, dom, stride, out), fn)
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [raw[32 * i:32 * i + 32] for i in range(n)]

    def signing_roots(self, object_roots, domains):
        """computeSigningRoot from object roots; `domains` is one 32-byte domain or a list."""
        return self._signing_roots("lsg_signing_roots", object_roots, 32, domains)

    def attestation_signing_roots(self, data128s, domains):
        """getAttestationDataSigningRoot from SSZ-serialized phase0.AttestationData (128 B each)."""
        return self._signing_roots("lsg_attestation_signing_roots", data128s, 128, domains)

    def hash_to_g2(self, msgs, dst=b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"):
        if not msgs:
            return []
        ml = len(msgs[0])
        assert all(len(m) == ml for m in msgs)
        out = ctypes.create_string_buffer(192 * len(msgs))
        self._check(self.lib.lsg_hash_to_g2(self.h, b"".join(msgs), ml, len(msgs), dst, len(dst), out), "lsg_hash_to_g2")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [raw[192 * i:192 * i + 192] for i in range(len(msgs))]

    def sig_decode(self, sigs):
        if not sigs:
            return []
        sl = len(sigs[0])
        assert all(len(s) == sl for s in sigs)
        out = ctypes.create_string_buffer(192 * len(sigs))
        err = (ctypes.c_int32 * len(sigs))()
        self._check(self.lib.lsg_sig_decode(self.h, b"".join(sigs), sl, len(sigs), out, err), "lsg_sig_decode")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [(raw[192 * i:192 * i + 192], err[i]) for i in range(len(sigs))]

    def batch_partial(self, sets, seed=0):
        b = SetBuffer(sets)
        out = ctypes.create_string_buffer(576)
        errs = (ctypes.c_int32 * max(b.n, 1))()
        anyerr = ctypes.c_int32()
        self._check(self.lib.lsg_batch_partial(self.h, b.arr, b.n, seed, out, errs, ctypes.byref(anyerr)),
                    "lsg_batch_partial")
        return out.raw, [errs[i] for i in range(b.n)], bool(anyerr.value)

    def final_verify(self, partials):
        v = ctypes.c_int32()
        self._check(self.lib.lsg_final_verify(self.h, b"".join(partials), len(partials), ctypes.byref(v)),
                    "lsg_final_verify")
        return bool(v.value)

    def final_submit(self, partials):
        t = ctypes.c_uint64()
        rc = self.lib.lsg_final_submit(self.h, b"".join(partials), len(partials), ctypes.byref(t))
        if rc == LSG_ERR_BUSY:
            return None
        self._check(rc, "lsg_final_submit")
        return t.value

    def final_wait(self, ticket):
        v = ctypes.c_int32()
        self._check(self.lib.lsg_final_wait(self.h, ticket, ctypes.byref(v)), "lsg_final_wait")
        return bool(v.value)

    def final_submit_groups(self, groups):
        """groups: list of equal-length lists of 576-byte partials -> one ticket, one final
        exponentiation per group."""
        ng = len(groups)
        pg = len(groups[0]) if groups else 0
        if any(len(g) != pg for g in groups):
            raise ValueError("every group needs the same number of partials")
        t = ctypes.c_uint64()
        rc = self.lib.lsg_final_submit_groups(self.h, b"".join(b"".join(g) for g in groups), ng, pg, ctypes.byref(t))
        if rc == LSG_ERR_BUSY:
            return None
        self._check(rc, "lsg_final_submit_groups")
        t_ng = ng
        return (t.value, t_ng)

    def final_wait_groups(self, ticket):
        t, ng = ticket
        v = (ctypes.c_int32 * max(ng, 1))()
        self._check(self.lib.lsg_final_wait_groups(self.h, t, v), "lsg_final_wait_groups")
        return [bool(x) for x in v[:ng]]

    def sign(self, sks, msgs):
        """sks: list of ints (< r); msgs: equal-length bytes.  Returns compressed signatures."""
        if not sks:
            return []
        ml = len(msgs[0])
        out = ctypes.create_string_buffer(96 * len(sks))
        skb = b"".join(int(k).to_bytes(32, "big") for k in sks)
        self._check(self.lib.lsg_sign(self.h, skb, b"".join(msgs), ml, len(sks), out), "lsg_sign")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [raw[96 * i:96 * i + 96] for i in range(len(sks))]

    def sk_to_pk(self, sks):
        if not sks:
            return []
        out = ctypes.create_string_buffer(96 * len(sks))
        skb = b"".join(int(k).to_bytes(32, "big") for k in sks)
        self._check(self.lib.lsg_sk_to_pk(self.h, skb, len(sks), out), "lsg_sk_to_pk")
        raw = out.raw  # (one copy: .raw copies the whole buffer on every access)
        return [raw[96 * i:96 * i + 96] for i in range(len(sks))]

    def check_fp2_mul(self, words):
        """lsg_check_fp2_mul: `words` = 56 u32 per item (a0, a1, b0, b1 in the pair layout,
        lodestar_bls.h); returns 28 u32 per item (c0, c1, raw)."""
        n = len(words) // 56
        assert len(words) == 56 * n
        out = ctypes.create_string_buffer(4 * 28 * n)
        src = struct.pack(f"<{len(words)}I", *words)
        self._check(self.lib.lsg_check_fp2_mul(self.h, src, n, out), "lsg_check_fp2_mul")
        return list(struct.unpack(f"<{28 * n}I", out.raw))

    def probe_fp_mul_rate(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.lsg_probe_fp_mul_rate(self.h, ctypes.byref(a), ctypes.byref(b)), "lsg_probe_fp_mul_rate")
        return a.value, b.value

    def last_kernel_times(self, max_entries=1024):
        names = (ctypes.c_char_p * max_entries)()
        ms = (ctypes.c_double * max_entries)()
        n = self.lib.lsg_last_kernel_times(self.h, names, ms, max_entries)
        return [(names[i].decode(), ms[i]) for i in range(n)]
