"""In-tree build of the gfx950 HIP library (lodestar_amd/liblodestar_bls.so).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container; the
built .so travels to the GPU box with the repository snapshot.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "liblodestar_bls.so")
# kernel translation units compile in parallel; lsg_host.hip is the orchestration + C ABI
SOURCES = ["lsg_k_hash.hip", "lsg_k_sig.hip", "lsg_k_pk.hip", "lsg_k_miller.hip", "lsg_k_reduce.hip", "lsg_slp.hip",
           "lsg_host.hip"]
HEADERS = ["lsg_types.hpp", "lsg_fp_lane.hpp", "lsg_fp_elem.hpp", "lsg_tower.hpp", "lsg_curve.hpp", "lsg_h2c.hpp",
           "lsg_pairing.hpp", "lsg_constants.hpp", "lsg_fp_pair.hpp", "lsg_constants_r29.hpp", "lsg_io.hpp",
           "lsg_serial.h", "lsg_kcommon.hpp", "lsg_launch.h", "lsg_layout.h", "lsg_slp_progs.h", "lsg_slp_exec.hpp", "lsg_inv.hpp",
           "lsg_ab.h"]
OBJ = os.path.join(HERE, "_obj")
# The A/B and test build (lsg_ab.h): the orchestration compiled with -DLSG_AB (its switches read
# from the environment) plus the row-backend serial kernels (LSG_SERIAL=row); every other
# translation unit is the shipped library's own object.  Tests that compare two forms of a
# stage load it beside the shipped library (lodestar_amd._native.load_library(AB_OUT)).
AB_OUT = os.path.join(HERE, "liblodestar_bls_ab.so")
AB_SOURCES = ["lsg_host.hip", "lsg_serial.hip", "lsg_serial_wide.hip"]
AB_FLAGS = ["-DLSG_AB=1"]


def hipcc():
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _deps():
    return [os.path.join(CSRC, f) for f in HEADERS] + [os.path.join(ROOT, "include", "lodestar_bls.h"),
                                                       os.path.abspath(__file__)]


def needs_rebuild(out=OUT, sources=SOURCES):
    if not os.path.exists(out):
        return True
    deps = [os.path.join(CSRC, f) for f in sources] + _deps()
    return max(os.path.getmtime(d) for d in deps if os.path.exists(d)) > os.path.getmtime(out)


# Tower functions (Fp2/Fp6/Fp12, LSG_BIGFN) inlined into the device kernels: as calls they
# passed Fp12 operands through stack frames (k_miller_accum<2>: 3408 B/lane of scratch,
# ~477 KB of memory-side traffic per set); inlined, the accumulation has no scratch at all
# (profiles/r01_pmc_traffic*.json, profiles/r01_inline_ab.txt).  Host builds keep the calls.
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DLSG_BIGFN=__host__ __device__ __forceinline__"]


def _obj_dir(extra):
    """objects of the default build in _obj/; A/B builds (extra flags) in their own directory"""
    if not extra:
        return OBJ
    import hashlib
    return OBJ + "_" + hashlib.sha1(" ".join(extra).encode()).hexdigest()[:10]


def _compile(src, verbose, extra):
    obj = os.path.join(_obj_dir(extra), os.path.splitext(src)[0] + ".o")
    srcp = os.path.join(CSRC, src)
    dep_t = max(os.path.getmtime(d) for d in [srcp] + _deps() if os.path.exists(d))
    if os.path.exists(obj) and os.path.getmtime(obj) >= dep_t:
        return obj
    cmd = [hipcc()] + CFLAGS + extra + ["-I", CSRC, "-I", os.path.join(ROOT, "include"), "-c", srcp, "-o", obj + ".tmp"]
    if verbose:
        print("[lodestar_amd.build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force=False, verbose=True, extra=None, out=None):
    """Compile the kernel translation units in parallel (hipcc --offload-arch=gfx950) and link
    liblodestar_bls.so (with RCCL for the multi-device partial exchange).  extra: additional
    compiler flags (A/B builds, written to `out` instead of the default library)."""
    from concurrent.futures import ThreadPoolExecutor
    gen = os.path.join(ROOT, "tools", "gen_constants.py")
    const = os.path.join(CSRC, "lsg_constants.hpp")
    if not os.path.exists(const) or os.path.getmtime(gen) > os.path.getmtime(const):
        subprocess.check_call([sys.executable, gen, const])
    gen_slp = os.path.join(ROOT, "tools", "gen_slp.py")
    progs = os.path.join(CSRC, "lsg_slp_progs.h")
    if not os.path.exists(progs) or os.path.getmtime(gen_slp) > os.path.getmtime(progs):
        subprocess.check_call([sys.executable, gen_slp, progs])
    extra = list(extra or [])
    out = out or OUT
    if not force and not extra and out == OUT and not needs_rebuild():
        if read_manifest(OUT) is None:
            write_manifest(OUT, SOURCES, [])
        return OUT
    odir = _obj_dir(extra)
    os.makedirs(odir, exist_ok=True)
    if force:
        for f in os.listdir(odir):
            os.remove(os.path.join(odir, f))
    jobs = int(os.environ.get("LSG_BUILD_JOBS", str(min(8, os.cpu_count() or 4))))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose, extra), SOURCES))
    _link(objs, out, verbose)
    write_manifest(out, SOURCES, extra)
    return out


def source_hash(sources=SOURCES):
    """sha256 over the library's sources, headers and the public header (sorted by name)"""
    import hashlib
    h = hashlib.sha256()
    files = sorted(set([os.path.join(CSRC, f) for f in list(sources) + HEADERS] +
                       [os.path.join(ROOT, "include", "lodestar_bls.h")]))
    for f in files:
        if os.path.exists(f):
            h.update(os.path.basename(f).encode() + b"\0")
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def _compiler_version():
    try:
        out = subprocess.run([hipcc(), "--version"], capture_output=True, text=True, timeout=60).stdout
        return next((ln.strip() for ln in out.splitlines() if "clang version" in ln), out.splitlines()[0].strip())
    except Exception as e:  # noqa: BLE001 (the manifest still records the rest)
        return "unknown (%s)" % e


def write_manifest(out, sources, extra):
    """one-line JSON manifest beside the .so: compiler, flags, source hash, build time"""
    import hashlib
    import json
    import time
    with open(out, "rb") as fh:
        so_sha = hashlib.sha256(fh.read()).hexdigest()
    rec = {"lib": os.path.basename(out), "so_sha256_16": so_sha[:16], "src_sha256": source_hash(sources),
           "compiler": _compiler_version(), "flags": CFLAGS + list(extra),
           "built_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    with open(out + ".manifest.json", "w") as fh:
        fh.write(json.dumps(rec, sort_keys=True) + "\n")
    return rec


def read_manifest(out=None):
    import json
    try:
        with open((out or OUT) + ".manifest.json") as fh:
            return json.loads(fh.read())
    except (OSError, ValueError):
        return None


def _link(objs, out, verbose):
    cmd = [hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared"] + objs + ["-L/opt/rocm/lib", "-lrccl",
                                                                           "-Wl,-rpath,/opt/rocm/lib", "-o", out + ".tmp"]
    if verbose:
        print("[lodestar_amd.build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)


def build_ab(verbose=True):
    """The A/B and test library (AB_OUT): AB_SOURCES with AB_FLAGS, the rest shared with the
    shipped build (build() first)."""
    from concurrent.futures import ThreadPoolExecutor
    build(verbose=verbose)
    if not needs_rebuild(AB_OUT, SOURCES + AB_SOURCES):
        return AB_OUT
    os.makedirs(_obj_dir(AB_FLAGS), exist_ok=True)
    with ThreadPoolExecutor(max_workers=len(AB_SOURCES)) as ex:
        ab = dict(zip(AB_SOURCES, ex.map(lambda s: _compile(s, verbose, AB_FLAGS), AB_SOURCES)))
    objs = [ab.get(s) or os.path.join(OBJ, os.path.splitext(s)[0] + ".o") for s in SOURCES]
    objs += [ab[s] for s in AB_SOURCES if s not in SOURCES]
    _link(objs, AB_OUT, verbose)
    write_manifest(AB_OUT, SOURCES + AB_SOURCES, AB_FLAGS)
    return AB_OUT


NAPI_SRC = os.path.join(HERE, "napi", "lsg_napi.c")
NAPI_OUT = os.path.join(HERE, "napi", "lsg_napi.node")
NODE_INCLUDE = "/usr/include/node"


def build_napi(verbose=True):
    """Thin N-API addon (lodestar_amd/napi/lsg_napi.node) over the C ABI, for the Node host
    (lodestar_amd/js/blsGpuVerifier.js).  Skipped (returns None) when Node's headers are absent."""
    if not os.path.exists(os.path.join(NODE_INCLUDE, "node_api.h")):
        return None
    deps = [NAPI_SRC, OUT, os.path.join(ROOT, "include", "lodestar_bls.h")]
    if os.path.exists(NAPI_OUT) and max(os.path.getmtime(d) for d in deps) <= os.path.getmtime(NAPI_OUT):
        return NAPI_OUT
    cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-shared", "-fPIC", "-DNODE_GYP_MODULE_NAME=lsg_napi",
           "-I", NODE_INCLUDE, "-I", os.path.join(ROOT, "include"), NAPI_SRC, "-o", NAPI_OUT + ".tmp",
           "-L", HERE, "-llodestar_bls", "-lpthread", "-Wl,-rpath,$ORIGIN/.."]
    if verbose:
        print("[lodestar_amd.build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(NAPI_OUT + ".tmp", NAPI_OUT)
    return NAPI_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_ab()
    build_napi()
