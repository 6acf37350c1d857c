"""The N-API addon (lodestar_amd/napi/lsg_napi.c) under AddressSanitizer + UBSan, on the CPU.

SURVEY.md section 5 asks for an ASan host build.  The addon is compiled with
-fsanitize=address,undefined and linked against tests/native/lsg_stub.c, a host-only stand-in
of the C ABI (no arithmetic: it copies every package byte at submit, as the library's pinned
staging does, and answers with a toy verdict rule after a short "device" delay).  Node -- not
itself instrumented -- loads it with the ASan runtime preloaded, and tests/js/
test_napi_sanitizers.js drives BlsGpuVerifier through it: the package threads, the priority
thread, verifyPacked's arena / descriptor marshalling, the threadsafe completions, close() with
packages in flight, forced garbage collections.  Any heap error, leak in the addon or the stub,
or undefined behaviour aborts the run.  Reference: multithread/index.ts:151-431 (the traffic),
SURVEY.md:224.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
NODE_INCLUDE = "/usr/include/node"
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-Wall",
       "-Werror", "-shared", "-fPIC"]
# leaks of node itself (OpenSSL CA loading, V8, libuv) are not ours
LSAN_SUPP = "leak:libnode.so\nleak:libuv.so\nleak:libv8\nleak:libcrypto\nleak:libssl\n"


def _tools():
    if not shutil.which("node") or not shutil.which("gcc"):
        return None
    if not os.path.exists(os.path.join(NODE_INCLUDE, "node_api.h")):
        return None
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return asan if asan and os.path.isabs(asan) and os.path.exists(asan) else None


def test_napi_addon_under_asan_ubsan(tmp_path):
    asan = _tools()
    if not asan:
        pytest.skip("node headers or the gcc ASan runtime are not available")
    inc = os.path.join(ROOT, "include")
    stub = tmp_path / "liblodestar_bls.so"
    addon = tmp_path / "lsg_napi.node"
    subprocess.check_call(["gcc"] + SAN + ["-I", inc, os.path.join(HERE, "native", "lsg_stub.c"), "-o", str(stub),
                                           "-lpthread"])
    subprocess.check_call(["gcc", "-std=gnu11"] + SAN + ["-DNODE_GYP_MODULE_NAME=lsg_napi", "-I", NODE_INCLUDE, "-I", inc,
                                                         os.path.join(ROOT, "lodestar_amd", "napi", "lsg_napi.c"),
                                                         "-o", str(addon), "-L", str(tmp_path), "-llodestar_bls",
                                                         f"-Wl,-rpath,{tmp_path}", "-lpthread"])
    supp = tmp_path / "lsan.supp"
    supp.write_text(LSAN_SUPP)
    env = dict(os.environ)
    # the ASan runtime first (node is not instrumented); anything already preloaded stays
    env["LD_PRELOAD"] = asan + (":" + env["LD_PRELOAD"] if env.get("LD_PRELOAD") else "")
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1:strict_string_checks=1"
    env["LSAN_OPTIONS"] = f"suppressions={supp}:print_suppressions=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    p = subprocess.run(["node", "--expose-gc", os.path.join(HERE, "js", "test_napi_sanitizers.js"), str(addon)],
                       env=env, capture_output=True, text=True, timeout=300)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-6000:]
    assert "napi sanitizer traffic ok" in out, out[-3000:]
    for bad in ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:"):
        assert bad not in out, out[-6000:]
