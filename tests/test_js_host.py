"""The Node host (lodestar_amd/js/blsGpuVerifier.js): queue, buffering, chunking and
error rules of BlsMultiThreadWorkerPool (multithread/index.ts) on the CPU, against a mock
of the N-API addon.  Needs only `node` (v12 is in the image); GPU verdicts through the real
addon are in tests/js/test_verifier_gpu.js (test_gpu_parity.py::test_node_host_on_gpu)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_host_queue_logic():
    r = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "test_verifier_host.js")], capture_output=True,
                       text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    # a test whose promise never settles lets node exit early with status 0: insist on the summary
    last = r.stdout.strip().splitlines()[-1]
    done, total = last.split()[0].split("/")
    assert last.endswith("passed") and done == total, r.stdout


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_napi_addon_loads_and_fails_loudly_without_gpu():
    addon = os.path.join(ROOT, "lodestar_amd", "napi", "lsg_napi.node")
    if not os.path.exists(addon):
        pytest.skip("addon not built (build() builds it when /usr/include/node exists)")
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    js = ("const a=require(process.argv[1]);"
          "const want=['open','close','slots','deviceName','verifyPacked','verifySets','aggregatePubkeys','hashToG2','sign','skToPk','pubkeyTableSet'];"
          "for(const k of want){if(typeof a[k]!=='function'){console.log('missing',k);process.exit(2);}}"
          "try{a.open(0);console.log('opened');process.exit(3);}catch(e){console.log(e.message);}")
    r = subprocess.run(["node", "-e", js, addon], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "lsg_init" in r.stdout
