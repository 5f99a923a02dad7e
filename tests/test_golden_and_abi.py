"""CPU tests: the committed golden fixture against the oracle, the C-ABI library's exported surface, and the
N-API addon's load/exports (no compute: there is no GPU here).  GPU use of the same fixture is in
tests/test_gpu_golden.py."""
import ctypes
import json
import os
import re
import shutil
import subprocess

import pytest

from oracle import bls12_381 as bls

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FX = json.load(open(os.path.join(ROOT, "tests", "golden", "verify_sets.json")))


def test_golden_keys_and_hashes_match_oracle():
    for k in FX["keys"]:
        assert bls.g1_serialize(bls.sk_to_pk(int(k["sk"], 16))).hex() == k["pk"]
    for h in FX["hash_to_g2"]:
        assert bls.g2_serialize(bls.hash_to_g2(bytes.fromhex(h["msg"]))).hex() == h["g2"]
    keys = [bls.g1_deserialize(bytes.fromhex(k["pk"])) for k in FX["keys"]]
    for a in FX["aggregate_pubkeys"]:
        assert bls.g1_serialize(bls.aggregate_pubkeys([keys[i] for i in a["pks"]])).hex() == a["pk"]


def test_golden_expected_results_match_oracle():
    from tools.gen_golden import expected_job

    keys = [bls.g1_deserialize(bytes.fromhex(k["pk"])) for k in FX["keys"]]
    case = next(c for c in FX["cases"] if c["name"] == "multi_set_jobs/plain")
    got = [expected_job([FX["sets"][k] for k in j], keys) for j in case["jobs"]]
    assert got == case["expected"]
    # the reference's own fixture rule: a 32-byte signature is BLST_INVALID_SIZE (multithread.test.ts:100)
    s = next(s for s in FX["sets"] if s["name"] == "invalid_size_32")
    assert bls.classify_signature(bytes.fromhex(s["sig"])) == bls.BLST_INVALID_SIZE


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "blsgpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(blsgpu_[a-z_]+)\s*\(", txt)))


def test_c_abi_exports_every_header_symbol():
    from lodestar_amd import native

    lib = native.load()  # in-tree libblsgpu.so, built by __graft_entry__.build()
    syms = header_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/blsgpu.h but not exported"
    assert sorted(native.EXPORTED_SYMBOLS) == syms
    assert native.code_name(native.INVALID_SIZE) == "BLST_INVALID_SIZE"
    assert native.code_name(native.ERR_CLOSED) == "QUEUE_ERROR_QUEUE_ABORTED"


def test_no_device_fails_loudly():
    """The product has no CPU path: without a GPU, blsgpu_init reports ERR_NO_DEVICE."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from lodestar_amd import native

    with pytest.raises(RuntimeError, match="NO_DEVICE"):
        native.Context()


NODE = shutil.which("node")
ADDON = os.path.join(ROOT, "lodestar_amd", "node", "blsgpu_napi.node")


@pytest.mark.skipif(NODE is None or not os.path.exists(ADDON), reason="node or the N-API addon is absent")
def test_node_addon_loads_and_exports():
    script = (
        "const m = require(process.argv[1]);"
        "const a = m.addon;"
        "const want = ['close','codeName','deviceCount','init','pubkeysCount','setOption','submit','uploadPubkeys'];"
        "for (const k of want) if (typeof a[k] !== 'function') throw new Error('missing ' + k);"
        "if (a.codeName(8) !== 'BLST_INVALID_SIZE') throw new Error('codeName');"
        "if (typeof m.BlsGpuVerifier !== 'function') throw new Error('class');"
        "let threw = null; try { new m.BlsGpuVerifier(); } catch (e) { threw = e.message; }"
        "console.log(JSON.stringify({threw}));"
    )
    out = subprocess.run([NODE, "-e", script, os.path.join(ROOT, "lodestar_amd", "node", "BlsGpuVerifier.cjs")],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    import torch

    if not torch.cuda.is_available():
        assert "NO_DEVICE" in json.loads(out.stdout)["threw"]


@pytest.mark.skipif(NODE is None or not os.path.exists(ADDON), reason="node or the N-API addon is absent")
def test_esm_entry_imports():
    """The ES-module entry (lodestar_amd/node/index.js, package.json "type": "module" like the reference's
    packages/beacon-node/package.json:15) imports the CommonJS implementation through createRequire and exposes the
    IBlsVerifier surface; without a GPU the constructor fails loudly."""
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "esm_entry.mjs")], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["esm"] and {"BlsGpuVerifier", "BlsGpuSingleThreadVerifier", "verifySignatureSet"} <= set(r["exports"])
    import torch

    if not torch.cuda.is_available():
        assert "NO_DEVICE" in r["threw"]
