"""Every runtime option blsgpu_set_option accepts (lodestar_amd/csrc/runtime.cpp) is documented in include/blsgpu.h
and listed in INTEGRATION.md, and the read-only keys blsgpu_get_option adds are the documented ones (host files
only; tests/test_gpu_options.py exercises the keys on a device)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _keys():
    src = open(os.path.join(ROOT, "lodestar_amd", "csrc", "runtime.cpp")).read()
    i, j = src.index("int blsgpu_set_option"), src.index("int blsgpu_get_option")
    set_keys = set(re.findall(r'k == "([a-z0-9_]+)"', src[i:j]))
    get_keys = set(re.findall(r'k == "([a-z0-9_]+)"', src[j:j + 10000]))
    return set_keys, get_keys


def test_every_option_documented():
    set_keys, get_keys = _keys()
    assert len(set_keys) > 30
    header = open(os.path.join(ROOT, "include", "blsgpu.h")).read()
    integration = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert sorted(k for k in set_keys if f'"{k}"' not in header) == []
    assert sorted(k for k in set_keys if f"`{k}`" not in integration) == []
    assert get_keys - set_keys == {"hw_queues", "abi_version", "spurious_groups"}
    assert set_keys <= get_keys


def test_gpu_option_test_covers_every_key():
    """tests/test_gpu_options.py round-trips every key but "slots" (resizing the dispatcher pool has its own tests)."""
    set_keys, _ = _keys()
    gpu_test = open(os.path.join(ROOT, "tests", "test_gpu_options.py")).read()
    covered = set(re.findall(r'"([a-z0-9_]+)": \(', gpu_test))
    assert sorted(set_keys - covered) == ["slots"]
    assert covered <= set_keys
