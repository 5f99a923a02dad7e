import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the library's fault-injection hook (blsgpu_debug_inject) is armed only in processes started with this set
os.environ.setdefault("BLSGPU_FAULT_INJECTION", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: slower CPU test")
