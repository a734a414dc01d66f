import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# One HIP runtime per process: torch ships its own libamdhip64, and if
# libxhe.so (linked against the system ROCm) initialises the runtime first, a
# later torch.cuda call in the same process finds "No HIP GPUs". Initialising
# torch first makes libxhe bind to the runtime torch loaded (as bench.py does).
try:
    import torch as _torch
    if _torch.cuda.is_available():
        _torch.cuda.init()
except Exception:  # no torch / no GPU: CPU-only runs
    pass
FIXTURES = ["paillier_2048_djn.json", "paillier_2048_nodjn.json", "paillier_3072_djn.json", "paillier_4096_djn.json",
            "paillier_8192_djn.json"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


_cache = {}


def load_fixture(name):
    if name not in _cache:
        with open(os.path.join(GOLDEN, name)) as f:
            _cache[name] = json.load(f)
    return _cache[name]


def hx(s):
    """Parse a fixture big-int string ('0x..' or '-0x..')."""
    return -int(s[1:], 16) if s.startswith("-") else int(s, 16)


def fl(s):
    return float.fromhex(s)


# The pure-Python oracle needs ~3 s per 8192-bit modexp: its CPU checks take
# the first few vectors of that fixture (the GPU tests check every vector).
CPU_VECTOR_LIMIT = {"paillier_8192_djn.json": 2}


@pytest.fixture(params=FIXTURES)
def golden(request):
    g = load_fixture(request.param)
    g["_name"] = request.param
    g["_cpu_limit"] = CPU_VECTOR_LIMIT.get(request.param)
    return g
