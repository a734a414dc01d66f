"""The CPU baseline (oracle/gmp_baseline.c on system GMP) computes the
reference's encryption: checked against the oracle before it is ever timed,
and its batch entry point (the checker of tests/test_gpu_prod_windows.py) is
pinned to the reference's own ciphertexts at every key size."""
import random

import numpy as np
import pytest

from oracle import bench_cpu
from oracle import paillier_oracle as O
from tests.conftest import FIXTURES, fl, hx, load_fixture


def _need_gmp():
    if bench_cpu._gmp_lib() is None:
        pytest.skip("libgmp.so.10 not loadable")


def _words(xs, nw):
    return np.array([np.frombuffer(int(x).to_bytes(4 * nw, "little"), dtype="<u4") for x in xs], dtype=np.uint32)


def test_gmp_port_matches_oracle():
    _need_gmp()
    k = bench_cpu._key(2048)
    r = random.Random(11)
    for m in (0, 1, -1, 2 ** 40, -(2 ** 50) + 3):
        a = r.getrandbits(1023)
        assert bench_cpu.gmp_encrypt_one(k, m, a) == O.encrypt_m(k, m % k["n"], a)


@pytest.mark.parametrize("fx", [f for f in FIXTURES if "nodjn" not in f])
def test_gmp_batch_matches_reference_ciphertexts(fx):
    """gmpb_encrypt_batch on the fixture's recorded draws gives the reference's
    raw ciphertexts (private DJN cases, paillier.py:189-209) bit-exactly."""
    _need_gmp()
    g = load_fixture(fx)
    kf = g["key"]
    k = O.derive_private(hx(kf["p"]), hx(kf["q"]), hx(kf["h_pow_n"]))
    nw = g["key_bits"] // 32
    aw = nw // 2
    ms, rs, want = [], [], []
    for case, c in g["encrypt"].items():
        if not isinstance(c, dict) or not c.get("private") or not c.get("obfuscation"):
            continue
        xs = [hx(v) for v in c["input"]] if c["kind"] == "int" else [fl(v) for v in c["input"]]
        for i, x in enumerate(xs):
            ms.append(O.encode_element(k, x, c["precision"], c["max_exponent"])[0])
            rs.append(hx(c["rand"][i]))
            want.append(hx(c["raw"][i]))
    assert len(ms) >= 8
    got = bench_cpu.gmp_encrypt_batch(k, _words(ms, nw), _words(rs, aw), threads=4)
    assert [int.from_bytes(row.tobytes(), "little") for row in got] == want
