"""The CPU baseline (oracle/gmp_baseline.c on system GMP) computes the
reference's encryption: checked against the oracle before it is ever timed."""
import random

import pytest

from oracle import bench_cpu
from oracle import paillier_oracle as O


def test_gmp_port_matches_oracle():
    if bench_cpu._gmp_lib() is None:
        pytest.skip("libgmp.so.10 not loadable")
    k = bench_cpu._key(2048)
    r = random.Random(11)
    for m in (0, 1, -1, 2 ** 40, -(2 ** 50) + 3):
        a = r.getrandbits(1023)
        assert bench_cpu.gmp_encrypt_one(k, m, a) == O.encrypt_m(k, m % k["n"], a)
