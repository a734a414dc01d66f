"""Host key generation through the system GMP (xfl_amd/paillier/_gmp.py):
mpz_nextprime / mpz_powm agree with the pure-Python fallbacks (the routines
gmpy2 wraps for the reference's getprimeover and h_pow_n, utils.py:79-89,
context.py:79-81)."""
import math
import random

import pytest

from xfl_amd.paillier import _gmp
from xfl_amd.paillier import utils as U

pytestmark = pytest.mark.skipif(not _gmp.available(), reason="no libgmp on this host")


def _py_next_prime(x):
    n = x + 1 + ((x + 1) % 2 == 0)
    while not U.is_probable_prime(n):
        n += 2
    return n


@pytest.mark.parametrize("bits", [2, 17, 64, 256, 768])
def test_next_prime_matches_python(bits):
    r = random.Random(bits)
    for _ in range(3):
        x = r.getrandbits(bits) | (1 << (bits - 1))
        assert _gmp.next_prime(x) == _py_next_prime(x)


def test_powmod_matches_python():
    r = random.Random(3)
    for bits in (64, 1024, 4096):
        b, e, m = r.getrandbits(bits), r.getrandbits(bits // 2), r.getrandbits(bits) | 1
        assert _gmp.powmod(b, e, m) == pow(b, e, m)
    assert _gmp.powmod(0, 5, 7) == 0 and _gmp.powmod(5, 0, 7) == 1


def test_djn_keygen_4096():
    from xfl_amd.paillier import PaillierContext
    c = PaillierContext.generate(4096, djn_on=True)
    assert 4094 <= c.n.bit_length() <= 4096
    assert math.gcd(c.p - 1, c.q - 1) == 2
