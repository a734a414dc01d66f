"""Host-side helpers of the drop-in package (mirrors python/common/crypto/paillier/utils.py).

Only key generation and small-integer helpers live here; every per-element
operation of the hot path runs on the GPU through xfl_amd._native.
"""
import multiprocessing
import secrets
from typing import Optional

MPZ = int  # the reference aliases gmpy2.mpz; Python ints play that role here

_SMALL_PRIMES = [p for p in range(3, 2000) if all(p % d for d in range(2, int(p ** 0.5) + 1))]


def get_core_num(expected_core_num):
    """utils.py:25-31"""
    max_cores = multiprocessing.cpu_count()
    if expected_core_num == -1:
        return max_cores
    return min(max(1, expected_core_num), max_cores)


def mul(a, b):
    return a * b


# Scalar helpers kept for API completeness (utils.py:38-68); the batched
# device path never calls them.
def crt(mp, mq, p, q, q_inverse, n):
    """utils.py:38-43"""
    u = ((mp - mq) * q_inverse) % p
    return int((mq + u * q) % n)


def mulmod(a, b, c):
    """utils.py:50-54"""
    return (a * b) % c


def powmod(a: int, b: int, c: int) -> int:
    """utils.py:57-68 (powmod(1, ., .) = 1 as in the reference)"""
    if a == 1:
        return 1
    return pow(a, b, c)


def invert(a, b):
    """utils.py:71-76: ZeroDivisionError when no inverse exists."""
    try:
        return pow(a, -1, b)
    except ValueError:
        raise ZeroDivisionError("invert(a, b) no inverse exists")


def is_probable_prime(n, rounds=32, rng=None):
    """Miller-Rabin (GMP's mpz_probab_prime_p plays this role for gmpy2.next_prime)."""
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    rng = rng or secrets.SystemRandom()
    for _ in range(rounds):
        a = rng.randrange(2, n - 1)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def next_prime(x, rng=None):
    """Smallest probable prime > x (gmpy2.next_prime semantics): GMP's
    mpz_nextprime when libgmp is present (what gmpy2 calls), else Miller-Rabin."""
    from . import _gmp
    if _gmp.available() and x >= 0:
        return _gmp.next_prime(int(x))
    n = x + 1
    if n <= 2:
        return 2
    if n % 2 == 0:
        n += 1
    while not is_probable_prime(n, rng=rng):
        n += 2
    return n


def getprimeover(n, seed: Optional[int] = None, rng=None):
    """utils.py:79-89: random n-bit number with the top bit set -> next_prime."""
    rng = rng or secrets.SystemRandom()
    r = rng.getrandbits(n) | (1 << (n - 1))
    return next_prime(r, rng=rng)
