"""CPU baseline worker for bench.py — TEST/BASELINE INFRASTRUCTURE ONLY.

Times the reference algorithm (DJN private-key CRT encryption,
paillier.py:189-209,273-287) restated in oracle/paillier_oracle.py with
pure-Python pow on this host; used as `cpu_baseline` (kind "port").
"""
import random
import time

from oracle import paillier_oracle as O

# fixed 2048/3072-bit DJN test keys are derived deterministically per worker
_KEYS = {}


def _key(bits):
    if bits not in _KEYS:
        from bench import make_key
        p, q, n, h = make_key(bits, seed=2024)
        _KEYS[bits] = O.derive_private(p, q, h)
    return _KEYS[bits]


def encrypt_for(arg):
    bits, seconds, wid = arg
    k = _key(bits)
    rng = random.Random(wid)
    bound = k["djn_exp_bound"]
    count = 0
    t0 = time.time()
    while time.time() - t0 < seconds:
        x = rng.gauss(0.0, 1.0)
        m, _ = O.encode_element(k, x, 7)
        O.encrypt_m(k, m, rng.randrange(1, bound))
        count += 1
    return count
