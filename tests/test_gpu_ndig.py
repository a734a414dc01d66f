"""Montgomery digits mod n^2 (PMDX, xfl_amd/csrc/pdigit_dev.hpp; the 2048-bit
public non-DJN encryption and the scalar powers of the batch shape): edge
inputs of the conversions (x = 1, n - 1, n, n^2 - 1; r = 1, n - 1; k = 0, 1,
a full 2048-bit k) and batches larger than one grid (grid-stride element
loop) against Python's pow (the reference's gmpy2 arithmetic, utils.py:46-76;
paillier.py:156-187, 228-230)."""
import random

import pytest

from tests.conftest import hx, load_fixture

pytestmark = pytest.mark.gpu

FX = "paillier_2048_djn.json"


def _key():
    k = load_fixture(FX)["key"]
    return hx(k["n"]), hx(k["p"]), hx(k["q"])


def test_public_nodjn_edges_and_grid_stride():
    from xfl_amd import _native as nat
    n, _, _ = _key()
    n2 = n * n
    dk = nat.DeviceKey(2048, n, None, None, None, device=0)
    rng = random.Random(21)
    count = 40000  # > 1024 blocks x 32 groups: some groups take a second element
    rs = [rng.randrange(1, n) for _ in range(count)]
    ms = [rng.randrange(n) for _ in range(count)]
    edges_r = [1, 2, n - 1, n - 2, (1 << 2047) % n, n // 2]
    edges_m = [0, 1, n - 1, n // 3, n - n // 3, 12345]
    rs[:len(edges_r)] = edges_r
    ms[:len(edges_m)] = edges_m
    ct = nat.words_to_ints(dk.encrypt_words(nat.ints_to_words(ms, dk.nw), nat.ints_to_words(rs, dk.rand_words)))
    check = list(range(len(edges_r))) + rng.sample(range(count), 24) + [32767, 32768, 32769, count - 1]
    for i in check:
        assert ct[i] == (1 + n * ms[i]) * pow(rs[i], n, n2) % n2, i


@pytest.mark.parametrize("invert_first", [False, True])
def test_powmod_edges_and_grid_stride(invert_first):
    from xfl_amd.paillier import PaillierContext, ops
    n, p, q = _key()
    ctx = PaillierContext().init(p, q).to_public()
    n2 = n * n
    rng = random.Random(22)
    count = 36000
    cs = [rng.randrange(1, n2) for _ in range(count)]
    ks = [rng.getrandbits(53) for _ in range(count)]
    edges_c = [1, n2 - 1, n + 1, n2 - n - 1, 2, (1 << 4095) % n2]
    edges_k = [0, 1, 15, 16, (1 << 53) - 1, 1 << 52]
    cs[:6] = edges_c
    ks[:6] = edges_k
    got = ops.powmod(ctx, cs, ks, invert_first=invert_first)
    for i in list(range(6)) + rng.sample(range(count), 24) + [32767, 32768, count - 1]:
        base = pow(cs[i], -1, n2) if invert_first else cs[i]
        assert got[i] == pow(base, ks[i], n2), i


def test_powmod_full_width_exponent():
    """k up to 2048 bits (the negative-branch powers n - k of _raw_mul)"""
    from xfl_amd.paillier import PaillierContext, ops
    n, p, q = _key()
    ctx = PaillierContext().init(p, q).to_public()
    n2 = n * n
    rng = random.Random(23)
    count = 5000
    cs = [rng.randrange(1, n2) for _ in range(count)]
    ks = [rng.randrange(n) for _ in range(count)]
    ks[0], ks[1] = n - 1, 0
    got = ops.powmod(ctx, cs, ks)
    for i in [0, 1, 2, 777, count - 1]:
        assert got[i] == pow(cs[i], ks[i], n2), i
