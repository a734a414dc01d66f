"""The one-product ciphertext add (k_add_barrett: product scanning + Barrett
reduction mod n^2, 2048-bit keys, equal exponents, batches in the 4-lane
regime) against Python's integers: c = a b mod n^2 (paillier.py:106-123,
153-154), for random residues, the edge values that drive Barrett's quotient
estimate to its limits (n^2 - 1 squared, 1, 0, values just below powers of
2^27 and operands >= n^2 up to 2^4096 - 1), and in the drop-in's resident
PaillierArray + PaillierArray (config 3's pairwise sum)."""
import random

import numpy as np
import pytest

from tests.conftest import hx, load_fixture

pytestmark = pytest.mark.gpu

COUNT = 6000  # above kN2RowMax (4096): the 4-lane regime


def _ctx(fx):
    from xfl_amd.paillier import PaillierContext
    k = load_fixture(fx)["key"]
    return PaillierContext().init(hx(k["p"]), hx(k["q"]))


def _edge(n2):
    top = (1 << 4096) - 1
    e = [0, 1, 2, n2 - 1, n2 - 2, n2 // 2, top, top - 1, n2, n2 + 1]
    e += [(1 << (27 * k)) - 1 for k in (1, 75, 150, 151)]
    e += [n2 - (1 << (27 * k)) for k in (1, 100, 150)]
    return e


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_2048_nodjn.json"])
def test_add_barrett_vs_python(fx):
    import torch

    from xfl_amd import _native as nat
    from xfl_amd.paillier import resident
    ctx = _ctx(fx)
    dk = ctx.device_key()
    n2 = ctx.n_square
    rng = random.Random(7)
    a = [rng.randrange(n2) for _ in range(COUNT)]
    b = [rng.randrange(n2) for _ in range(COUNT)]
    edge = _edge(n2)
    for i, x in enumerate(edge):  # every edge value against every other one, and squared
        for j, y in enumerate(edge):
            a[len(edge) * i + j], b[len(edge) * i + j] = x, y
    a[-1], b[-1] = n2 - 1, n2 - 1
    dev = dk.device
    da = resident.upload(nat.ints_to_words(a, dk.n2w), dev)
    db = resident.upload(nat.ints_to_words(b, dk.n2w), dev)
    ea = np.arange(COUNT, dtype=np.int32) % 5 - 40
    out = resident.mulmod(dk, da, ea, db, ea.copy(), 0)
    got = nat.words_to_ints(resident.download(out))
    bad = [i for i in range(COUNT) if got[i] != a[i] * b[i] % n2]
    assert not bad, f"{len(bad)} wrong, first {bad[:5]}"
    # the exponents come back as min(ea, eb) = ea
    eo = torch.empty(COUNT, dtype=torch.int32, device=f"cuda:{dev}")
    L = nat.lib()
    da_e = resident.upload(ea, dev)
    nat.check(L.xhe_mulmod(dk.handle, resident._dp(da), resident._dp(da_e), resident._dp(db), resident._dp(da_e),
                           COUNT, 0, resident._dp(out), resident._dp(eo), resident._sp(dev)), "mulmod")
    torch.cuda.synchronize(dev)  # (the library ran on the drop-in's stream)
    assert np.array_equal(eo.cpu().numpy(), ea)
    assert nat.words_to_ints(resident.download(out)) == got


def test_add_barrett_dropin_pairwise_sum():
    """config 3's pairwise sum c + d on resident arrays of 20 k float32
    gradients decrypts to the sums (the kernel inside the drop-in path)."""
    from xfl_amd.paillier import Paillier
    ctx = _ctx("paillier_2048_djn.json")
    rng = np.random.default_rng(9)
    x = rng.standard_normal(20000).astype(np.float32)
    y = rng.standard_normal(20000).astype(np.float32)
    ex = Paillier.encrypt(ctx, x, precision=7)
    ey = Paillier.encrypt(ctx, y, precision=7)
    s = ex + ey
    assert s.is_resident
    got = Paillier.decrypt(ctx, s)
    assert np.allclose(got, x.astype(np.float64) + y, rtol=1e-6, atol=2e-7)
