"""Batch inversion mod n^2 (xhe_invert: PaillierCiphertext._raw_mul's
invert branch, paillier.py:173-187, utils.py:71-76) across the batch sizes
of its shapes - the whole-block product tree (2048-bit keys, up to 256
elements, k_wtree_*) and the level-by-level tree of larger batches - against
Python's pow(c, -1, n^2), with odd sizes (lone children at every level) and
edge residues; a non-invertible element fails with XHE_ENOINV."""
import random

import numpy as np
import pytest

from tests.conftest import hx, load_fixture

pytestmark = pytest.mark.gpu


def _run(counts, seed=7):
    import torch

    from xfl_amd import _native as nat
    k = load_fixture("paillier_2048_djn.json")["key"]
    n, p = hx(k["n"]), hx(k["p"])
    n2 = n * n
    dk = nat.DeviceKey(2048, n, None, None, None, device=0)
    L = nat.lib()
    rng = random.Random(seed)
    s = torch.cuda.current_stream().cuda_stream
    for count in counts:
        cs = [rng.randrange(1, n2) for _ in range(count)]
        edges = [1, n2 - 1, n + 1, 2, (1 << 4095) % n2]
        cs[:min(count, len(edges))] = edges[:count]
        cs = [c if c % p and c % (n // p) else c + 1 for c in cs]
        dc = torch.from_numpy(nat.ints_to_words(cs, dk.n2w).view(np.int32).copy()).cuda()
        out = torch.empty_like(dc)
        nat.check(L.xhe_invert(dk.handle, dc.data_ptr(), count, out.data_ptr(), s), "invert")
        torch.cuda.synchronize()
        got = nat.words_to_ints(out.cpu().numpy().view(np.uint32))
        for i, (c, g) in enumerate(zip(cs, got)):
            assert g == pow(c, -1, n2), (count, i)
    # an element sharing the factor p has no inverse
    bad = torch.from_numpy(nat.ints_to_words([3, p * 5, 7], dk.n2w).view(np.int32).copy()).cuda()
    out = torch.empty_like(bad)
    assert L.xhe_invert(dk.handle, bad.data_ptr(), 3, out.data_ptr(), s) == nat.XHE_ENOINV


@pytest.mark.parametrize("counts", [[1, 2, 3, 7, 64], [129, 255, 256], [257, 1000]])
def test_invert_batch_sizes(counts):
    _run(counts)

