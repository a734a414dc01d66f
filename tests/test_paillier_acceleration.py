"""CPU: xfl_amd.paillier_acceleration (drop-in for
algorithm/core/paillier_acceleration.py) against the reference's packed
fixture (embed output recorded by XFL's own embed) and the oracle restatement,
including negative values, zeros, exact halves and 3-way packing."""
import numpy as np

from oracle import paillier_oracle as O
from tests.conftest import FIXTURES, fl, hx, load_fixture
from xfl_amd.paillier_acceleration import embed, umbed, unpack


def test_embed_matches_reference_fixture():
    c = load_fixture(FIXTURES[0])["encrypt"]["priv_packed_p0"]
    g = np.array([fl(v) for v in c["g"]])
    h = np.array([fl(v) for v in c["h"]])
    assert [int(v) for v in embed([g, h])] == [hx(v) for v in c["input"]]


def test_embed_umbed_vs_restatement():
    rng = np.random.default_rng(5)
    g = np.concatenate([rng.random(200) - 0.5, [0.0, -0.0, 0.5, -0.5, 2.0 ** -70, -(2.0 ** -64), 1 - 2.0 ** -53]])
    h = np.concatenate([(rng.random(200) - 0.2) * 100, [0.0, 1.0, -1.0, 3.0, 2.0 ** -64, 0.25, 7.5]])
    e = [int(v) for v in embed([g, h])]
    assert e == O.embed_ref([g, h])
    sums = [sum(e[:k]) for k in range(1, len(e) + 1, 13)]  # homomorphic-sum-like inputs
    for vals in (e, sums, [-v for v in e]):
        got = umbed(vals, 2)
        want = O.umbed_ref(vals, 2)
        for j in range(2):
            assert np.array_equal(np.array(got[j], np.float32).view(np.uint32),
                                  np.array(want[j], np.float32).view(np.uint32))
    three = [g[:50], h[:50], g[50:100] * 3]
    assert [int(v) for v in embed(three)] == O.embed_ref(three)
    for x in e[:20] + sums[:5]:
        assert unpack(x, 2) == O.unpack_ref(x, 2)
        assert unpack(-x, 3) == O.unpack_ref(-x, 3)
