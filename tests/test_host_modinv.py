"""CPU: the host extended Euclid used for the single inverse at the root of the
device batch inversion (xhe_invert: utils.invert over n^2 for the negative
scalar branch, paillier.py:178,184) agrees with Python's pow(x, -1, m),
including the no-inverse case (ZeroDivisionError in the reference)."""
import os
import random
import subprocess

import pytest

from tests.conftest import FIXTURES, hx, load_fixture

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("modinv") / "modinv_host")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "modinv_host.cpp"), "-o", exe],
                   check=True)
    return exe


def test_modinv_words_matches_python(harness):
    rng = random.Random(11)
    cases = []
    for fx in FIXTURES:
        k = load_fixture(fx)["key"]
        n = hx(k["n"])
        n2 = n * n
        nw = (n2.bit_length() + 31) // 32
        for _ in range(6):
            cases.append((nw, rng.randrange(1, n2), n2))
        cases.append((nw, 1, n2))
        cases.append((nw, n2 - 1, n2))
        cases.append((nw, hx(k["p"]) * rng.randrange(1, 1 << 64), n2))  # shares a factor: no inverse
    inp = "".join(f"{nw} {x:x} {m:x}\n" for nw, x, m in cases)
    out = subprocess.run([harness], input=inp, capture_output=True, text=True, check=True).stdout.split()
    assert len(out) == len(cases)
    for (nw, x, m), got in zip(cases, out):
        try:
            want = f"{pow(x, -1, m):0{8 * nw}x}"
        except ValueError:
            want = "none"
        assert got == want


def test_modinv_words_random_sizes(harness):
    """62-step batches (round 4): random odd moduli of 1..130 words, operands
    of every size below them (the exact path up to 128 bits, the approximate
    one above, the boundary around 2 words), small and structured operands.
    The batched steps must converge on every case: the harness reports how
    often the binary fallback ran, and it must be never."""
    rng = random.Random(12)
    cases = []
    for _ in range(1500):
        nw = rng.choice([1, 2, 3, 4, 5, 8, 16, 33, 64, 96, 128, 130])
        bits = rng.randrange(max(2, 32 * nw - 40), 32 * nw + 1)
        m = rng.getrandbits(bits) | 1 | (1 << (bits - 1))
        kind = rng.randrange(5)
        if kind == 0:
            x = rng.randrange(1, m)
        elif kind == 1:
            x = rng.randrange(1, min(m, 1 << rng.randrange(1, 130)))
        elif kind == 2:
            x = m - rng.randrange(1, min(m, 1 << 20))
        elif kind == 3:
            x = (1 << rng.randrange(0, bits - 1)) % m or 1
        else:
            x = rng.randrange(1, m) | ((1 << (bits - 1)) - 1) % m or 1
        cases.append((nw, x, m))
    inp = "".join(f"{nw} {x:x} {m:x}\n" for nw, x, m in cases)
    r = subprocess.run([harness], input=inp, capture_output=True, text=True, check=True)
    out = r.stdout.split()
    assert len(out) == len(cases)
    for (nw, x, m), got in zip(cases, out):
        try:
            want = f"{pow(x, -1, m):0{8 * nw}x}"
        except ValueError:
            want = "none"
        assert got == want, (nw, hex(x), hex(m))
    assert "fallbacks 0" in r.stderr, r.stderr
