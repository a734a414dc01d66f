"""The base-P digit arithmetic planned for the next kernel step (DESIGN.md §4,
tools/pdigit_model.py): its limb schedule (64-bit lazy columns of 28-bit
limbs, truncated Barrett quotient) is exact mod P^2, no column sum overflows,
and it needs ~35 % fewer multiply-adds than the Montgomery product mod P^2.
CPU, pure Python."""
import random

from tools.pdigit_model import Counter, Digits, random_prime_like


def test_digit_products_exact_and_cheaper():
    rng = random.Random(7)
    for t in range(10):
        P = random_prime_like(1024, rng)
        D = Digits(P)
        P2 = P * P
        edge = [0, 1, P2 - 1, P - 1, P, P2 - P]
        x = edge[t] if t < len(edge) else rng.randrange(P2)
        y = edge[-1 - t] if t < len(edge) else rng.randrange(P2)
        cm, cs = Counter(), Counter()
        z = D.mul(D.split(x), D.split(y), cm)
        s = D.sqr(D.split(x), cs)
        assert z[0] + P * z[1] == x * y % P2 and 0 <= z[0] < P and 0 <= z[1] < P
        assert s[0] + P * s[1] == x * x % P2
        assert max(cm.max_col, cs.max_col) < 1 << 62
    S = 74
    assert cm.mads < 0.66 * (2 * S * S + S)
    assert cs.mads < 0.62 * (S * (S + 1) // 2 + S * S + S)


def test_decrypt_shortcut_low_digit_is_one():
    """c^(P-1) = 1 (mod P) for a prime P, so in digit form the exponentiation's
    result is (1, L) with L the reference's L function of c^(P-1) mod P^2
    (paillier.py:341-368: (x - 1) // p)."""
    P = (1 << 127) - 1  # a Mersenne prime, small enough for a square-and-multiply in Python
    D = Digits(P)
    rng = random.Random(3)
    for _ in range(3):
        c = rng.randrange(2, P * P)
        if c % P == 0:
            continue
        acc = D.split(1)
        base = D.split(c)
        for bit in bin(P - 1)[2:]:
            acc = D.sqr(acc, Counter())
            if bit == "1":
                acc = D.mul(acc, base, Counter())
        x = pow(c, P - 1, P * P)
        assert acc == (1, (x - 1) // P)
