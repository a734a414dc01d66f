"""Limb-level model of arithmetic mod P^2 in base-P digits (DESIGN.md §4,
"Next: arithmetic mod p^2 in base-p digits"): x = x0 + P x1, 0 <= x0, x1 < P,

    (x0 + P x1)(y0 + P y1) = d0 + P ((d1 + x0 y1 + x1 y0) mod P)   (mod P^2)
    with x0 y0 = d0 + P d1, split by Barrett reduction (HAC 14.42) in
    radix b = 2^28 with a truncated quotient product.

It follows the schedule a kernel would run - 64-bit lazy column sums of 28-bit
limbs, one carry normalisation per product - checks every result against
Python integers, checks that no column sum reaches 2^64, and counts the
32x32->64 multiply-adds (v_mad_u64_u32) per product and per squaring next to
the current Montgomery product mod P^2 (2 S^2 + S, S = 74).

    python tools/pdigit_model.py [--bits 2048] [--trials 300]
"""
import argparse
import json
import random

W = 28
B = 1 << W
MASK = B - 1


def limbs(x, n):
    out = [(x >> (W * i)) & MASK for i in range(n)]
    assert x >> (W * n) == 0, "value does not fit"
    return out


def value(l):
    return sum(v << (W * i) for i, v in enumerate(l))


class Counter:
    def __init__(self):
        self.mads = 0
        self.max_col = 0


def cols_mul(a, b, ctr, lo=0, hi=None, acc=None):
    """lazy column sums of a*b for columns lo..hi-1 (hi default: all)"""
    n = len(a) + len(b) - 1
    hi = n if hi is None else hi
    acc = acc if acc is not None else [0] * (hi - lo)
    for i, ai in enumerate(a):
        for j, bj in enumerate(b):
            c = i + j
            if lo <= c < hi:
                acc[c - lo] += ai * bj
                ctr.mads += 1
    ctr.max_col = max(ctr.max_col, max(acc) if acc else 0)
    return acc


def normalize(cols, n, wrap=False):
    """carry-propagate lazy columns into n limbs (wrap: modulo b^n)"""
    out, carry = [], 0
    for i in range(n):
        x = (cols[i] if i < len(cols) else 0) + carry
        out.append(x & MASK)
        carry = x >> W
    assert wrap or carry == 0, "normalisation overflow"
    return out


class Digits:
    """Z/P^2 Z in base-P digits with Barrett reduction by P."""

    def __init__(self, P):
        self.P = P
        self.k = -(-P.bit_length() // W)          # limbs of P (37 at 1024 bits)
        self.Pl = limbs(P, self.k)
        self.mu = (1 << (W * 2 * self.k)) // P     # floor(b^2k / P)
        self.mul_ = limbs(self.mu, self.k + 1)

    def barrett(self, T, ctr, want_q):
        """(q, r) with T = q P + r, 0 <= r < P, for T < b^2k given as 2k limbs.
        q3 from the columns >= k-1 of q1*mu only (truncated): q - q3 <= 3."""
        k = self.k
        assert len(T) == 2 * k and value(T) < B ** (2 * k)
        q1 = T[k - 1:]                                     # floor(T / b^(k-1)): k+1 limbs
        top = cols_mul(q1, self.mul_, ctr, lo=k - 1)       # columns k-1 .. 2k+1
        # top[i] is column k-1+i: floor(q1 mu / b^(k+1)) = floor(v / b^2)
        v = sum(c << (W * i) for i, c in enumerate(top))
        q3 = v >> (2 * W)
        q3l = limbs(q3, k + 1)
        r2 = normalize(cols_mul(q3l, self.Pl, ctr, hi=k + 1), k + 1, wrap=True)  # (q3 P) mod b^(k+1)
        r = value(T[:k + 1]) - value(r2)
        if r < 0:
            r += B ** (k + 1)
        q, fix = q3, 0
        while r >= self.P:
            r -= self.P
            q += 1
            fix += 1
        assert fix <= 3, f"Barrett needed {fix} corrections"
        ctr.fix = max(getattr(ctr, "fix", 0), fix)
        return (q if want_q else None), r

    def split(self, x):
        return x % self.P, x // self.P

    def mul(self, x, y, ctr):
        (x0, x1), (y0, y1) = x, y
        k = self.k
        a0, a1, b0, b1 = (limbs(v, k) for v in (x0, x1, y0, y1))
        T = normalize(cols_mul(a0, b0, ctr), 2 * k)
        d1, d0 = self.barrett(T, ctr, True)
        U = cols_mul(a0, b1, ctr)
        U = cols_mul(a1, b0, ctr, acc=U)
        U = [u + dl for u, dl in zip(U, limbs(d1, k) + [0] * len(U))]
        ctr.max_col = max(ctr.max_col, max(U))
        U = normalize(U, 2 * k)
        _, z1 = self.barrett(U, ctr, False)
        return d0, z1

    def sqr(self, x, ctr):
        x0, x1 = x
        k = self.k
        a0, a1 = limbs(x0, k), limbs(x1, k)
        # x0^2 by product scanning: i < j pairs doubled, plus the squares
        cols = [0] * (2 * k - 1)
        for i in range(k):
            for j in range(i, k):
                cols[i + j] += a0[i] * a0[j] * (1 if i == j else 2)
                ctr.mads += 1
        ctr.max_col = max(ctr.max_col, max(cols))
        T = normalize(cols, 2 * k)
        d1, d0 = self.barrett(T, ctr, True)
        U = cols_mul(a0, a1, ctr)
        U = [2 * u + dl for u, dl in zip(U, limbs(d1, k) + [0] * len(U))]
        ctr.max_col = max(ctr.max_col, max(U))
        U = normalize(U, 2 * k)
        _, z1 = self.barrett(U, ctr, False)
        return d0, z1


class MontDigits:
    """Z/P^2 Z in MONTGOMERY digits - the form the device kernel runs
    (xfl_amd/csrc/pdigit_dev.hpp PMD): with R = b^k (b = 2^28, k limbs of P),
    a residue x is held as two k-limb integers (a, c) with

        x R^2 = R a + P c   (mod P^2)

    and the product of (a, c) and (e, f) is (a', c') with
        a' = REDC(a e)                  = (a e + m P) / R
        c' = REDC(a f + c e) + (R-1-m) + E,   E = (1 - R) mod P
    where m is the first REDC's quotient (a e = R a' - m P exactly), so that
    R a' + P c' = (R a + P c)(R e + P f) R^-2 (mod P^2). Both REDCs run as one
    operand-scanning loop over the limbs of (e, f) with lazy 64-bit
    accumulators; (R - 1 - m) + E enters limb by limb at the top of the second
    accumulator (limb i of m is known at step i and lands at weight b^i).
    Each step: k mads e_i*a + k mads m_i*P (first) and 3k mads e_i*c + f_i*a +
    m'_i*P (second): 5k^2 per product vs 2(2k)^2 for Montgomery mod P^2."""

    def __init__(self, P):
        self.P = P
        self.k = -(-P.bit_length() // W)
        self.R = 1 << (W * self.k)
        self.Pl = limbs(P, self.k)
        self.n0inv = (-pow(P, -1, B)) % B
        self.E = (1 - self.R) % P
        self.El = limbs(self.E, self.k)

    def to_form(self, x):
        """(a, c) with R a + P c = x R^2 mod P^2, a, c < P"""
        P, R = self.P, self.R
        X = x * R * R % (P * P)
        a = X * pow(R, -1, P) % P
        c = ((X - R * a) // P) % P  # exact: X = R a (mod P)
        return a, c

    def value(self, a, c):
        P2 = self.P * self.P
        return (self.R * a + self.P * c) * pow(self.R, -2, P2) % P2

    def mul(self, x, y, ctr):
        """one product, as the kernel's step schedule; returns (a', c')"""
        k, P = self.k, self.P
        (a, c), (e, f) = x, y
        al, cl = limbs_loose(a, k), limbs_loose(c, k)
        el, fl = limbs(e, k), limbs(f, k)
        T1 = [0] * k
        T2 = [0] * k
        for i in range(k):
            # position 0 first: the quotient digits
            x1 = T1[0] + el[i] * al[0]
            m1 = (x1 * self.n0inv) & MASK
            x1 += m1 * self.Pl[0]
            x2 = T2[0] + el[i] * cl[0] + fl[i] * al[0]
            m2 = (x2 * self.n0inv) & MASK
            x2 += m2 * self.Pl[0]
            assert x1 & MASK == 0 and x2 & MASK == 0
            ctr.mads += 5
            for j in range(1, k):
                T1[j - 1] = T1[j] + el[i] * al[j] + m1 * self.Pl[j]
                T2[j - 1] = T2[j] + el[i] * cl[j] + fl[i] * al[j] + m2 * self.Pl[j]
                ctr.mads += 5
            T1[k - 1] = 0
            T2[k - 1] = (MASK - m1) + self.El[i]
            T1[0] += x1 >> W
            T2[0] += x2 >> W
            ctr.max_col = max(ctr.max_col, max(T1), max(T2))
        a2 = _norm_value(T1)
        c2 = _norm_value(T2)
        return a2, c2


def limbs_loose(x, n):
    """limbs with the top one unmasked (values up to ~b^n * 2)"""
    out = [(x >> (W * i)) & MASK for i in range(n - 1)]
    out.append(x >> (W * (n - 1)))
    assert out[-1] < (1 << 32)
    return out


def _norm_value(T):
    return sum(t << (W * i) for i, t in enumerate(T))


def mont_digits_check(bits, trials, rng):
    worst, amax, cmax = 0, 0, 0
    for t in range(trials):
        P = random_prime_like(bits // 2, rng)
        D = MontDigits(P)
        P2 = P * P
        x = rng.randrange(P2)
        state = D.to_form(x)
        acc = x
        for s in range(6):  # a chain, as the fixed-base loop runs it
            y = rng.randrange(P2)
            ctr = Counter()
            state = D.mul(state, D.to_form(y), ctr)
            acc = acc * y % P2
            assert D.value(*state) == acc, "Montgomery-digit product wrong"
            worst = max(worst, ctr.max_col)
            amax = max(amax, state[0] / P)
            cmax = max(cmax, (state[1] - D.R) / P)
            assert state[1] < (1 << (W * D.k + 1)), "second digit outgrew its top limb"
    return {"mont_digit_mads_per_product": ctr.mads, "mont_digit_product_ratio": ctr.mads / (2 * (2 * D.k) ** 2),
            "mont_digit_max_column_log2": worst.bit_length(), "mont_digit_a_over_P": amax,
            "mont_digit_c_minus_R_over_P": cmax, "mont_digit_chain_trials": trials}


def random_prime_like(bits, rng):
    """an odd number with the top bit set (primality is irrelevant to the
    arithmetic being modelled)"""
    return rng.getrandbits(bits) | (1 << (bits - 1)) | 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=2048, help="key size; P has bits/2 bits")
    ap.add_argument("--trials", type=int, default=300)
    args = ap.parse_args()
    rng = random.Random(1)
    res = {"bits": args.bits}
    worst_col = 0
    fix = 0
    for t in range(args.trials):
        P = random_prime_like(args.bits // 2, rng)
        D = Digits(P)
        P2 = P * P
        edge = [0, 1, P2 - 1, P2 - P, P - 1, P]
        x = edge[t % len(edge)] if t < 12 else rng.randrange(P2)
        y = edge[(t // 2) % len(edge)] if t < 12 else rng.randrange(P2)
        cm, cs = Counter(), Counter()
        z = D.mul(D.split(x), D.split(y), cm)
        assert z[0] + P * z[1] == x * y % P2
        s = D.sqr(D.split(x), cs)
        assert s[0] + P * s[1] == x * x % P2
        worst_col = max(worst_col, cm.max_col, cs.max_col)
        fix = max(fix, getattr(cm, "fix", 0), getattr(cs, "fix", 0))
        res["mads_per_product"] = cm.mads
        res["mads_per_squaring"] = cs.mads
        res["k_limbs"] = D.k
    S = -(-args.bits // W)
    res["montgomery_mod_P2_mads"] = 2 * S * S + S
    res["montgomery_square_mads"] = S * (S + 1) // 2 + S * S + S
    res["product_ratio"] = res["mads_per_product"] / res["montgomery_mod_P2_mads"]
    res["squaring_ratio"] = res["mads_per_squaring"] / res["montgomery_square_mads"]
    res["max_column_sum_log2"] = worst_col.bit_length()
    res["max_barrett_corrections"] = fix
    res["trials_bit_exact"] = args.trials
    assert worst_col < (1 << 64)
    res.update(mont_digits_check(args.bits, max(4, args.trials // 10), rng))
    assert res["mont_digit_max_column_log2"] <= 64
    print(json.dumps(res))


if __name__ == "__main__":
    main()


# ---------------------------------------------------------------------------
# Montgomery digits mod n^2 (n = p q, public): the same product with the
# modulus n, W = 27-bit limbs and K = 80 (R = 2^2160 > 2^100 n at 2048 bits;
# 28-bit limbs would overflow the 64-bit lazy columns at K > 41), plus the
# conversions a kernel needs from and to plain residues mod n^2:
#   in:  X = x + ceil(R/n) n^2  (= x mod n^2, and REDC(X) = t lands in [n, 2n+))
#        REDC(X): X + m n = R t  ->  (t - n, R - m) are the digits of x R^-2
#        (R (t - n) + n (R - m) = X - R n ... = x + ceil(R/n) n^2 - R n + ...;
#        exactly: R(t-n) + n(R-m) = R t - n m = X == x (mod n^2)), then one
#        digit product by the digits of R^2 mod n^2 (a constant row) -> x
#   out: y0 = REDC(a) (quotient m_a, delta = [REDC(a) >= n]),
#        y1 = (REDC(REDC(c) - m_a + R n) + delta) mod n,   y = y0 + n y1
class NDigits(MontDigits):
    def __init__(self, n, W_=27, K=None):
        self.W = W_
        self.B = 1 << W_
        self.MASK = self.B - 1
        self.P = n
        self.k = K or -(-(n.bit_length() + 13) // W_)
        self.R = 1 << (W_ * self.k)
        self.n0inv = (-pow(n, -1, self.B)) % self.B
        self.E = (1 - self.R) % n
        self.Kn2 = -(-self.R // n) * n * n
        # digits of R^2 mod n^2 (the input conversion's constant row)
        X4 = pow(self.R, 4, n * n)
        e = X4 * pow(self.R, -1, n) % n
        self.w = (e, ((X4 - self.R * e) // n) % n)

    def limbs(self, x):
        out = [(x >> (self.W * i)) & self.MASK for i in range(self.k - 1)]
        out.append(x >> (self.W * (self.k - 1)))
        assert out[-1] < (1 << 32), "top limb overflows 32 bits"
        return out

    def redc(self, T, nlimbs, ctr):
        """operand-scanning REDC of an nlimbs-limb value (lazy columns):
        returns (t, m) with value + m n = R t"""
        n, W_ = self.P, self.W
        cols = [(T >> (W_ * i)) & self.MASK for i in range(nlimbs)]
        cols[-1] = T >> (W_ * (nlimbs - 1))
        cols += [0] * max(0, 2 * self.k - nlimbs)
        m = 0
        nl = [(n >> (W_ * j)) & self.MASK for j in range(self.k)]
        carry = 0
        for i in range(self.k):
            x = cols[i] + carry
            mi = (x * self.n0inv) & self.MASK
            m |= mi << (W_ * i)
            x += mi * nl[0]
            assert x & self.MASK == 0
            carry = x >> W_
            for j in range(1, self.k):
                cols[i + j] += mi * nl[j]
                ctr.max_col = max(ctr.max_col, cols[i + j])
            ctr.mads += self.k
        rest = sum(cols[i] << (W_ * (i - self.k)) for i in range(self.k, len(cols))) + carry
        assert (T + m * n) == rest * self.R
        return rest, m

    def mul(self, x, y, ctr):
        """MontDigits.mul with this W (limbs_loose for the state)"""
        k, n, W_ = self.k, self.P, self.W
        (a, c), (e, f) = x, y
        al, cl, el, fl = self.limbs(a), self.limbs(c), self.limbs(e), self.limbs(f)
        nl = [(n >> (W_ * j)) & self.MASK for j in range(k)]
        El = [(self.E >> (W_ * j)) & self.MASK for j in range(k)]
        T1, T2 = [0] * k, [0] * k
        for i in range(k):
            x1 = T1[0] + el[i] * al[0]
            m1 = (x1 * self.n0inv) & self.MASK
            x1 += m1 * nl[0]
            x2 = T2[0] + el[i] * cl[0] + fl[i] * al[0]
            m2 = (x2 * self.n0inv) & self.MASK
            x2 += m2 * nl[0]
            assert x1 & self.MASK == 0 and x2 & self.MASK == 0
            for j in range(1, k):
                T1[j - 1] = T1[j] + el[i] * al[j] + m1 * nl[j]
                T2[j - 1] = T2[j] + el[i] * cl[j] + fl[i] * al[j] + m2 * nl[j]
            ctr.mads += 5 * k
            T1[k - 1] = 0
            T2[k - 1] = (self.MASK - m1) + El[i]
            T1[0] += x1 >> W_
            T2[0] += x2 >> W_
            ctr.max_col = max(ctr.max_col, max(T1), max(T2))
        return (sum(t << (W_ * i) for i, t in enumerate(T1)), sum(t << (W_ * i) for i, t in enumerate(T2)))

    def to_digits(self, x, ctr):
        t, m = self.redc(x + self.Kn2, 2 * self.k + 1, ctr)
        assert self.P <= t < 2 * self.P + 2, "REDC(x + Kn2) left [n, 2n]"
        return self.mul((t - self.P, self.R - m), self.w, ctr)

    def from_digits(self, a, c, ctr):
        n = self.P
        ta, ma = self.redc(a, self.k, ctr)
        assert ta <= n
        delta = 1 if ta >= n else 0
        y0 = ta - delta * n
        u, _ = self.redc(c, self.k, ctr)
        tw, _ = self.redc(u - ma + self.R * n, 2 * self.k, ctr)
        y1 = (tw + delta) % n
        assert tw + delta < 3 * n
        return y0 + n * y1


def ndigits_check(bits, trials, rng):
    worst = 0
    for t in range(trials):
        n = random_prime_like(bits // 2, rng) * random_prime_like(bits // 2, rng)
        D = NDigits(n)
        n2 = n * n
        ctr = Counter()
        x = rng.randrange(n2) if t % 3 else rng.randrange(n)
        st = D.to_digits(x, ctr)
        assert D.value(*st) == x, "input conversion"
        acc = x
        for s in range(5):
            if s % 2:
                st = D.mul(st, st, ctr)  # squaring: the state as its own operand
                acc = acc * acc % n2
            else:
                y = rng.randrange(n2)
                st = D.mul(st, D.to_digits(y, ctr), ctr)
                acc = acc * y % n2
            assert D.value(*st) == acc
            assert st[0] < 2 * n and st[1] < D.R + 6 * n, "state bounds"
        assert D.from_digits(*st, ctr) == acc, "output conversion"
        worst = max(worst, ctr.max_col)
    return {"ndigit_K": D.k, "ndigit_W": D.W, "ndigit_max_column_log2": worst.bit_length(),
            "ndigit_trials": trials}
