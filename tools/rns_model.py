"""Limb-level model of the RNS Montgomery exponentiation planned for the
small-batch decrypt (k_dec_rns): x^(P-1) mod P^2 with every product done in a
residue number system - two bases B, B' of K 28-bit primes and a redundant
channel mod 2^32 - so a product is two all-to-all exchanges (base
extensions) instead of WaveMont's six LDS column phases.

Per product of x, y (each given in B, B' and mod 2^32, value < LAM N):
  t = x y per channel
  xi_i  = t_i |-N^-1 M_i^-1|_{m_i}                      (B)
  qh'_j = sum_i xi_i |M_i|_{m'_j}  mod m'_j              (B': fast extension, qh = q + alpha M, alpha < K)
  qh_r  = sum_i xi_i |M_i|_{2^32}  mod 2^32              (redundant channel)
  r'_j  = (t'_j + qh'_j N) |M^-1|_{m'_j}                 (B')
  r_r   = (t_r + qh_r N) M^-1 mod 2^32                   (exact: r = (t + qh N) / M is an integer)
  xi'_j = r'_j |M'_j^-1|_{m'_j}                          (B')
  beta  = (sum_j xi'_j |M'_j|_{2^32} - r_r) M'^-1 mod 2^32    (exact: Shenoy-Kumaresan)
  r_i   = sum_j xi'_j |M'_j|_{m_i} - beta |M'|_{m_i}    (B: exact extension)
r = x y M^-1 mod N, r < LAM N when M >= (K+1)^2 N (LAM = K + 1).

The model checks every bound the kernel relies on (64-bit column sums, the
Barrett reductions' quotient estimates, alpha / beta ranges, the closure
r < LAM N) on random inputs and on whole exponentiations against pow().
    python tools/rns_model.py [--keys 3] [--products 2000]
"""
import argparse
import random

W = 28
K = 74           # moduli per base: M, M' ~ 2^2071 >= (K + 1)^2 2^2048
LAM = K + 1      # every RNS value stays below LAM * N


def primes_below(limit, count):
    """the `count` largest primes below `limit` (deterministic Miller-Rabin for < 2^64)"""
    out = []
    c = limit - 1
    while len(out) < count:
        if c % 2 and is_prime(c):
            out.append(c)
        c -= 1
    return out


def is_prime(n):
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
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


PR = primes_below(1 << W, 2 * K)
B, B2 = PR[0::2], PR[1::2]   # interleaved so both products are alike
M = 1
for m in B:
    M *= m
M2 = 1
for m in B2:
    M2 *= m
R32 = 1 << 32


class Key:
    """the per-key constants the kernel reads (N = P^2)"""

    def __init__(self, P):
        N = P * P
        self.P, self.N = P, N
        assert M >= (K + 1) ** 2 * N and M2 >= LAM * N, "bases too small"
        self.c1 = [(-pow(N, -1, m) * pow(M // m, -1, m)) % m for m in B]
        self.NB2 = [N % m for m in B2]
        self.Nr = N % R32
        self.Minv2 = [pow(M, -1, m) for m in B2]
        self.Mrinv = pow(M, -1, R32)
        self.M2i_inv = [pow(M2 // m, -1, m) for m in B2]
        self.C = [[(M // mi) % mj for mi in B] for mj in B2]     # row j: |M_i|_{m'_j}
        self.E = [(M // mi) % R32 for mi in B]
        self.C2 = [[(M2 // mj) % mi for mj in B2] for mi in B]   # row i: |M'_j|_{m_i}
        self.D = [(M2 // mj) % R32 for mj in B2]
        self.M2B = [M2 % mi for mi in B]
        self.M2rinv = pow(M2, -1, R32)


def to_rns(x):
    return [x % m for m in B], [x % m for m in B2], x % R32


def from_rns(v):
    """exact value from the B residues + the redundant channel (the kernel's exit)"""
    xb, _, xr = v
    xi = [(xb[i] * pow(M // B[i], -1, B[i])) % B[i] for i in range(K)]
    s = sum(xi[i] * (M // B[i]) for i in range(K))
    alpha = ((sum(xi[i] * ((M // B[i]) % R32) for i in range(K)) - xr) * pow(M, -1, R32)) % R32
    assert alpha < K
    return s - alpha * M


def mont(k, x, y, stats):
    xb, xb2, xr = x
    yb, yb2, yr = y
    t = [a * b % m for a, b, m in zip(xb, yb, B)]
    t2 = [a * b % m for a, b, m in zip(xb2, yb2, B2)]
    tr = xr * yr % R32
    xi = [ti * c % m for ti, c, m in zip(t, k.c1, B)]
    # B': fast extension of qh = sum xi_i M_i (64-bit column sums)
    r2, xi2 = [], []
    for j, mj in enumerate(B2):
        acc = sum(xi[i] * k.C[j][i] for i in range(K))
        stats["acc_max"] = max(stats["acc_max"], acc)
        qh = acc % mj
        rj = (t2[j] + qh * k.NB2[j]) * k.Minv2[j] % mj
        r2.append(rj)
        xi2.append(rj * k.M2i_inv[j] % mj)
    qhr = sum(xi[i] * k.E[i] for i in range(K)) % R32
    rr = (tr + qhr * k.Nr) * k.Mrinv % R32
    # B: exact extension from B'
    S = sum(xi2[j] * k.D[j] for j in range(K)) % R32
    beta = (S - rr) * k.M2rinv % R32
    assert beta < K, beta
    stats["beta_max"] = max(stats["beta_max"], beta)
    rb = []
    for i, mi in enumerate(B):
        acc = sum(xi2[j] * k.C2[i][j] for j in range(K))
        stats["acc_max"] = max(stats["acc_max"], acc)
        rb.append((acc - beta * k.M2B[i]) % mi)
    return rb, r2, rr


def check_product(k, x, y, stats):
    r = mont(k, to_rns(x), to_rns(y), stats)
    v = from_rns(r)
    # the three representations are one integer, congruent to x y M^-1, below LAM N
    assert r[1] == [v % m for m in B2] and r[2] == v % R32
    assert v % k.N == x * y * pow(M, -1, k.N) % k.N
    assert v < LAM * k.N, (v // k.N)
    stats["ratio_max"] = max(stats["ratio_max"], v / k.N)
    return v


def powmod_rns(k, c, e):
    """c^e mod N by left-to-right square-and-multiply in RNS Montgomery form
    (entry: REDC(c) then * M^3; exit: * 1, then exact reduction mod N)"""
    stats = {"acc_max": 0, "beta_max": 0, "ratio_max": 0}
    N = k.N
    x = mont(k, to_rns(c), to_rns(1), stats)                 # c M^-1 (c < 2^4096 < M N)
    x = mont(k, x, to_rns(pow(M, 3, N)), stats)              # c M
    acc = x
    for bit in bin(e)[3:]:
        acc = mont(k, acc, acc, stats)
        if bit == "1":
            acc = mont(k, acc, x, stats)
    v = from_rns(mont(k, acc, to_rns(1), stats))
    assert v < LAM * N
    return v % N, stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=2)
    ap.add_argument("--products", type=int, default=300)
    ap.add_argument("--ops", action="store_true", help="also check the kernel's channel arithmetic")
    args = ap.parse_args()
    rng = random.Random(5)
    print(f"K={K} moduli of {W} bits per base: M ~ 2^{M.bit_length()}, M' ~ 2^{M2.bit_length()}")
    for _ in range(args.keys):
        while True:
            P = rng.getrandbits(1024) | (1 << 1023) | 1
            if is_prime(P):
                break
        k = Key(P)
        N = k.N
        stats = {"acc_max": 0, "beta_max": 0, "ratio_max": 0}
        edge = [0, 1, N - 1, LAM * N - 1, (LAM - 1) * N]
        for t in range(args.products):
            x = edge[t % len(edge)] if t < 25 else rng.randrange(LAM * N)
            y = edge[(t // len(edge)) % len(edge)] if t < 25 else rng.randrange(LAM * N)
            check_product(k, x, y, stats)
        c = rng.getrandbits(4096)
        v, st2 = powmod_rns(k, c, P - 1)
        assert v == pow(c, P - 1, N)
        print(f"key ok: acc max 2^{stats['acc_max'].bit_length()} (< 2^64), beta max {stats['beta_max']}, "
              f"r/N max {stats['ratio_max']:.2f} (< {LAM}); c^(P-1) mod P^2 exact, exp r/N max {st2['ratio_max']:.2f}")


if __name__ == "__main__":
    main()


# ---- the kernel's channel arithmetic (32-bit registers), checked exhaustively
# at the edges and on random operands for every modulus
U32 = (1 << 32) - 1


def k_red(x, m, mu):
    """x < 2^59 -> x mod m: q = mulhi(x >> 27, mu), r = lo32(x) - q m, three min-corrections"""
    assert x < 1 << 59
    q = ((x >> 27) * mu) >> 32
    r = (x - q * m) & U32
    for _ in range(3):
        r = min(r, (r - m) & U32)
    return r


def k_red64(x, m, mu, t32):
    """x < 2^63 (the 74-term column sums): fold the high word by 2^32 mod m first"""
    assert x < 1 << 63
    return k_red((x >> 32) * t32 + (x & U32), m, mu)


def check_channel_ops(rng, n=20000):
    for m in B + B2:
        mu = (1 << 59) // m
        assert (1 << 31) < mu < (1 << 32)
        t32 = (1 << 32) % m
        for x in [0, 1, m - 1, m, (m - 1) ** 2, (1 << 59) - 1] + [rng.randrange(1 << 59) for _ in range(n // 100)]:
            assert k_red(x, m, mu) == x % m, (m, x)
        for x in [(1 << 63) - 1, 74 * (m - 1) ** 2] + [rng.randrange(1 << 63) for _ in range(n // 100)]:
            assert k_red64(x, m, mu, t32) == x % m, (m, x)
    print("channel arithmetic: Barrett reductions exact for every modulus")


if __name__ == "__main__" and "--ops" in __import__("sys").argv:
    check_channel_ops(random.Random(9))
