"""Limb-level model of k_add_barrett (the one-product ciphertext add mod n^2),
checked against Python integers before the kernel is written.

c = x y mod N, N = n^2 (K = 4096 bits at 2048-bit keys), 27-bit limbs
(beta = 2^27, S = 152 limbs: N < beta^S, N >= beta^(S-1)), Barrett (HAC
14.42) with product-scanning column sums:

  T  = x y                                 all 2S columns
  q1 = floor(T / beta^(S-1))               T's limbs S-1 .. 2S-1
  q2 = q1 mu (mu = floor(beta^(2S) / N))   only columns >= 148 (truncated)
  q3 = floor(q2 / beta^(S+1))
  r  = (T - q3 N) mod beta^(S+1)           only columns <= S of q3 N
  while r >= N: r -= N

Every column is a lazy 64-bit sum of 27x27-bit products (at most S+1 terms
< 2^54, < 2^62), normalised in rounds of 32 columns as
the kernel does (8 lanes x 4 columns per round): each lane carries its 4
columns locally, hands its carry to the next lane, and the round's carry goes
to the next round. The model asserts
every column sum < 2^64 and records how many final subtractions were needed.

    python tools/barrett_model.py [trials]
"""
import random
import sys

W = 27
BETA = 1 << W
MASK = BETA - 1


def limbs(v, n):
    out = []
    for _ in range(n):
        out.append(v & MASK)
        v >>= W
    assert v == 0, "value does not fit"
    return out


def value(ls):
    return sum(l << (W * i) for i, l in enumerate(ls))


def columns(a, b, lo, hi):
    """Column sums c in [lo, hi) of the product of limb lists a, b."""
    out = []
    for c in range(lo, hi):
        s = 0
        for i in range(max(0, c - len(b) + 1), min(c, len(a) - 1) + 1):
            s += a[i] * b[c - i]
        assert s < 1 << 64, "column overflow"
        out.append(s)
    return out


LANES = 8          # lanes per element (bar::G)
ROUND = 4 * LANES  # columns per round
B0 = 148           # first column of q1 mu computed (bar::B0 = S - 4)


def normalise_rounds(cols, carry_in=0, round_cols=ROUND, lanes=LANES):
    """The kernel's normalisation: rounds of lanes x (round_cols/lanes) columns;
    within a lane a sequential carry, then lane to lane, then round to round.
    Returns (limbs, final carry)."""
    per = round_cols // lanes
    out = []
    carry = carry_in
    for r0 in range(0, len(cols), round_cols):
        rc = cols[r0:r0 + round_cols]
        # pass 1: each lane alone
        lane_limbs, lane_c = [], []
        for g in range(lanes):
            c = 0
            ls = []
            for s in rc[g * per:(g + 1) * per]:
                x = s + c
                ls.append(x & MASK)
                c = x >> W
            lane_limbs.append(ls)
            lane_c.append(c)
            assert c < 1 << 40
        # pass 2: predecessor's carry (lane 0: the previous round's), then ripple
        cin = [carry] + lane_c[:-1]
        ripple = 0
        for g in range(lanes):
            c = cin[g] + ripple
            ls = lane_limbs[g]
            for k in range(len(ls)):
                x = ls[k] + c
                ls[k] = x & MASK
                c = x >> W
            ripple = c  # the lane's own big carry was handed on already
            out += ls
        carry = lane_c[-1] + ripple
    return out, carry


def barrett_mul(x, y, N, S, lo=B0):
    mu = (1 << (2 * W * S)) // N
    xl, yl = limbs(x, S), limbs(y, S)
    # T = x y: 2S columns, normalised limb by limb
    T, c = normalise_rounds(columns(xl, yl, 0, 2 * S))
    assert c == 0 and value(T) == x * y
    q1 = T[S - 1:2 * S]                      # S+1 limbs
    ml = limbs(mu, S + 1)
    q2c = columns(q1, ml, lo, 2 * S + 2)   # truncated: columns >= lo
    pad = (-len(q2c)) % ROUND
    q2, c2 = normalise_rounds(q2c + [0] * pad)
    q2v = value(q2) + (c2 << (W * len(q2)))  # = floor-truncated q2 / beta^lo
    q3 = q2v >> (W * (S + 1 - lo))
    true_q3 = ((x * y) // (1 << (W * (S - 1))) * mu) >> (W * (S + 1))
    assert true_q3 - 1 <= q3 <= true_q3, (q3, true_q3)
    q3l = limbs(q3, S + 1)
    nl = limbs(N, S)
    r2c = columns(q3l, nl, 0, S + 1)
    pad = (-len(r2c)) % ROUND
    r2, _ = normalise_rounds(r2c + [0] * pad)
    r2 = r2[:S + 1]
    mod = 1 << (W * (S + 1))
    r = (value(T[:S + 1]) - value(r2)) % mod
    assert r == (x * y - q3 * N), "r is T - q3 N exactly (it is below beta^(S+1))"
    subs = 0
    while r >= N:
        r -= N
        subs += 1
    assert r == x * y % N
    return r, subs


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = random.Random(1)
    S = 152
    worst = 0
    for t in range(trials):
        bits = rng.choice([4095, 4096])
        n_ = rng.getrandbits(bits // 2) | (1 << (bits // 2 - 1)) | 1
        N = n_ * n_
        if t % 4 == 0:
            x, y = N - 1, N - 1
        else:
            x, y = rng.randrange(N), rng.randrange(N)
        _, subs = barrett_mul(x, y, N, S)
        worst = max(worst, subs)
    print(f"{trials} products bit-exact; at most {worst} final subtractions")


if __name__ == "__main__":
    main()
