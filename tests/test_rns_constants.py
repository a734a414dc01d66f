"""CPU: the small-batch decrypt's RNS constants (xhe_rns_constants, the blocks
k_dec_rns reads; rns_dev.hpp) against tools/rns_model.py, and the kernel's
per-thread algorithm - every channel's Barrett arithmetic, the two base
extensions per product, the DPP partial sums, the exit's columns and the
reduction mod P^2 - emulated in numpy on those blocks, through a whole
c^(P-1) mod P^2 against Python's pow. The model itself is checked against
Python integers (bounds, exactness) by its own asserts."""
import ctypes
import os
import sys

import numpy as np
import pytest

from tests.conftest import hx, load_fixture

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

RK, RKP, NT, RLANE = 74, 76, 256, 202
S_M, S_MU, S_T32, S_B, S_C, S_D, S_ROWS = 0, 256, 512, 768, 1024, 1280, 1536
S_MPOS = S_ROWS + RKP * NT
S_MFULL = S_MPOS + RK * RKP
S_M2RINV = S_MFULL + RKP
P_A, P_A2, P_M3, P_NS, P_SCHED, P_SCHED_MAX = 0, 256, 512, 768, 772, 1280
P_WORDS = P_SCHED + P_SCHED_MAX + 4
U32 = (1 << 32) - 1


def _blocks(P):
    from xfl_amd import _native as nat
    L = nat.lib()
    pw = nat.ints_to_words([P], (P.bit_length() + 31) // 32)[0]
    sh = np.zeros(26696, np.uint32)
    pb = np.zeros(P_WORDS, np.uint32)
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    nat.check(L.xhe_rns_constants(vp(pw), pw.shape[0], vp(sh), vp(pb)), "rns constants")
    return sh, pb


@pytest.fixture(scope="module")
def model():
    import rns_model
    return rns_model


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_2048_nodjn.json"])
def test_constants_match_model(model, fx):
    k = load_fixture(fx)["key"]
    for P in (hx(k["p"]), hx(k["q"])):
        sh, pb = _blocks(P)
        mk = model.Key(P)
        for t in range(NT):
            gB, ch = t < 128, (t if t < 128 else t - 128)
            if t == RLANE:
                assert sh[S_M + t] == 0 and [int(sh[S_ROWS + i * NT + t]) for i in range(RK)] == mk.E
                assert sh[S_B + t] == mk.Mrinv and pb[P_A + t] == mk.Nr and pb[P_M3 + t] == pow(model.M, 3, mk.N) % 2 ** 32
                continue
            if ch >= RK:
                assert sh[S_M + t] == 0 and not any(sh[S_ROWS + i * NT + t] for i in range(RKP))
                continue
            m = model.B[ch] if gB else model.B2[ch]
            assert sh[S_M + t] == m and sh[S_MU + t] == (1 << 59) // m and sh[S_T32 + t] == (1 << 32) % m
            row = [int(sh[S_ROWS + i * NT + t]) for i in range(RKP)]
            assert row == (mk.C2[ch] if gB else mk.C[ch]) + [0, 0]
            if gB:
                assert sh[S_B + t] == mk.M2B[ch] and sh[S_C + t] == pow(model.M // m, -1, m)
                assert pb[P_A + t] == mk.c1[ch]
            else:
                a1 = mk.Minv2[ch] * mk.M2i_inv[ch] % m
                assert sh[S_B + t] == mk.Minv2[ch] and sh[S_C + t] == a1 and sh[S_D + t] == mk.D[ch]
                assert pb[P_A + t] == mk.NB2[ch] * mk.Minv2[ch] % m and pb[P_A2 + t] == mk.NB2[ch] * a1 % m
            assert pb[P_M3 + t] == pow(model.M, 3, mk.N) % m
        assert sh[S_M2RINV] == mk.M2rinv
        for i in range(RK):
            limbs = [int(v) for v in sh[S_MPOS + i * RKP:S_MPOS + (i + 1) * RKP]]
            assert sum(v << (28 * c) for c, v in enumerate(limbs)) == model.M // model.B[i]
        assert sum(int(v) << (28 * c) for c, v in enumerate(sh[S_MFULL:S_MFULL + RKP])) == model.M
        _check_schedule(pb, P - 1)


def _check_schedule(pb, e):
    """the window schedule spells e, with bench.sliding_window_ops' counts"""
    from bench import sliding_window_ops
    ns = int(pb[P_NS])
    sc = [int(v) for v in pb[P_SCHED:P_SCHED + ns]]
    assert 0 < ns <= P_SCHED_MAX and sc[0] < 16
    v, sq, mul = 2 * sc[0] + 1, 1, 15
    for w in sc[1:]:
        assert w >> 8 or w & 0xFF
        v <<= w >> 8
        sq += w >> 8
        if w & 0xFF:
            assert (w & 0xFF) <= 16 and (w >> 8) >= 1
            v += 2 * ((w & 0xFF) - 1) + 1
            mul += 1
    assert v == e
    assert (sq, mul) == sliding_window_ops(e)


class _Kernel:
    """k_dec_rns, thread for thread in numpy (uint64 lanes): the same blocks,
    the same channel arithmetic (red / red64 with 32-bit wraps)"""

    def __init__(self, sh, pb):
        t = np.arange(NT)
        self.m = sh[S_M:S_M + NT].astype(np.uint64)
        self.mu = sh[S_MU:S_MU + NT].astype(np.uint64)
        self.t32 = sh[S_T32:S_T32 + NT].astype(np.uint64)
        self.cb, self.cc, self.cd = (sh[o:o + NT].astype(np.uint64) for o in (S_B, S_C, S_D))
        self.ca, self.ca2, self.m3 = (pb[o:o + NT].astype(np.uint64) for o in (P_A, P_A2, P_M3))
        self.sched = [int(v) for v in pb[P_SCHED:P_SCHED + int(pb[P_NS])]]
        self.rows = sh[S_ROWS:S_ROWS + RKP * NT].reshape(RKP, NT).astype(np.uint64)  # [i][t]
        self.m2rinv = int(sh[S_M2RINV])
        self.gB = t < 128
        ch = np.where(self.gB, t, t - 128)
        self.isr = t == RLANE
        self.actB = self.gB & (ch < RK)
        self.actB2 = ~self.gB & (ch < RK)
        self.ch = ch
        self.sh = sh

    def red(self, x):
        x = x.astype(np.uint64)
        assert np.all(x < (1 << 59))
        q = (((x >> np.uint64(27)) & np.uint64(U32)) * self.mu) >> np.uint64(32)
        r = (x - q * self.m) & np.uint64(U32)
        for _ in range(3):
            r = np.minimum(r, (r - self.m) & np.uint64(U32))
        return r

    def red64(self, x):
        return self.red((x >> np.uint64(32)) * self.t32 + (x & np.uint64(U32)))

    def cmul(self, a, b):
        p = a * b
        return np.where(self.isr, p & np.uint64(U32), self.red(np.where(self.isr, 0, p)))

    def cadd(self, a, b):
        s = (a + b) & np.uint64(U32)
        return np.where(self.isr, s, np.minimum(s, (s - self.m) & np.uint64(U32)))

    def mul(self, x, y):
        tt = self.cmul(x, y)
        xi = np.zeros(RKP, np.uint64)
        xi[:RK] = self.cmul(tt, self.ca)[:RK]
        acc = (xi[:, None] * self.rows).sum(axis=0, dtype=np.uint64)  # every thread's sum (B' read)
        assert np.all(acc[self.actB2] < (1 << 63))
        qh = self.red64(acc)
        tm, ta = self.cmul(tt, self.cb), self.cmul(tt, self.cc)  # before the barrier
        res2 = self.cadd(tm, self.cmul(qh, self.ca))
        x2 = self.cadd(ta, self.cmul(qh, self.ca2))
        rr = ((int(tt[RLANE]) + (int(acc[RLANE]) & U32) * int(self.ca[RLANE])) * int(self.cb[RLANE])) & U32
        u = np.where(self.actB2, (x2 * self.cd) & np.uint64(U32), 0)
        part = int(u.sum()) & U32
        xi2 = np.zeros(RKP, np.uint64)
        xi2[:RK] = x2[128:128 + RK]
        accB = (xi2[:, None] * self.rows).sum(axis=0, dtype=np.uint64)
        beta = ((part - rr) * self.m2rinv) & U32
        assert beta < RK
        d = (self.red64(accB) - self.cmul(np.full(NT, beta, np.uint64), self.cb)) & np.uint64(U32)
        resB = np.minimum(d, (d + self.m) & np.uint64(U32))
        out = np.where(self.gB, resB, res2)
        out[RLANE] = rr
        return out

    def value(self, x, N):
        """the exit: sum xi_i M_i - alpha M, then mod N (as thread 0 does)"""
        sh = self.sh
        xi = np.zeros(RKP, np.uint64)
        xi[:RK] = self.cmul(x, self.cc)[:RK]
        alpha = int((((xi * self.rows[:, RLANE]).sum(dtype=np.uint64) & np.uint64(U32)) - x[RLANE]) * self.cb[RLANE]) & U32
        assert alpha < RK
        mpos = sh[S_MPOS:S_MPOS + RK * RKP].reshape(RK, RKP).astype(np.uint64)
        cols = [int((xi[:RK] * mpos[:, c]).sum(dtype=np.uint64)) - alpha * int(sh[S_MFULL + c]) for c in range(RKP)]
        X = sum(v << (28 * c) for c, v in enumerate(cols))
        assert 0 <= X < (RK + 1) * N
        return X % N


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json"])
def test_kernel_emulation_exponentiation(fx):
    k = load_fixture(fx)["key"]
    P = hx(k["p"])
    N = P * P
    sh, pb = _blocks(P)
    kern = _Kernel(sh, pb)
    rng = np.random.default_rng(3)
    c = int.from_bytes(rng.bytes(512), "little")
    m = kern.m.astype(object)

    def chans(v):  # every thread's residue (inactive threads: 0)
        out = np.zeros(NT, np.uint64)
        for t in range(NT):
            if t == RLANE:
                out[t] = v & U32
            elif m[t]:
                out[t] = v % int(m[t])
        return out
    one = np.ones(NT, np.uint64)
    x = kern.mul(chans(c), one)          # c M^-1
    x = kern.mul(x, kern.m3)            # c M
    # a short exponent by square-and-multiply, then P - 1 through the kernel's
    # window schedule and table of odd powers
    e = 1 << 9 | 37
    acc = x
    for b in bin(e)[3:]:
        acc = kern.mul(acc, acc)
        if b == "1":
            acc = kern.mul(acc, x)
    assert kern.value(kern.mul(acc, one), N) == pow(c, e, N)
    tab = [x]
    x2 = kern.mul(x, x)
    for _ in range(15):
        tab.append(kern.mul(tab[-1], x2))
    acc = tab[kern.sched[0]]
    for w in kern.sched[1:]:
        for _ in range(w >> 8):
            acc = kern.mul(acc, acc)
        if w & 0xFF:
            acc = kern.mul(acc, tab[(w & 0xFF) - 1])
    got = kern.value(kern.mul(acc, one), N)
    assert got == pow(c, P - 1, N) and got % P == 1
