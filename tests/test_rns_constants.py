"""CPU: the small-batch decrypt's RNS constants (xhe_rns_constants, the blocks
k_dec_rns reads; rns_dev.hpp) against tools/rns_model.py, and the kernel's
per-channel algorithm - every channel's Barrett and Shoup arithmetic, the two
base extensions per product summed in two halves, the DPP partial sums, the
exit's columns and the reduction mod P^2 - emulated in numpy on those blocks,
through a whole c^(P-1) mod P^2 on the kernel's window schedule against
Python's pow. The model itself is checked against Python integers (bounds,
exactness) by its own asserts."""
import ctypes
import os
import sys

import numpy as np
import pytest

from tests.conftest import hx, load_fixture

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# rns_dev.hpp's layout
RK, RKP, RT, HT, NSLOT, RCH = 74, 76, 80, 40, 160, 74
RSLOT = 80 + RCH  # the r channel's slot
S_M, S_MU, S_T32, S_B, S_BS, S_C, S_CS, S_D = 0, 160, 320, 480, 640, 800, 960, 1120
S_ROWS = 1280
S_MPOS = S_ROWS + RT * NSLOT
S_MFULL = S_MPOS + RK * RKP
S_M2RINV = S_MFULL + RKP
S_WORDS = S_M2RINV + 4
P_A, P_AS, P_A2, P_A2S, P_M3, P_NS, P_SCHED, P_SCHED_MAX = 0, 160, 320, 480, 640, 800, 804, 1280
P_WORDS = P_SCHED + P_SCHED_MAX + 4
U32 = (1 << 32) - 1


def _blocks(P):
    from xfl_amd import _native as nat
    L = nat.lib()
    pw = nat.ints_to_words([P], (P.bit_length() + 31) // 32)[0]
    sh = np.zeros(S_WORDS, np.uint32)
    pb = np.zeros(P_WORDS, np.uint32)
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    nat.check(L.xhe_rns_constants(vp(pw), pw.shape[0], vp(sh), vp(pb)), "rns constants")
    return sh, pb


@pytest.fixture(scope="module")
def model():
    import rns_model
    return rns_model


def test_header_sizes():
    hdr = open(os.path.join(ROOT, "include", "xhe.h")).read()
    assert f"#define XHE_RNS_SHARED_WORDS {S_WORDS}" in hdr and f"#define XHE_RNS_PRIME_WORDS {P_WORDS}" in hdr


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_2048_nodjn.json"])
def test_constants_match_model(model, fx):
    k = load_fixture(fx)["key"]
    shoup = lambda w, m: (w << 32) // m  # noqa: E731
    for P in (hx(k["p"]), hx(k["q"])):
        sh, pb = _blocks(P)
        mk = model.Key(P)
        for slot in range(NSLOT):
            gB, ch = slot < 80, slot % 80
            row = [int(sh[S_ROWS + i * NSLOT + slot]) for i in range(RT)]
            if slot == RSLOT:
                assert sh[S_M + slot] == 0 and row == mk.E + [0] * (RT - RK)
                assert sh[S_B + slot] == mk.Mrinv and pb[P_A + slot] == mk.Nr
                assert pb[P_M3 + slot] == pow(model.M, 3, mk.N) % 2 ** 32
                continue
            if ch >= RK:
                assert sh[S_M + slot] == 0 and not any(row)
                continue
            m = model.B[ch] if gB else model.B2[ch]
            assert sh[S_M + slot] == m and sh[S_MU + slot] == (1 << 59) // m and sh[S_T32 + slot] == (1 << 32) % m
            assert row == (mk.C2[ch] if gB else mk.C[ch]) + [0] * (RT - RK)
            if gB:
                assert sh[S_B + slot] == mk.M2B[ch] and sh[S_C + slot] == pow(model.M // m, -1, m)
                assert pb[P_A + slot] == mk.c1[ch]
            else:
                a1 = mk.Minv2[ch] * mk.M2i_inv[ch] % m
                assert sh[S_B + slot] == mk.Minv2[ch] and sh[S_C + slot] == a1 and sh[S_D + slot] == mk.D[ch]
                assert pb[P_A + slot] == mk.NB2[ch] * mk.Minv2[ch] % m and pb[P_A2 + slot] == mk.NB2[ch] * a1 % m
                assert pb[P_A2S + slot] == shoup(int(pb[P_A2 + slot]), m)
            assert sh[S_BS + slot] == shoup(int(sh[S_B + slot]), m)
            assert sh[S_CS + slot] == shoup(int(sh[S_C + slot]), m)
            assert pb[P_AS + slot] == shoup(int(pb[P_A + slot]), m)
            assert pb[P_M3 + slot] == pow(model.M, 3, mk.N) % m
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
    """k_dec_rns, channel slot for channel slot in numpy (uint64 lanes): the
    same blocks, the same channel arithmetic (red / red64 / Shoup with 32-bit
    wraps), each extension summed as the kernel's two 40-term halves"""

    def __init__(self, sh, pb):
        g = lambda o: sh[o:o + NSLOT].astype(np.uint64)  # noqa: E731
        self.m, self.mu, self.t32 = g(S_M), g(S_MU), g(S_T32)
        self.cb, self.cbs, self.cc, self.ccs, self.cd = g(S_B), g(S_BS), g(S_C), g(S_CS), g(S_D)
        p = lambda o: pb[o:o + NSLOT].astype(np.uint64)  # noqa: E731
        self.ca, self.cas, self.ca2, self.ca2s, self.m3 = p(P_A), p(P_AS), p(P_A2), p(P_A2S), p(P_M3)
        self.sched = [int(v) for v in pb[P_SCHED:P_SCHED + int(pb[P_NS])]]
        self.rows = sh[S_ROWS:S_ROWS + RT * NSLOT].reshape(RT, NSLOT).astype(np.uint64)  # [i][slot]
        self.m2rinv = int(sh[S_M2RINV])
        slot = np.arange(NSLOT)
        self.gB = slot < 80
        self.isr = slot == RSLOT
        self.actB = self.gB & (slot < RK)
        self.actB2 = (slot >= 80) & (slot - 80 < RK)
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

    def shoup(self, a, w, ws):
        q = (a * ws) >> np.uint64(32)
        r = (a * w - q * self.m) & np.uint64(U32)
        return np.minimum(r, (r - self.m) & np.uint64(U32))

    def cmul(self, a, b):
        p = a * b
        return np.where(self.isr, p & np.uint64(U32), self.red(np.where(self.isr, 0, p)))

    def cadd(self, a, b):
        s = (a + b) & np.uint64(U32)
        return np.where(self.isr, s, np.minimum(s, (s - self.m) & np.uint64(U32)))

    def ext(self, v):
        """every slot's sum over the 80 terms, as the two halves and their total"""
        lo = (v[:HT, None] * self.rows[:HT]).sum(axis=0, dtype=np.uint64)
        hi = (v[HT:, None] * self.rows[HT:]).sum(axis=0, dtype=np.uint64)
        return lo, hi, lo + hi

    def mul(self, x, y):
        tt = self.cmul(x, y)
        xi = np.zeros(RT, np.uint64)
        xi[:RK] = self.shoup(tt, self.ca, self.cas)[:RK]
        lo, hi, acc = self.ext(xi)
        for a in (lo, hi, acc):  # the halves and their sum below 2^63 (no wrap)
            assert np.all(a[self.actB2] < (1 << 63))
        qh = self.red64(acc)
        tm, ta = self.shoup(tt, self.cb, self.cbs), self.shoup(tt, self.cc, self.ccs)  # before the barrier
        res2 = self.cadd(tm, self.shoup(qh, self.ca, self.cas))
        x2 = self.cadd(ta, self.shoup(qh, self.ca2, self.ca2s))
        rr = ((int(tt[RSLOT]) + (int(acc[RSLOT]) & U32) * int(self.ca[RSLOT])) * int(self.cb[RSLOT])) & U32
        u = np.where(self.actB2, (x2 * self.cd) & np.uint64(U32), 0)
        part = int(u.sum()) & U32  # the three B' waves' DPP sums
        xi2 = np.zeros(RT, np.uint64)
        xi2[:RK] = x2[80:80 + RK]
        lo, hi, accB = self.ext(xi2)
        for a in (lo, hi, accB):
            assert np.all(a[self.actB] < (1 << 63))
        beta = ((part - rr) * self.m2rinv) & U32
        assert beta < RK
        d = (self.red64(accB) - self.shoup(np.full(NSLOT, beta, np.uint64), self.cb, self.cbs)) & np.uint64(U32)
        resB = np.minimum(d, (d + self.m) & np.uint64(U32))
        out = np.where(self.gB, resB, res2)
        out[RSLOT] = rr
        return out

    def value(self, x, N):
        """the exit: sum xi_i M_i - alpha M, then mod N (as thread 0 does)"""
        sh = self.sh
        xi = np.zeros(RT, np.uint64)
        xi[:RK] = self.cmul(x, self.cc)[:RK]
        sx = int(self.ext(xi)[2][RSLOT]) & U32
        alpha = ((sx - int(x[RSLOT])) * int(self.cb[RSLOT])) & U32
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

    def chans(v):  # every slot's residue (inactive slots: 0)
        out = np.zeros(NSLOT, np.uint64)
        for s in range(NSLOT):
            if s == RSLOT:
                out[s] = v & U32
            elif m[s]:
                out[s] = v % int(m[s])
        return out
    one = np.ones(NSLOT, np.uint64)
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
