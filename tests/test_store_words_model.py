"""Model of Mont::store_words (xfl_amd/csrc/bn_dev.hpp), the register-direct
packing of a residue's W-bit limbs (L per lane, TPI lanes) into 32-bit words:
every lane builds local words u[] from its own limbs and the next lane's first
two, then writes the words that start in its bits with one funnel shift by its
runtime bit offset. This checks the index arithmetic for every limb shape the
library instantiates against plain little-endian packing (the GPU tests check
the compiled kernels; a per-lane-branch form of this code was miscompiled at
3072 bits)."""
import random

import pytest

# (S, W, TPI, nwords) for every Mont shape whose store_packed runs (xhe.hip shapes)
SHAPES = [
    (152, 27, 4, 128), (160, 27, 16, 128), (76, 28, 4, 64),            # 2048: n^2, n^2 rows, p^2 words
    (228, 27, 4, 192), (240, 27, 16, 192), (112, 28, 4, 96), (60, 27, 4, 48),  # 3072
    (304, 27, 16, 256), (152, 27, 4, 128), (80, 27, 4, 64),            # 4096
    (640, 26, 16, 512), (304, 27, 16, 256),                            # 8192
    (37, 28, 1, 32), (74, 28, 1, 64),                                  # one-lane shapes
]


def store_words_model(limbs, S, W, TPI, nwords):
    L = S // TPI
    out = [None] * nwords
    LB = L * W
    NWM = (LB + 31) // 32 + 1
    for g in range(TPI):
        b = limbs[g * L:(g + 1) * L]
        n0 = limbs[(g + 1) * L] if g < TPI - 1 else 0
        n1 = limbs[(g + 1) * L + 1] if g < TPI - 1 and L > 1 else 0

        def limb(x):
            return b[x] if x < L else n0 if x == L else n1 if x == L + 1 else 0

        u = []
        for i in range(NWM + 1):
            bit = 32 * i
            jl, sh = divmod(bit, W)
            v = limb(jl) | (limb(jl + 1) << W) | (limb(jl + 2) << (2 * W))
            u.append((v >> sh) & 0xFFFFFFFF)
        b0 = g * LB
        ks = (b0 + 31) >> 5
        off = (ks << 5) - b0
        assert 0 <= off < 32
        ke = (b0 + LB + 31) >> 5
        kend = min(ke, nwords)
        for i in range(NWM):
            w = (((u[i + 1] << 32) | u[i]) >> off) & 0xFFFFFFFF
            if ks + i < kend:
                assert out[ks + i] is None, "word written twice"
                out[ks + i] = w
    return out


@pytest.mark.parametrize("S,W,TPI,nwords", SHAPES)
def test_store_words_model(S, W, TPI, nwords):
    rng = random.Random(S * 131 + W * 7 + TPI)
    assert S * W >= 32 * nwords
    for trial in range(20):
        bits = 32 * nwords if trial % 2 == 0 else 32 * nwords - rng.randrange(1, 64)
        x = rng.getrandbits(bits) if trial else (1 << (32 * nwords)) - 1
        limbs = [(x >> (W * j)) & ((1 << W) - 1) for j in range(S)]
        words = store_words_model(limbs, S, W, TPI, nwords)
        assert None not in words, "word never written"
        assert words == [(x >> (32 * k)) & 0xFFFFFFFF for k in range(nwords)]
