"""Parity at the fixed-base windows production actually runs.

The headline (bench.py) builds 2048-bit tables at window 23 (2 x 96.6 GB, row
offsets far past 2^32 words); the drop-in rebuilds at 20 and 22
(PaillierContext.WIN_STEPS); 3072-bit keys run at 22 (225 GB) and 4096 at 21.
Each case runs in a fresh child process (so its 100-225 GB of tables are built
and released with nothing else on the device) and encrypts >= 20,000 elements
through the device-resident C ABI - at 2048 bits that is k_djn_pmd's one-lane
shape (batches > 16 k) - then compares EVERY ciphertext with the reference's
DJN-CRT encryption (paillier.py:189-209,283; utils.py:38-43) computed by the
GMP checker (oracle/gmp_baseline.c gmpb_encrypt_batch, pinned to the
reference's golden ciphertexts by tests/test_cpu_baseline.py) on the same a,
and decrypts them back. The exponents include the edge draws: a = 0, 1,
2^bits - 1, the top bit alone, a full digit in every window (incl. the last,
partial one) and bit pairs straddling every 32-bit word boundary.

The 2048-bit w23 case also runs the headline step itself (device encode of
float64 + ChaCha draw + encrypt of 1 M elements, bench.py's encrypt_shard),
checks 8,192 of its ciphertexts with GMP and all 1 M by decrypt round trip.
"""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import sys, os, random, time
sys.path.insert(0, {root!r})
import numpy as np
import torch
torch.cuda.init()
from tests.conftest import hx, load_fixture
from xfl_amd import _native as nat
from oracle import paillier_oracle as O
from oracle import bench_cpu

fx, win, count, headline = {fx!r}, {win}, {count}, {headline}
g = load_fixture(fx)
k = g["key"]
p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
n = p * q
bits = g["key_bits"]
t0 = time.time()
dk = nat.DeviceKey(bits, n, p, q, h, device=0, win_bits=win)
torch.cuda.synchronize()
print("key", bits, "win", win, "tables", nat.table_bytes(bits, win), "built_s", round(time.time() - t0, 2), flush=True)
L = nat.lib()
okey = O.derive_private(p, q, h)
RB = dk.rand_bits
nwin = nat.win_layout(RB, win)[0]

# edge exponents: 0, 1, all ones, top bit, a full digit per window, bit pairs
# across every 32-bit word boundary; then random draws below 2^RB
edge = [0, 1, (1 << RB) - 1, 1 << (RB - 1)]
edge += [(((1 << win) - 1) << (win * w)) & ((1 << RB) - 1) for w in range(nwin)]
edge += [3 << (32 * j - 1) for j in range(1, RB // 32)]
rng = random.Random(bits * 100 + win)
a = edge + [rng.randrange(1, 1 << RB) for _ in range(count - len(edge))]
ms = [0, n - 1, 1, n // 3] + [rng.randrange(n) for _ in range(count - 4)]
mw = nat.ints_to_words(ms, dk.nw)
aw = nat.ints_to_words(a, dk.rand_words)
stream = torch.cuda.current_stream().cuda_stream
md = torch.from_numpy(mw.view(np.int32)).cuda()
ad = torch.from_numpy(aw.view(np.int32)).cuda()
ct = torch.empty((count, dk.n2w), dtype=torch.int32, device="cuda")
nat.check(L.xhe_encrypt(dk.handle, md.data_ptr(), ad.data_ptr(), count, ct.data_ptr(), stream), "encrypt")
got = ct.cpu().numpy().view(np.uint32)
want = bench_cpu.gmp_encrypt_batch(okey, mw, aw, threads=16)
bad = np.nonzero(np.any(got != want, axis=1))[0]
assert bad.size == 0, f"{{bad.size}} of {{count}} ciphertexts differ, first {{bad[:8].tolist()}}"
m2 = torch.empty_like(md)
nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), count, m2.data_ptr(), stream), "decrypt")
assert torch.equal(m2, md), "decrypt round trip differs"
print("ok words", count, "vs gmp", flush=True)

if headline:
    N = 1 << 20 if headline > 1 else 1_000_000
    x = torch.from_numpy(np.random.default_rng(5).standard_normal(N)).cuda()
    m = torch.empty((N, dk.nw), dtype=torch.int32, device="cuda")
    ex = torch.empty(N, dtype=torch.int32, device="cuda")
    st = torch.empty(N, dtype=torch.int32, device="cuda")
    rnd = torch.empty((N, dk.rand_words), dtype=torch.int32, device="cuda")
    ct = torch.empty((N, dk.n2w), dtype=torch.int32, device="cuda")
    nat.check(L.xhe_encode_f64(dk.handle, x.data_ptr(), N, 7, 0, 0, m.data_ptr(), ex.data_ptr(), st.data_ptr(),
                               stream), "encode")
    nat.check(L.xhe_rand(dk.handle, os.urandom(32), 7, N, rnd.data_ptr(), None, stream), "rand")
    nat.check(L.xhe_encrypt(dk.handle, m.data_ptr(), rnd.data_ptr(), N, ct.data_ptr(), stream), "encrypt")
    m2 = torch.empty_like(m)
    nat.check(L.xhe_decrypt(dk.handle, ct.data_ptr(), N, m2.data_ptr(), stream), "decrypt")
    assert torch.equal(m, m2), "headline round trip differs"
    sel = np.unique(np.concatenate([np.arange(4096), np.random.default_rng(6).integers(0, N, 4092), [N - 4, N - 3, N - 2, N - 1]]))
    xs = x.cpu().numpy()
    # the device encoder against the oracle's encode (encoder.py:29-54) on the sample
    mh = m.cpu().numpy().view(np.uint32)[sel]
    enc = [O.encode_element(okey, float(xs[i]), 7)[0] for i in sel]
    assert nat.words_to_ints(mh) == enc, "device encode differs"
    want = bench_cpu.gmp_encrypt_batch(okey, mh, rnd.cpu().numpy().view(np.uint32)[sel], threads=16)
    got = ct.cpu().numpy().view(np.uint32)[sel]
    assert np.array_equal(got, want), "headline ciphertexts differ from GMP"
    print("ok headline", N, "sample", sel.size, flush=True)
del dk
print("done", flush=True)
"""


def _run(fx, win, count=20000, headline=0, timeout=600):
    r = subprocess.run([sys.executable, "-u", "-c", _CHILD.format(root=ROOT, fx=fx, win=win, count=count,
                                                                  headline=headline)],
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0 and "done" in r.stdout, r.stdout[-3000:] + r.stderr[-4000:]
    return r.stdout


def test_2048_w23_headline_window():
    """The bench's window: 193 GB of tables, the headline step at 1 M elements."""
    out = _run("paillier_2048_djn.json", 23, headline=1)
    assert "ok headline" in out


@pytest.mark.parametrize("win", [20, 22])
def test_2048_dropin_rebuild_windows(win):
    """The drop-in's rebuild steps (context.py WIN_STEPS: 20 after 8 M elements, 22 after 64 M)."""
    _run("paillier_2048_djn.json", win)


def test_3072_w22():
    """Config 4's window (bench.pick_window at 3072 bits: 2 x 112.7 GB)."""
    _run("paillier_3072_djn.json", 22)


def test_4096_w21():
    _run("paillier_4096_djn.json", 21, count=20000)


def test_dropin_set_device_window_roundtrip():
    """The drop-in at a pinned wide window (set_device_window, the API the
    window policy uses): Paillier.encrypt -> decrypt of 50 k float64 is exact to
    the encoding precision, and the context's key really runs at that window."""
    import numpy as np

    from xfl_amd.paillier import Paillier, PaillierContext
    from tests.conftest import hx, load_fixture
    k = load_fixture("paillier_2048_djn.json")["key"]
    ctx = PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=hx(k["h_pow_n"]))
    ctx.set_device_window(20)
    x = np.random.default_rng(3).standard_normal(50_000)
    enc = Paillier.encrypt(ctx, x, precision=7)
    back = Paillier.decrypt(ctx, enc)
    assert max(d.win_bits for d in ctx._dev.values()) == 20
    # precision 7 encodes at 2^-24 (error <= 2^-25), then the float32 result
    assert np.allclose(back, x, rtol=1e-6, atol=1e-7)
    del enc
    ctx._dev = {}
