"""Host-buffer entry points (include/xhe.h *_host) run element-chunked through
the pinned pipeline (xhe.hip host_pipeline: 64 k - 256 k-element chunks,
per-slot streams, serialised kernels). Each is checked bit-exactly
against the same operation on device-resident buffers, at batch sizes that
cross several chunk boundaries and leave a ragged last chunk - the chunking
must be invisible (paillier.py:79-123, 156-187, 273-287, 341-398 semantics
are the device kernels', already pinned by test_gpu_parity)."""
import ctypes

import numpy as np
import pytest

from tests.conftest import FIXTURES, hx, load_fixture
from tests.test_gpu_parity import _dkey

pytestmark = pytest.mark.gpu


def vp(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


@pytest.fixture(scope="module")
def env():
    import torch

    from xfl_amd import _native as nat
    g = load_fixture(FIXTURES[0])
    dk = _dkey(g)
    dk.n_int = hx(g["key"]["n"])
    return nat, nat.lib(), dk, torch


def _cipher(env, n, seed, mwords=None):
    """n ciphertexts (device-encrypted random m < 2^(32 mwords)) as host words"""
    nat, L, dk, torch = env
    rng = np.random.default_rng(seed)
    m = rng.integers(0, 1 << 32, (n, dk.nw), dtype=np.uint64).astype(np.uint32)
    m[:, (mwords or dk.nw - 1):] = 0  # m < n
    md = torch.from_numpy(m.view(np.int32)).cuda()
    r = torch.empty((n, dk.rand_words), dtype=torch.int32, device="cuda")
    c = torch.empty((n, dk.n2w), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    nat.check(L.xhe_rand(dk.handle, bytes(range(32)), seed, n, r.data_ptr(), None, s))
    nat.check(L.xhe_encrypt(dk.handle, md.data_ptr(), r.data_ptr(), n, c.data_ptr(), s))
    torch.cuda.synchronize()
    return m, r.cpu().numpy().view(np.uint32), c.cpu().numpy().view(np.uint32)


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def test_encrypt_words_and_raw_host(env):
    nat, L, dk, torch = env
    n = 300_001  # 128 k chunks (encrypt_host) and 256 k chunks (words_host), ragged ends
    m, r, c = _cipher(env, n, 11)
    out = np.empty((n, dk.n2w), np.uint32)
    nat.check(L.xhe_encrypt_host(dk.handle, vp(m), vp(r), n, vp(out)), "encrypt_host")
    assert np.array_equal(out, c)
    # device draws at global positions: the words-host call equals rand + encrypt of the whole batch
    nat.check(L.xhe_encrypt_words_host(dk.handle, vp(m), n, 1, bytes(range(32)), 11, vp(out)), "words_host")
    assert np.array_equal(out, c)


def test_mulmod_host_chunked(env):
    nat, L, dk, torch = env
    n = 140_003
    _, _, a = _cipher(env, n, 21)
    _, _, b = _cipher(env, n, 22)
    rng = np.random.default_rng(5)
    ea = rng.integers(-30, -27, n).astype(np.int32)
    eb = rng.integers(-30, -27, n).astype(np.int32)
    dmax = int(np.max(np.abs(ea.astype(np.int64) - eb)))
    out = np.empty_like(a)
    eo = np.empty(n, np.int32)
    nat.check(L.xhe_mulmod_host(dk.handle, vp(a), vp(ea), vp(b), vp(eb), n, dmax, vp(out), vp(eo)), "add")
    da, db, dea, deb = _dev(torch, a), _dev(torch, b), _dev(torch, ea), _dev(torch, eb)
    do = torch.empty_like(da)
    deo = torch.empty_like(dea)
    s = torch.cuda.current_stream().cuda_stream
    nat.check(L.xhe_mulmod(dk.handle, da.data_ptr(), dea.data_ptr(), db.data_ptr(), deb.data_ptr(), n, dmax,
                           do.data_ptr(), deo.data_ptr(), s))
    torch.cuda.synchronize()
    assert np.array_equal(out, do.cpu().numpy().view(np.uint32))
    assert np.array_equal(eo, deo.cpu().numpy()) and np.array_equal(eo, np.minimum(ea, eb))
    # optional exponent arguments absent: plain products
    nat.check(L.xhe_mulmod_host(dk.handle, vp(a), None, vp(b), None, n, 0, vp(out), None), "add plain")
    nat.check(L.xhe_mulmod(dk.handle, da.data_ptr(), None, db.data_ptr(), None, n, 0, do.data_ptr(), None, s))
    torch.cuda.synchronize()
    assert np.array_equal(out, do.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("invert", [0, 1])
def test_powmod_host_chunked(env, invert):
    nat, L, dk, torch = env
    n = 70_001
    _, _, c = _cipher(env, n, 31 + invert)
    k = np.random.default_rng(7).integers(0, 1 << 32, (n, 2), dtype=np.uint64).astype(np.uint32)
    k[:, 1] &= (1 << 21) - 1
    out = np.empty_like(c)
    nat.check(L.xhe_powmod_host(dk.handle, vp(c), vp(k), 2, 53, n, invert, vp(out)), "powmod_host")
    dc, dkk = _dev(torch, c), _dev(torch, k)
    base = dc
    s = torch.cuda.current_stream().cuda_stream
    if invert:
        base = torch.empty_like(dc)
        nat.check(L.xhe_invert(dk.handle, dc.data_ptr(), n, base.data_ptr(), s))
    do = torch.empty_like(dc)
    nat.check(L.xhe_powmod(dk.handle, base.data_ptr(), dkk.data_ptr(), 2, 53, n, do.data_ptr(), s))
    torch.cuda.synchronize()
    assert np.array_equal(out, do.cpu().numpy().view(np.uint32))
    for i in (0, 65535, 65536, n - 1):  # spot check against Python's pow across the chunk boundary
        n2 = dk.n_int ** 2
        ci = nat.words_to_ints(c[i])
        if invert:
            ci = pow(ci, -1, n2)
        assert nat.words_to_ints(out[i]) == pow(ci, nat.words_to_ints(k[i]), n2)


def test_decrypt_host_chunked(env):
    nat, L, dk, torch = env
    n = 140_001
    m, _, c = _cipher(env, n, 41, mwords=2)  # 64-bit m: finite decodes at 2^-24
    got = np.empty((n, dk.nw), np.uint32)
    nat.check(L.xhe_decrypt_host(dk.handle, vp(c), n, vp(got)), "decrypt_host")
    assert np.array_equal(got, m)
    ex = np.full(n, -24, np.int32)
    f64, f32, st, mo = np.empty(n), np.empty(n, np.float32), np.empty(n, np.int32), np.empty((n, dk.nw), np.uint32)
    nat.check(L.xhe_decrypt_decode_host(dk.handle, vp(c), vp(ex), n, vp(f64), vp(f32), vp(st), vp(mo)), "dd")
    assert np.array_equal(mo, m)
    dm, de = _dev(torch, m), _dev(torch, ex)
    d64 = torch.empty(n, dtype=torch.float64, device="cuda")
    d32 = torch.empty(n, dtype=torch.float32, device="cuda")
    ds = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    nat.check(L.xhe_decode(dk.handle, dm.data_ptr(), de.data_ptr(), n, d64.data_ptr(), d32.data_ptr(),
                           ds.data_ptr(), s))
    torch.cuda.synchronize()
    assert np.array_equal(st, ds.cpu().numpy())
    ok = st == 0
    assert ok.all()
    assert np.array_equal(f64[ok].view(np.uint64), d64.cpu().numpy()[ok].view(np.uint64))
    assert np.array_equal(f32[ok].view(np.uint32), d32.cpu().numpy()[ok].view(np.uint32))
    # without the m output (internal scratch)
    f64b = np.empty(n)
    nat.check(L.xhe_decrypt_decode_host(dk.handle, vp(c), vp(ex), n, vp(f64b), vp(f32), vp(st), None), "dd2")
    assert np.array_equal(f64b[ok].view(np.uint64), f64[ok].view(np.uint64))


_FAIL_SCRIPT = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, {root!r})
import torch
torch.cuda.init()
from tests.conftest import FIXTURES, hx, load_fixture
from tests.test_gpu_parity import _dkey
from xfl_amd import _native as nat
L = nat.lib()
dk = _dkey(load_fixture(FIXTURES[0]))
vp = lambda a: ctypes.c_void_p(a.ctypes.data)
n = 5 * (1 << 17) + 17            # 6 chunks of xhe_encrypt_host (128 k), staged through the pinned ring
rng = np.random.default_rng(3)
m = rng.integers(0, 1 << 32, (n, dk.nw), dtype=np.uint64).astype(np.uint32)
m[:, dk.nw - 1:] = 0
r = rng.integers(0, 1 << 32, (n, dk.rand_words), dtype=np.uint64).astype(np.uint32)
r[:, 0] |= 1
out = np.zeros((n, dk.n2w), np.uint32)
rc = L.xhe_encrypt_host(dk.handle, vp(m), vp(r), n, vp(out))
assert rc == nat.XHE_EINVAL and b"injected" in L.xhe_last_error(), (rc, L.xhe_last_error())
# the ring is free again and holds no stale copies: a full call in the same
# process equals the device-resident result
out2 = np.zeros((n, dk.n2w), np.uint32)
nat.check(L.xhe_encrypt_host(dk.handle, vp(m), vp(r), n, vp(out2)), "encrypt_host")
md, rd = torch.from_numpy(m.view(np.int32)).cuda(), torch.from_numpy(r.view(np.int32)).cuda()
c = torch.empty((n, dk.n2w), dtype=torch.int32, device="cuda")
nat.check(L.xhe_encrypt(dk.handle, md.data_ptr(), rd.data_ptr(), n, c.data_ptr(), torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
assert np.array_equal(out2, c.cpu().numpy().view(np.uint32))
print("ok")
"""


def test_failing_chunk_leaves_pipeline_usable():
    """A run() that fails in the middle of a multi-chunk call (the
    $XHE_TEST_FAIL_CHUNK hook, chunk 3 of 6) returns its error after the slot
    streams have drained (the pinned ring is released last); the next call in
    the same process is bit-exact."""
    import os
    import subprocess
    import sys

    from tests.conftest import ROOT
    env_ = dict(os.environ, XHE_TEST_HOOKS="1", XHE_TEST_FAIL_CHUNK="3")
    r = subprocess.run([sys.executable, "-c", _FAIL_SCRIPT.format(root=ROOT)], env=env_, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
