"""CPU: the drop-in's host logic against the reference's golden vectors, with
the eight device entry points of xfl_amd.paillier.ops replaced by the oracle
(tests/oracle_ops.py). The same checks run on the real kernels in
tests/test_gpu_dropin.py; this copy exercises PaillierArray's flat buffers,
broadcasting, scalar encoding, alignment, sign branches, decode dtype paths
and the wire codec on any machine (2048-bit fixtures: pure-Python modexp)."""
import pytest

from tests import dropin_cases as C
from tests import oracle_ops

HOST_FIXTURES = ["paillier_2048_djn.json", "paillier_2048_nodjn.json"]


@pytest.fixture(autouse=True)
def _oracle_ops(monkeypatch):
    oracle_ops.install(monkeypatch)


@pytest.mark.parametrize("vectorized", [False, True])
@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_ops_bit_exact(fx, vectorized):
    C.ops_bit_exact(fx, vectorized)


def test_histogram_groupby_bit_exact():
    C.histogram_groupby(HOST_FIXTURES[0])


@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_decrypt_matches_reference(fx):
    C.decrypt_matches_reference(fx)


@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_wire_roundtrip_with_reference_pickles(fx):
    C.wire_roundtrip(fx)


@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_array_protocol(fx):
    C.array_protocol(fx)


@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_encrypt_decrypt_shapes(fx):
    C.encrypt_decrypt_shapes(fx)


def test_sharded_slices_cover_the_batch(monkeypatch):
    """ops.sharded: contiguous slices, one per shard device, small batches on
    the first device only, devices taken from $XHE_DEVICES / num_cores."""
    import threading

    from xfl_amd.paillier import ops
    from xfl_amd.paillier.context import PaillierContext

    class Ctx:
        def __init__(self):
            self.keys = []

        shard_devices = staticmethod(PaillierContext.shard_devices)

        def device_key(self, d):
            self.keys.append(d)
            return d

    monkeypatch.setattr(ops, "MIN_SHARD", 10)
    for spec, count, want_k in (("0,1,2,3", 1000, 4), ("0,1,2,3", 25, 2), ("5", 1000, 1), ("0,0,0", 31, 3),
                                ("0,1", 9, 1)):
        monkeypatch.setenv("XHE_DEVICES", spec)
        ctx = Ctx()
        seen = []
        lock = threading.Lock()

        def body(dk, lo, hi):
            with lock:
                seen.append((dk, lo, hi))
        ops.sharded(ctx, count, body)
        seen.sort(key=lambda t: t[1])
        assert len(seen) == want_k
        assert seen[0][1] == 0 and seen[-1][2] == count
        assert all(seen[i][2] == seen[i + 1][1] for i in range(len(seen) - 1))
        devs = [int(d) for d in spec.split(",")]
        assert [s[0] for s in seen] == devs[:want_k]
    monkeypatch.delenv("XHE_DEVICES")
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.setattr("xfl_amd._native.visible_devices", lambda: 8)
    # default: the process's own GPU only (no key/tables on the other GPUs)
    assert PaillierContext.shard_devices(-1) == [0]
    assert PaillierContext.shard_devices(3) == [0, 1, 2]
    assert PaillierContext.shard_devices(1) == [0]
    monkeypatch.setenv("LOCAL_RANK", "6")
    assert PaillierContext.shard_devices(-1) == [6]
    assert PaillierContext.shard_devices(3) == [6, 7, 0]
    monkeypatch.setenv("XHE_DEVICES", "all")
    assert PaillierContext.shard_devices(-1) == list(range(8))


def test_table_window_policy(monkeypatch):
    """The fixed-base window follows the key's encrypted volume (16 -> 20 ->
    22) as far as free HBM allows; pinned by set_device_window / $XHE_WIN_BITS;
    public and non-DJN keys carry no tables."""
    import xfl_amd._native as nat
    from tests.conftest import load_fixture
    built = []

    class FakeKey:
        def __init__(self, bits, n, p=None, q=None, h=None, device=0, win_bits=0):
            wb = win_bits if (p is not None and h) else 0
            self.win_bits = wb & 0xFF
            self.win_split = bool(wb & 0x100)
            built.append((device, self.win_bits))

    monkeypatch.setattr(nat, "DeviceKey", FakeKey)
    free = {"b": 200 << 30}
    monkeypatch.setattr(nat, "device_free_bytes", lambda d=0: free["b"])
    monkeypatch.delenv("XHE_WIN_BITS", raising=False)
    priv, pub = C.ctxs(load_fixture("paillier_2048_djn.json"))
    assert priv.device_key().win_bits == 16
    priv.note_encrypt_volume(7_000_000)
    assert priv.device_key().win_bits == 16 and len(built) == 1
    priv.note_encrypt_volume(2_000_000)
    assert priv.device_key().win_bits == 20
    priv.note_encrypt_volume(100_000_000)
    free["b"] = 90 << 30  # 2 x 50.4 GB + 32 GiB margin does not fit next to the win-20 tables' 27.9 GB
    assert priv.device_key().win_bits == 20
    free["b"] = 200 << 30
    assert priv.device_key().win_bits == 22
    assert [w for _, w in built] == [16, 20, 22]
    priv.set_device_window(18)
    assert priv.device_key().win_bits == 18
    monkeypatch.setenv("XHE_WIN_BITS", "12")
    priv.set_device_window(None)
    assert priv.device_key().win_bits == 12
    # split layouts: the masked window and the layout flag compare separately,
    # so a built split key is reused, not rebuilt on every call
    from xfl_amd._native import XHE_WIN_SPLIT
    n_before = len(built)
    priv.set_device_window("18s")
    k1 = priv.device_key()
    assert k1.win_bits == 18 and k1.win_split
    assert priv.device_key() is k1 and len(built) == n_before + 1
    priv.set_device_window(18 | XHE_WIN_SPLIT)
    assert priv.device_key().win_split and len(built) == n_before + 2
    monkeypatch.setenv("XHE_WIN_BITS", "14s")
    priv.set_device_window(None)
    assert priv.device_key().win_bits == 14 and priv.device_key().win_split
    assert pub.device_key().win_bits == 0
    nodjn, _ = C.ctxs(load_fixture("paillier_2048_nodjn.json"))
    assert nodjn.device_key().win_bits == 0


def test_window_layouts():
    """Split table layouts (include/xhe.h XHE_WIN_SPLIT): floor(rand_bits/w)
    windows, the first rand_bits mod w of them w+1 bits wide; the bench picks
    the uniform layout with the fewest table products that fits (split ones
    on request)."""
    import bench
    from xfl_amd._native import XHE_WIN_SPLIT as S
    from xfl_amd._native import parse_win, table_bytes, win_layout, win_spec
    assert win_layout(1024, 23) == (45, 0) and win_layout(1024, 23 | S) == (44, 12)
    assert win_layout(1024, 16 | S) == (64, 0)  # divides evenly: uniform
    for rb, wb in ((1024, 23 | S), (1536, 22), (2048, 21 | S), (1024, 7 | S)):
        nwin, nhi = win_layout(rb, wb)
        w = wb & 0xFF
        assert nhi * (w + 1) + (nwin - nhi) * w == rb or (nhi == 0 and nwin * w >= rb)
    assert table_bytes(2048, 23) == 2 * 45 * (1 << 23) * 256
    assert table_bytes(2048, 23 | S) == 2 * 56 * (1 << 23) * 256
    assert parse_win("23s") == 23 | S and parse_win("22") == 22 and win_spec(23 | S) == "23s"
    assert bench.pick_window(2048, 287 * 10**9) == 23
    assert bench.pick_window(2048, 287 * 10**9, split=True) == 23 | S
    assert bench.pick_window(2048, 230 * 10**9, split=True) == 23  # 240.5 GB + 16 GiB does not fit
    assert bench.pick_window(3072, 287 * 10**9, split=True) == 22
    assert bench.pick_window(4096, 287 * 10**9) == 21


@pytest.mark.parametrize("vectorized", [False, True])
@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_gap_alignment_negative_branch(fx, vectorized):
    C.gap_alignment(fx, vectorized)


def test_shifted_words_matches_python_ints():
    import numpy as np
    """the aligned mat-vec exponents k << shift built with numpy equal the
    Python-int construction (and kbits bounds every value)"""
    from xfl_amd._native import words_to_ints
    from xfl_amd.paillier.array import _shifted_words
    rng = np.random.default_rng(0)
    for t in range(200):
        n = int(rng.integers(1, 40))
        k = rng.integers(0, 2 ** 63, size=n, dtype=np.int64) >> rng.integers(0, 63, size=n)
        if t % 5 == 0:
            k[1:] = 0
        s = rng.integers(0, 200, size=n)
        w, kbits = _shifted_words(k, s)
        want = [int(a) << int(b) for a, b in zip(k, s)]
        assert words_to_ints(w) == want
        assert max(v.bit_length() for v in want) <= kbits



def test_encode_at_aligned_exponent_matches_encoder():
    """array._encode_at (the host half of ciphertext + scalar's aligned
    operand): each scalar's encoding at min(its own exponent, the
    ciphertext's) is the reference's encode_single at its own exponent times
    2^d mod n - the plaintext of (1 + n m)^(2^d), what _decrease_exponent_to
    makes of the encrypted scalar (paillier.py:79-86) - for floats of both
    signs, zero, float32, ints and gaps up to ~1,100 bits; None when a value
    would come near n."""
    import numpy as np
    from oracle import paillier_oracle as O
    from xfl_amd._native import words_to_ints
    from tests.conftest import load_fixture
    from xfl_amd.paillier.array import _encode_at
    g = load_fixture("paillier_2048_djn.json")
    priv, _ = C.ctxs(g)
    ok = O.derive_private(priv.p, priv.q, priv.h_pow_n)
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.standard_normal(20) * 10.0 ** rng.integers(-30, 12, 20), [0.0, -1.0, 2.0 ** 52]])
    cases = ((x, rng.integers(-1100, 10, x.size)), (x.astype(np.float32), np.full(x.size, -40)),
             (rng.integers(-10 ** 6, 10 ** 6, 9), rng.integers(-900, 5, 9)))
    for P, ec in cases:
        m, enew = _encode_at(priv, P, ec)
        for v, c, e, got in zip(P.tolist(), ec.tolist(), enew.tolist(), words_to_ints(m)):
            ep = 0 if isinstance(v, int) else O.cal_exponent_float(v, None)
            assert e == min(ep, c)
            assert got == (O.encode(ok, v, ep) << (ep - e)) % priv.n, (v, ep, e)
    assert _encode_at(priv, np.array([3.0]), np.array([-2100])) is None


@pytest.mark.parametrize("fx", HOST_FIXTURES)
def test_xgb_histogram_pandas_columns(fx):
    C.xgb_histogram_pandas(fx)
