"""CPU: which GPU the drop-in's host paths use and when a batch stays in HBM
(host logic only; the device key and library are stand-ins)."""
from tests import dropin_cases as C


def test_host_path_keys_on_own_gpu(monkeypatch):
    """With $LOCAL_RANK set (one rank per GPU), the default device key, the
    host-array segmented product and the host mat-vec use that rank's GPU:
    ctx._dev only ever gets a key for it (GPU 0 in every rank)."""
    import numpy as np

    import xfl_amd._native as nat
    from tests.conftest import load_fixture
    from xfl_amd.paillier import ops

    class FakeKey:
        def __init__(self, bits, n, p=None, q=None, h=None, device=0, win_bits=0):
            self.win_bits, self.win_split, self.handle = win_bits & 0xFF, False, device

    calls = []

    class FakeLib:
        def xhe_segprod_host(self, handle, *a):
            calls.append(("segprod", handle))
            return 0

        def xhe_multiexp_host(self, handle, *a):
            calls.append(("multiexp", handle))
            return 0

    monkeypatch.setattr(nat, "DeviceKey", FakeKey)
    monkeypatch.setattr(nat, "device_free_bytes", lambda d=0: 200 << 30)
    monkeypatch.setattr(nat, "visible_devices", lambda: 4)
    monkeypatch.setattr(nat, "lib", lambda: FakeLib())
    monkeypatch.setenv("LOCAL_RANK", "6")
    monkeypatch.delenv("XHE_DEVICES", raising=False)
    monkeypatch.delenv("XHE_WIN_BITS", raising=False)
    priv, _ = C.ctxs(load_fixture("paillier_2048_djn.json"))
    priv.device_key()
    n2w = 128
    ops.segprod_words(priv, np.ones((3, n2w), np.uint32), np.zeros(3, np.int32), np.array([0, 3], np.int64))
    ops.multiexp_words(priv, np.ones((2, n2w), np.uint32), np.zeros((1, 2), np.int32), np.ones((1, 2, 1), np.uint32), 1)
    assert set(priv._dev) == {2}
    assert calls == [("segprod", 2), ("multiexp", 2)]


def test_resident_batches_capped_by_hbm_budget(monkeypatch):
    """Paillier.encrypt keeps a batch in HBM only while it fits the resident
    budget; a larger batch goes to the host-buffer path."""
    from tests.conftest import load_fixture
    from xfl_amd.paillier import resident

    monkeypatch.setattr(resident, "available", lambda: True)
    monkeypatch.delenv("XHE_RESIDENT", raising=False)
    monkeypatch.delenv("XHE_DEVICES", raising=False)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    priv, _ = C.ctxs(load_fixture("paillier_2048_djn.json"))
    per = 4 * 128 + 16
    monkeypatch.setenv("XHE_RESIDENT_MAX_BYTES", str(1000 * per))
    assert resident.device_for(priv, -1, 1000, per) == 0
    assert resident.device_for(priv, -1, 1001, per) is None
    assert resident.device_for(priv, -1) == 0  # existing arrays: no count, no cap
    monkeypatch.setenv("XHE_RESIDENT", "0")
    assert resident.device_for(priv, -1, 1, per) is None


def test_small_resident_batches_skip_the_hbm_query(monkeypatch):
    """Batches below RESIDENT_QUERY_MIN take the resident path without
    querying torch's allocator (a per-call cost on the latency-bound LR
    shapes); larger ones still check the budget."""
    from tests.conftest import load_fixture
    from xfl_amd import _native
    from xfl_amd.paillier import resident

    monkeypatch.setattr(resident, "available", lambda: True)
    for v in ("XHE_RESIDENT", "XHE_DEVICES", "LOCAL_RANK", "XHE_RESIDENT_MAX_BYTES"):
        monkeypatch.delenv(v, raising=False)
    priv, _ = C.ctxs(load_fixture("paillier_2048_djn.json"))
    queried = []
    monkeypatch.setattr(_native, "device_free_bytes", lambda dev: queried.append(dev) or 0)
    per = 4 * 128 + 16
    assert resident.device_for(priv, -1, 64, per) == 0
    assert queried == []
    big = resident.RESIDENT_QUERY_MIN // per + 1
    assert resident.device_for(priv, -1, big, per) is None  # 0 bytes free
    assert queried == [0]
