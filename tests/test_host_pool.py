"""The host result-buffer cache behind nat.empty (xfl_amd/_native.py): large
ciphertext arrays returned by the drop-in (Paillier.encrypt and the batched
operators, paillier.py:289-339) are recycled only once no array refers to
them any more. CPU only."""
import gc

import numpy as np

from xfl_amd import _native as nat

SHAPE = (70_000, 128)  # 35.8 MB of uint32: above the 32 MiB pooling threshold


def test_small_buffers_are_plain_numpy():
    a = nat.empty((10, 128), np.uint32)
    assert a.base is None and a.shape == (10, 128)


def test_buffer_recycled_only_after_every_view_is_gone():
    gc.collect()
    a = nat.empty(SHAPE, np.uint32)
    assert a.flags.c_contiguous and a.flags.writeable and a.dtype == np.uint32
    a[:] = 5
    addr = a.ctypes.data
    view = a[100:200]          # a slice keeps the allocation alive
    before = nat._pool_bytes
    del a
    gc.collect()
    assert nat._pool_bytes == before and int(view[0, 0]) == 5
    b = nat.empty(SHAPE, np.uint32)  # must not reuse the block the view still uses
    assert b.ctypes.data != addr
    del view
    gc.collect()
    assert nat._pool_bytes == before + 70_000 * 128 * 4
    c = nat.empty(SHAPE, np.uint32)  # now it comes back from the cache
    assert c.ctypes.data == addr and nat._pool_bytes == before
    del b, c
    gc.collect()


def test_pool_is_bounded(monkeypatch):
    gc.collect()
    monkeypatch.setattr(nat, "POOL_PER_SIZE", 2)
    arrs = [nat.empty(SHAPE, np.uint32) for _ in range(4)]
    start = nat._pool_bytes
    del arrs
    gc.collect()
    kept = len(nat._pool_free.get(70_000 * 128 * 4, []))
    assert kept <= 2 and nat._pool_bytes - start <= 2 * 70_000 * 128 * 4


def test_pickle_and_copy_of_pooled_arrays():
    import pickle
    a = nat.empty(SHAPE, np.uint32)
    a[:] = np.arange(SHAPE[1], dtype=np.uint32)
    b = pickle.loads(pickle.dumps(a[:3]))
    assert np.array_equal(b, a[:3])
    c = a.copy()
    del a
    gc.collect()
    assert int(c[2, 7]) == 7
