"""Debug: 8192-bit DJN private encryption, batch kernel vs the 16-lane one."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import hx, load_fixture
from xfl_amd import _native as nat

k = load_fixture("paillier_8192_djn.json")["key"]
p, q, h = hx(k["p"]), hx(k["q"]), hx(k["h_pow_n"])
dk = nat.DeviceKey(8192, p * q, p, q, h, device=0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
rng = np.random.default_rng(1)
m = rng.integers(0, 2**32, size=(N, dk.nw), dtype=np.uint64).astype(np.uint32)
m[:, dk.nw - 1] = 0
r = rng.integers(0, 2**32, size=(N, dk.rand_words), dtype=np.uint64).astype(np.uint32)
r[:, -1] &= 0x7FFFFFFF
ct = dk.encrypt_words(m, r)
back = dk.decrypt_words(ct)
bad = np.nonzero(np.any(back != m, axis=1))[0]
print("N", N, "bad", len(bad), bad[:5], bad[-5:] if len(bad) else "")
zero_ct = np.nonzero(np.all(ct == 0, axis=1))[0]
print("all-zero ct rows", len(zero_ct), zero_ct[:5])
if len(bad):
    i = bad[0]
    print("first bad back words", back[i][:4], "want", m[i][:4])
