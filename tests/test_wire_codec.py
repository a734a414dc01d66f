"""CPU: the native wire codec (xhe_wire_encode / xhe_wire_decode, host code in
libxhe) against Python's pickle in both directions, the reference's own wire
bytes (gmpy2 mpz values, tests/golden ops.wire_a4) and malformed input;
Paillier.serialize / ciphertext_from round trips through it."""
import pickle
import random

import numpy as np
import pytest

from tests.conftest import FIXTURES, hx, load_fixture


def _vals(n, seed=0, bits=4095):
    rng = random.Random(seed)
    raws = [rng.getrandbits(bits) for _ in range(n)] + [0, 1, 127, 128, 255, 256, 2 ** 31, 2 ** 32 - 1, 2 ** bits + 5]
    exps = [rng.choice([-24, 0, -60, 7, -(2 ** 31), 2 ** 31 - 1]) for _ in raws]
    return raws, exps


def test_native_bytes_load_with_python_pickle():
    from xfl_amd.compat import loads
    from xfl_amd.paillier import wire
    raws, exps = _vals(50)
    n = len(raws)
    b = wire.encode(raws, exps, (n,), 129)
    obj = loads(b)
    assert isinstance(obj, np.ndarray) and obj.dtype == object and obj.shape == (n,)
    assert [o.value for o in obj] == raws and [o.exp for o in obj] == exps
    b2 = wire.encode(raws[:54], exps[:54], (6, 9), 129)
    assert loads(b2).shape == (6, 9)
    assert loads(wire.encode([], [], (0,), 129)).shape == (0,)


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_python_pickles_decode_natively(protocol):
    from xfl_amd.paillier import wire
    from xfl_amd.paillier.paillier import RawCiphertext
    raws, exps = _vals(1200, seed=protocol)  # > 1000: several APPENDS batches
    arr = np.empty(len(raws), dtype=object)
    for i, (r, e) in enumerate(zip(raws, exps)):
        arr[i] = RawCiphertext(r, e)
    from xfl_amd.compat import _register_alias
    _register_alias()
    b = pickle.dumps(arr.reshape(3, -1) if len(raws) % 3 == 0 else arr, protocol=protocol)
    got_r, got_e, shape = wire.decode(b, 129)
    assert got_r == raws and list(got_e) == exps and int(np.prod(shape)) == len(raws)


def test_reference_wire_bytes_with_gmpy2_values():
    from xfl_amd.paillier import wire
    g = load_fixture(FIXTURES[0])
    raws, exps, shape = wire.decode(bytes.fromhex(g["ops"]["wire_a4"]), 128)
    assert raws == [hx(r) for r in g["ops"]["a"]["raw"][:4]]
    assert list(exps) == g["ops"]["a"]["exp"][:4] and shape == (4,)


def test_malformed_input_rejected():
    from xfl_amd.paillier import wire
    raws, exps = _vals(3)
    b = wire.encode(raws, exps, (len(raws),), 129)
    crafted = (b"K\x01a.",                                  # APPEND with no list under it (was a heap write)
               b"K\x01K\x02s.",                             # SETITEM with no dict
               b")K\x01K\x02s.",                            # SETITEM into a tuple
               b"\x8e" + b"\xff" * 7 + b"\x7f" + b"x",       # BINBYTES8 of length INT64_MAX (pos + k overflow)
               b"\x8d" + b"\xf0" + b"\xff" * 6 + b"\x7f" + b"x",
               b"K\x01r\xff\xff\xff\x03.")                  # memo index far beyond the input size
    for bad in (b[:-7], b"\x80\x04garbage", pickle.dumps([1, 2, 3]), pickle.dumps(np.arange(4))) + crafted:
        with pytest.raises(ValueError):
            wire.decode(bad, 129)
    with pytest.raises(ValueError):  # value wider than the word budget
        wire.decode(b, 4)


@pytest.mark.parametrize("compression", [False, True])
def test_paillier_serialize_roundtrip(compression):
    from xfl_amd.paillier import Paillier, PaillierCiphertext, PaillierContext
    k = load_fixture(FIXTURES[0])["key"]
    pub = PaillierContext().init(hx(k["p"]), hx(k["q"])).to_public()
    rng = random.Random(4)
    arr = np.array([PaillierCiphertext(pub, rng.randrange(pub.n_square), rng.choice([-24, 0]))
                    for _ in range(60)], dtype=object).reshape(5, 12)
    back = Paillier.ciphertext_from(pub, Paillier.serialize(arr, compression), compression)
    assert back.shape == (5, 12)
    assert [(c.raw_ciphertext, c.exponent) for c in back.reshape(-1)] == \
        [(c.raw_ciphertext, c.exponent) for c in arr.reshape(-1)]
    none_ctx = Paillier.ciphertext_from(None, Paillier.serialize(arr, compression), compression)
    assert none_ctx.reshape(-1)[7].raw_ciphertext == arr.reshape(-1)[7].raw_ciphertext
