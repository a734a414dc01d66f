"""Pin the CPU oracle (oracle/paillier_oracle.py) to the reference's own outputs.

The fixtures were produced by XFL's Paillier code (tests/golden/gen_golden.py);
an oracle that disagrees with any of them is not trusted as a checker.
"""
import math

import numpy as np
import pytest

from oracle import paillier_oracle as O
from tests.conftest import fl, hx


def _key(g, private=True):
    k = g["key"]
    h = hx(k["h_pow_n"]) if k["djn_on"] else None
    if private:
        return O.derive_private(hx(k["p"]), hx(k["q"]), h)
    return O.derive_public(hx(k["n"]), h)


def test_key_derivation(golden):
    k = _key(golden)
    for name, val in golden["key"].items():
        if name == "djn_on":
            assert k["djn_on"] == val
        else:
            assert k[name] == hx(val), name


def _inputs(case):
    if case["kind"] == "int":
        return [hx(v) for v in case["input"]]
    return [fl(v) for v in case["input"]]


@pytest.mark.parametrize("case", ["priv_f32_p7", "pub_f32_p7", "priv_f64_none", "priv_edge_p7_noobf",
                                  "pub_f64_none_max-60", "priv_packed_p0", "pub_i32_none"])
def test_encrypt_matches_reference(golden, case):
    c = golden["encrypt"][case]
    k = _key(golden, c["private"])
    xs = _inputs(c)
    rand = [hx(r) for r in c["rand"]] if c["obfuscation"] else [None] * len(xs)
    for i, x in enumerate(xs[:golden["_cpu_limit"]]):
        m, e = O.encode_element(k, x, c["precision"], c["max_exponent"])
        assert e == c["exp"][i]
        assert O.encrypt_m(k, m, rand[i]) == hx(c["raw"][i]), (case, i)


def test_encode_errors(golden):
    k = _key(golden)
    for rec in golden["encrypt"]["encode_errors_none"]:
        x = fl(rec["x"])
        if rec["raises"] is None:
            O.encode_element(k, x, None)
        else:
            with pytest.raises(getattr(__builtins__, rec["raises"], None) or eval(rec["raises"])):
                O.encode_element(k, x, None)


@pytest.mark.parametrize("case", ["priv_f32_p7", "pub_f32_p7", "priv_f64_none", "priv_edge_p7_noobf",
                                  "pub_f64_none_max-60", "priv_packed_p0", "pub_i32_none"])
def test_decrypt_matches_reference(golden, case):
    k = _key(golden)
    enc = golden["encrypt"][case]
    dec = golden["decrypt"][case]
    ms = dec["m"][len(dec["m"]) - len(enc["raw"]):]   # np.vectorize probes element 0 once more
    for i, raw in enumerate(enc["raw"][:golden["_cpu_limit"]]):
        m = O.decrypt_raw(k, hx(raw))
        assert m == hx(ms[i])
        e = enc["exp"][i]
        o = O.decode_origin(k, m, e)
        if e < 0:
            assert o.hex() == dec["origin_f64"][i]
        else:
            assert float(o).hex() == dec["origin_f64"][i] or float(O.int_to_double_gmpy(o)).hex() == dec["origin_f64"][i]
        assert O.decode_float32(k, m, e).hex() == dec["float32"][i]


def test_decode_crafted(golden):
    k = _key(golden)
    for rec in golden["decrypt"]["crafted"]:
        m, e = hx(rec["m"]), rec["exp"]
        o = O.decode_origin(k, m, e)
        if e < 0:
            assert o.hex() == rec["origin"]
        else:
            assert o == hx(rec["origin"])
        if rec["float32"] == "OverflowError":
            with pytest.raises(OverflowError):
                O.decode_float32(k, m, e)
        else:
            assert O.decode_float32(k, m, e).hex() == rec["float32"]
    for rec in golden["decrypt"]["overflow"]:
        with pytest.raises(OverflowError):
            O.decode_origin(k, hx(rec["m"]), 0)


def _cts(d):
    return [hx(r) for r in d["raw"]], d["exp"]


def test_homomorphic_ops(golden):
    kpub = _key(golden, private=False)
    ops = golden["ops"]
    ar, ae = _cts(ops["a"])
    br, be = _cts(ops["b"])
    rr, re_ = _cts(ops["add"])
    for i in range(len(ar))[:golden["_cpu_limit"]]:
        assert O.add_ct(kpub, ar[i], ae[i], br[i], be[i]) == (rr[i], re_[i])
    rr, re_ = _cts(ops["sub"])
    for i in range(len(ar))[:golden["_cpu_limit"]]:
        nb = O.mul_ct(kpub, br[i], be[i], -1)
        assert O.add_ct(kpub, ar[i], ae[i], nb[0], nb[1]) == (rr[i], re_[i])
    sc = [fl(s) if isinstance(s, str) else s for s in ops["mul_pub"]["scalar"]]
    for name in ("mul_pub", "mul_priv"):
        rr, re_ = _cts(ops[name])
        for i in range(len(ar))[:golden["_cpu_limit"]]:
            assert O.mul_ct(kpub, ar[i], ae[i], sc[i]) == (rr[i], re_[i]), (name, i)
    rr, re_ = _cts(ops["add_scalar"])
    for i in range(len(ar))[:golden["_cpu_limit"]]:
        assert O.add_scalar(kpub, ar[i], ae[i], sc[i]) == (rr[i], re_[i])
    rr, re_ = _cts(ops["rsub_scalar"])
    for i in range(len(ar))[:golden["_cpu_limit"]]:
        neg = O.mul_ct(kpub, ar[i], ae[i], -1)
        assert O.add_scalar(kpub, neg[0], neg[1], sc[i]) == (rr[i], re_[i])
    rr, re_ = _cts(ops["truediv"])
    for i in range(len(ar))[:golden["_cpu_limit"]]:
        assert O.mul_ct(kpub, ar[i], ae[i], 1 / 4.0) == (rr[i], re_[i])
    for name in ("sum_a", "sum_pyfold"):
        rr, re_ = _cts(ops[name])
        assert O.sum_ct(kpub, ar, ae) == (rr[0], re_[0])


def test_matmul_and_hist(golden):
    if golden["_cpu_limit"]:
        pytest.skip("8192-bit mat-mul/histogram restatement is minutes of pure-Python modexp; "
                    "the GPU tests check these vectors")
    kpub = _key(golden, private=False)
    ops = golden["ops"]
    ar, ae = _cts(ops["a"])
    X = [[fl(v) for v in row] for row in ops["matmul"]["X"]]
    rr, re_ = _cts(ops["matmul"])
    for j in range(len(X[0])):
        terms = [O.mul_ct(kpub, ar[i], ae[i], float(np.float32(X[i][j]))) for i in range(len(ar))]
        acc = terms[0]
        for t in terms[1:]:
            acc = O.add_ct(kpub, acc[0], acc[1], t[0], t[1])
        assert acc == (rr[j], re_[j])
    h = ops["hist"]
    cr, ce = _cts(h["ct"])
    sr, se = _cts(h["sum"])
    for idx, b in enumerate(h["bin_ids"]):
        members = [i for i, bb in enumerate(h["bins"]) if bb == b]
        assert len(members) == h["count"][idx]
        assert O.sum_ct(kpub, [cr[i] for i in members], [ce[i] for i in members]) == (sr[idx], se[idx])


@pytest.mark.parametrize("fx", ["paillier_2048_djn.json", "paillier_2048_nodjn.json"])
def test_alignment_gap_negative_branch(fx):
    """Additions whose alignment gap d has 1 << d >= min_value_for_negative
    (the 2048-bit fixtures' gap cases): _raw_mul's negative branch gives
    c^(2^d - n) (paillier.py:79-86, 173-187). The oracle's add_ct reproduces
    the reference's bits for single adds, its left fold those of np.sum and
    Python's sum (which starts from 0 + x0 = x0 + Enc(0)); the order-free
    product does not (which is why the device path tracks the addition tree)."""
    from tests.conftest import load_fixture
    g = load_fixture(fx)
    k = _key(g, private=False)
    ops = g["ops"]
    assert ops["gap"]["dneg"] == (k["min_value_for_negative"] - 1).bit_length()
    cr, ce = _cts(ops["gap"])
    scale = fl(ops["gap"]["scale"])
    t = O.mul_ct(k, cr[0], ce[0], scale)
    t = O.mul_ct(k, t[0], t[1], scale)
    gr, ge = _cts(ops["gap_operands"])
    assert (gr[0], ge[0]) == t and gr[1:] == cr[1:] and ge[1:] == ce[1:]
    for name in ("gap_add_pub", "gap_add_priv"):
        rr, re_ = _cts(ops[name])
        for idx, (i, j) in enumerate(ops["gap"]["pairs"]):
            assert O.add_ct(k, gr[i], ge[i], gr[j], ge[j]) == (rr[idx], re_[idx]), (name, i, j)
    sr, se = _cts(ops["gap_sum"])
    pr, pe = _cts(ops["gap_pyfold"])
    differs = 0
    for idx, o in enumerate(ops["gap_sum"]["orders"]):
        acc = (gr[o[0]], ge[o[0]])
        for i in o[1:]:
            acc = O.add_ct(k, acc[0], acc[1], gr[i], ge[i])
        assert acc == (sr[idx], se[idx])
        acc = O.add_ct(k, gr[o[0]], ge[o[0]], 1, 0)  # 0 + x0 -> x0.__radd__(0) = x0 + Enc(0)
        for i in o[1:]:
            acc = O.add_ct(k, acc[0], acc[1], gr[i], ge[i])
        assert acc == (pr[idx], pe[idx])
        differs += O.sum_ct(k, [gr[i] for i in o], [ge[i] for i in o]) != (sr[idx], se[idx])
    assert differs >= 1
