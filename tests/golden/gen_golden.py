"""Golden-vector generator: runs XFL's OWN Paillier code and records its outputs.

Run ONLY in the survey container, with the interpreter that has gmpy2:

    PYTHONPATH=tests/golden/_standins:/root/reference/python \
        /opt/conda/bin/python3.9 -B tests/golden/gen_golden.py

It imports the reference package `common.crypto.paillier` from
/root/reference/python (read-only; `-B` keeps __pycache__ out of it) and makes
its randomness deterministic by replacing `secrets.SystemRandom` with a seeded
recorder, so keys (context.py:73-84, utils.py:79-89) and the obfuscation draws
(paillier.py:195,211,215,229) are reproducible and every drawn `a`/`r` is
written next to the ciphertext it produced.

Outputs small JSON fixtures into tests/golden/. Big integers are hex strings,
floats are `float.hex()` strings. Nothing from the reference is copied: the
files hold inputs and the reference's outputs only.
"""
import json
import os
import random
import secrets
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


class _Recorder(random.Random):
    """Seeded drop-in for secrets.SystemRandom that logs randrange() draws."""
    state = random.Random(0)
    log = []

    def __init__(self, seed=None):  # SystemRandom ignores seeds too
        super().__init__(0)

    def random(self):
        return _Recorder.state.random()

    def getrandbits(self, k):
        return _Recorder.state.getrandbits(k)

    def randrange(self, start, stop=None, step=1):
        v = _Recorder.state.randrange(start, stop, step)
        _Recorder.log.append(v)
        return v


secrets.SystemRandom = _Recorder

import gmpy2  # noqa: E402
import pandas as pd  # noqa: E402
from algorithm.core.paillier_acceleration import embed  # noqa: E402
from common.crypto.paillier import encoder as enc_mod  # noqa: E402
from common.crypto.paillier.context import PaillierContext  # noqa: E402
from common.crypto.paillier.paillier import Paillier, PaillierCiphertext  # noqa: E402

_decode_log = []
_orig_decode = enc_mod.PaillierEncoder.decode_single.__func__


def _logged_decode(cls, context, data, exponent):
    _decode_log.append((int(data), int(exponent)))
    return _orig_decode(cls, context, data, exponent)


enc_mod.PaillierEncoder.decode_single = classmethod(_logged_decode)


def H(x):
    return hex(int(x))


def F(x):
    return float(x).hex()


def key_record(ctx):
    d = {"n": H(ctx.n), "n_square": H(ctx.n_square),
         "max_value_for_positive": H(ctx.max_value_for_positive),
         "min_value_for_negative": H(ctx.min_value_for_negative),
         "djn_on": bool(ctx.djn_on)}
    if ctx.is_private():
        for k in ("p", "q"):
            d[k] = H(getattr(ctx, k))
        for k in ("q_inverse_p", "p_square", "q_square", "q2_inverse_p2", "hp", "hq",
                  "phi_p2", "phi_q2", "ep", "eq"):
            d[k] = H(getattr(ctx, k))
    if ctx.djn_on:
        d["h_pow_n"] = H(ctx.h_pow_n)
        d["djn_exp_bound"] = H(ctx.djn_exp_bound)
        if ctx.is_private():
            d["h_pow_n_modp2"] = H(ctx.h_pow_n_modp2)
            d["h_pow_n_modq2"] = H(ctx.h_pow_n_modq2)
    return d


def cts(arr):
    flat = np.asarray(arr, dtype=object).reshape(-1)
    return {"raw": [H(c.raw_ciphertext) for c in flat], "exp": [int(c.exponent) for c in flat]}


def encrypt_case(ctx, data, precision, max_exponent=None, obfuscation=True, kind="f64"):
    _Recorder.log.clear()
    c = Paillier.encrypt(ctx, data, precision=precision, max_exponent=max_exponent,
                         obfuscation=obfuscation, num_cores=1)
    rnd = list(_Recorder.log)
    if kind == "int":
        inp = [H(int(x)) if int(x) >= 0 else "-" + H(-int(x)) for x in data.reshape(-1)]
    else:
        inp = [F(x) for x in np.asarray(data, dtype=np.float64).reshape(-1)]
    rec = {"kind": kind, "input": inp, "precision": precision, "max_exponent": max_exponent,
           "obfuscation": obfuscation, "private": ctx.is_private(),
           "rand": [H(r) for r in rnd]}
    rec.update(cts(c))
    return rec, c


def decrypt_case(priv, c):
    _decode_log.clear()
    origin = Paillier.decrypt(priv, c, num_cores=1, out_origin=True)
    dec = list(_decode_log)
    f32 = Paillier.decrypt(priv, c, num_cores=1, dtype="float")
    rec = {"m": [H(m) for m, _ in dec], "m_exp": [e for _, e in dec],
           "origin_f64": [F(v) for v in origin.reshape(-1)],
           "float32": [F(np.float64(v)) for v in f32.reshape(-1)]}
    return rec


def gen_key_fixture(bits, djn, seed, n_vec):
    _Recorder.state = random.Random(seed)
    priv = Paillier.context(bits, djn_on=djn)
    pub = priv.to_public()
    rng = np.random.default_rng(seed)
    out = {"key_bits": bits, "seed": seed, "key": key_record(priv), "encrypt": {}, "decrypt": {}, "ops": {}}

    # Encrypt: label-trainer residual path (float32, precision 7, private CRT).
    x32 = (rng.random(n_vec).astype(np.float32) * 100 - 50).astype(np.float32)
    x32[:4] = np.array([0.0, -0.0, 1.0, -1.0], dtype=np.float32)
    r, c_p7 = encrypt_case(priv, x32, 7, kind="f32")
    out["encrypt"]["priv_f32_p7"] = r
    out["decrypt"]["priv_f32_p7"] = decrypt_case(priv, c_p7)

    # Same data with the public context (remote-party path).
    r, c_pub = encrypt_case(pub, x32, 7, kind="f32")
    out["encrypt"]["pub_f32_p7"] = r
    out["decrypt"]["pub_f32_p7"] = decrypt_case(priv, c_pub)

    # float64, precision None (frexp exponents), private.
    x64 = rng.standard_normal(n_vec) * np.exp2(rng.integers(-30, 30, n_vec))
    x64[:6] = [1e-200, -2.0 ** -960, 2.0 ** 52, -(2.0 ** 52) + 1, 0.1, 12345.678]
    r, c_none = encrypt_case(priv, x64, None, kind="f64")
    out["encrypt"]["priv_f64_none"] = r
    errs = []
    for v in [1e-300, -2.0 ** -980, float("inf"), float("nan"), 2.0 ** 60]:
        try:
            Paillier.encrypt(priv, np.array([v]), precision=None, obfuscation=False, num_cores=1)
            errs.append({"x": F(v), "raises": None})
        except (OverflowError, ValueError) as exc:
            errs.append({"x": F(v), "raises": type(exc).__name__})
    out["encrypt"]["encode_errors_none"] = errs
    out["decrypt"]["priv_f64_none"] = decrypt_case(priv, c_none)

    # Rounding edge cases at precision 7 (exponent -24), no obfuscation.
    u = 2.0 ** -24
    xe = np.array([0.5 * u, 1.5 * u, 2.5 * u, -0.5 * u, -1.5 * u, -2.5 * u, 3.5 * u,
                   0.49999999 * u, 1e-9, -1e-9, 123456.789, -98765.4321], dtype=np.float64)
    r, c_edge = encrypt_case(priv, xe, 7, obfuscation=False, kind="f64")
    out["encrypt"]["priv_edge_p7_noobf"] = r
    out["decrypt"]["priv_edge_p7_noobf"] = decrypt_case(priv, c_edge)

    # max_exponent clamp, public context.
    r, c_mx = encrypt_case(pub, x64[:16], None, max_exponent=-60, kind="f64")
    out["encrypt"]["pub_f64_none_max-60"] = r
    out["decrypt"]["pub_f64_none_max-60"] = decrypt_case(priv, c_mx)

    # Packed ints (XGBoost histogram config): embed(grad, hess), precision 0.
    g = rng.random(16) - 0.5
    h = rng.random(16) * 0.25
    packed = embed([g, h])
    r, c_pk = encrypt_case(priv, packed, 0, kind="int")
    out["encrypt"]["priv_packed_p0"] = r
    out["decrypt"]["priv_packed_p0"] = decrypt_case(priv, c_pk)
    out["encrypt"]["priv_packed_p0"]["g"] = [F(v) for v in g]
    out["encrypt"]["priv_packed_p0"]["h"] = [F(v) for v in h]

    # int32 inputs with precision None (exponent 0), public.
    xi = rng.integers(-1000, 1000, 16).astype(np.int32)
    r, c_i = encrypt_case(pub, xi, None, kind="int")
    out["encrypt"]["pub_i32_none"] = r
    dec = decrypt_case(priv, c_i)
    dec["int32"] = [int(v) for v in Paillier.decrypt(priv, c_i, num_cores=1, dtype="int")]
    out["decrypt"]["pub_i32_none"] = dec

    # Decode edge cases: crafted encoded numbers (double rounding, overflow).
    n = priv.n
    crafted = []
    for m, e in [((1 << 54) + (1 << 30) + 1, -54), (n - ((1 << 54) + (1 << 30) + 1), -54),
                 ((1 << 53) + 1, -1), (1 << 200, -190), (int(priv.max_value_for_positive), -2000),
                 (int(priv.min_value_for_negative), 0), (7, 3)]:
        c = PaillierCiphertext(priv, (n * m + 1) % priv.n_square, e)
        _decode_log.clear()
        v = Paillier.decrypt(priv, c, num_cores=1, out_origin=True)
        try:
            f32 = F(np.float64(np.array([v]).astype(np.float32)[0]))
        except OverflowError:
            f32 = "OverflowError"
        ov = int(v)
        crafted.append({"m": H(m), "exp": e, "origin": F(v) if e < 0 else (H(ov) if ov >= 0 else "-" + H(-ov)),
                        "float32": f32})
    out["decrypt"]["crafted"] = crafted
    over = []
    for m in [int(priv.max_value_for_positive) + 1, int(priv.min_value_for_negative) - 1]:
        c = PaillierCiphertext(priv, (n * m + 1) % priv.n_square, 0)
        try:
            Paillier.decrypt(priv, c, num_cores=1)
            over.append({"m": H(m), "raises": None})
        except OverflowError:
            over.append({"m": H(m), "raises": "OverflowError"})
    out["decrypt"]["overflow"] = over

    # Homomorphic operations, public context (the trainer side) and private (CRT branch).
    a_vals = x64[:16]
    b_vals = (rng.standard_normal(16) * 1e3)
    _, ca = encrypt_case(pub, a_vals, None, kind="f64")
    _, cb = encrypt_case(pub, b_vals, None, kind="f64")
    ops = out["ops"]
    ops["a"] = dict(cts(ca), input=[F(v) for v in a_vals])
    ops["b"] = dict(cts(cb), input=[F(v) for v in b_vals])
    ops["add"] = cts(ca + cb)
    ops["sub"] = cts(ca - cb)
    scal = [2.0, -2.0, 0.5, -0.37, 3, -3, -1, 1, 1e-7, -123456.0, 0.0, 7.25e10, -1e-12, 65536, 12, -5]
    for ctx_name, base in (("pub", ca), ("priv", Paillier.ciphertext_from(priv, Paillier.serialize(ca, compression=False), compression=False))):
        ops[f"mul_{ctx_name}"] = dict(cts(np.array([base[i] * scal[i] for i in range(16)], dtype=object)),
                                      scalar=[F(s) if isinstance(s, float) else s for s in scal])
    ops["add_scalar"] = dict(cts(np.array([ca[i] + scal[i] for i in range(16)], dtype=object)),
                             scalar=[F(s) if isinstance(s, float) else s for s in scal])
    ops["rsub_scalar"] = dict(cts(np.array([scal[i] - ca[i] for i in range(16)], dtype=object)),
                              scalar=[F(s) if isinstance(s, float) else s for s in scal])
    ops["truediv"] = cts(ca / 4.0)
    ops["sum_a"] = cts(np.array([np.sum(ca)], dtype=object))
    ops["sum_pyfold"] = cts(np.array([sum(ca)], dtype=object))
    # Vertical-LR gradient: enc(residual)[B] @ X[B x D] (logistic_regression/trainer.py:166).
    X = rng.standard_normal((16, 3)).astype(np.float32)
    ops["matmul"] = dict(cts(np.matmul(ca, X)), X=[[F(v) for v in row] for row in X.astype(np.float64)])
    # Decrypt of op outputs.
    ops["decrypt_add"] = decrypt_case(priv, ca + cb)
    ops["decrypt_matmul"] = decrypt_case(priv, np.matmul(ca, X))

    # HE histogram: groupby-sum of packed-int ciphertexts (decision_tree_trainer.py:151-160).
    gg = rng.random(40) - 0.5
    hh = rng.random(40) * 0.25
    _, chist = encrypt_case(priv, embed([gg, hh]), 0, kind="int")
    bins = rng.integers(0, 4, 40)
    df = pd.DataFrame({"bin": bins, "xfl_grad_hess": chist})
    agg = df.groupby(["bin"])["xfl_grad_hess"].agg(["count", "sum"])
    ops["hist"] = {"ct": cts(chist), "bins": [int(b) for b in bins],
                   "g": [F(v) for v in gg], "h": [F(v) for v in hh],
                   "bin_ids": [int(i) for i in agg.index], "count": [int(v) for v in agg["count"]],
                   "sum": cts(np.array(list(agg["sum"]), dtype=object))}
    # Wire format: pickle of RawCiphertext objects (paillier.py:244-258), uncompressed.
    ops["wire_a4"] = Paillier.serialize(ca[:4], compression=False).hex()
    ops["wire_ctx_pub"] = pub.serialize().hex()
    if bits == 2048:
        # Alignment across gaps of ~bitlen(n) exponent steps:
        # _decrease_exponent_to's scalar 1 << d reaches min_value_for_negative
        # and _raw_mul takes its negative branch (paillier.py:79-86, 173-187).
        # Encoded floats have exponents in [-1023, 0] (a float scalar at
        # precision None as well), so the small operand is a product: Enc(1.0) *
        # 2^-960 * 2^-960, exponent -2076. Exponents of gc: -2076, -31, -30, -29,
        # -28, -36, 0, -49 (gaps to gc[0]: 2045 .. 2048, 2040, 2076, 2027).
        gx = np.array([1.0, 2.0 ** 21, -1.5 * 2.0 ** 22, 2.0 ** 23, 2.0 ** 24, -(2.0 ** 16), 1.5 * 2.0 ** 52, 12.5],
                      dtype=np.float64)
        scale = 2.0 ** -960
        _, cg = encrypt_case(pub, gx, None, kind="f64")
        gc = np.array([cg[0] * scale * scale] + list(cg[1:]), dtype=object)
        gcp = Paillier.ciphertext_from(priv, Paillier.serialize(gc, compression=False), compression=False)
        pairs = [(0, 1), (1, 0), (0, 2), (0, 3), (3, 0), (0, 4), (0, 5), (5, 0), (0, 6), (0, 7), (7, 7), (1, 6)]
        ops["gap"] = dict(cts(cg), input=[F(v) for v in gx], scale=F(scale), pairs=pairs,
                          dneg=(int(priv.min_value_for_negative) - 1).bit_length())
        ops["gap_operands"] = cts(gc)
        ops["gap_add_pub"] = cts(np.array([gc[i] + gc[j] for i, j in pairs], dtype=object))
        ops["gap_add_priv"] = cts(np.array([gcp[i] + gcp[j] for i, j in pairs], dtype=object))
        orders = [[6, 5, 0, 7, 2], [6, 0, 4, 1], [3, 6, 0, 2], [0, 6, 1]]
        ops["gap_sum"] = dict(cts(np.array([np.sum(gc[o]) for o in orders], dtype=object)), orders=orders)
        ops["gap_pyfold"] = cts(np.array([sum(gc[o]) for o in orders], dtype=object))
    return out


def main():
    warnings.simplefilter("ignore")
    specs = [("paillier_2048_djn.json", 2048, True, 11, 48),
             ("paillier_2048_nodjn.json", 2048, False, 12, 24),
             ("paillier_3072_djn.json", 3072, True, 13, 16),
             ("paillier_4096_djn.json", 4096, True, 14, 16),
             ("paillier_8192_djn.json", 8192, True, 15, 16)]
    only = set(sys.argv[1:])
    for fname, bits, djn, seed, nvec in specs:
        if only and fname not in only:
            continue
        fx = gen_key_fixture(bits, djn, seed, nvec)
        fx["generator"] = {"python": sys.version.split()[0], "gmpy2": gmpy2.version(),
                           "numpy": np.__version__, "pandas": pd.__version__}
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump(fx, f, indent=0)
        print("wrote", fname, os.path.getsize(os.path.join(HERE, fname)), "bytes")


if __name__ == "__main__":
    main()
