"""CPU restatement of XFL's Paillier hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle. It is imported only by tests/, by
`__graft_entry__.smoke()` and by bench.py's `cpu_baseline` leg, always as the
checker and never as the thing measured or shipped. The product path
(xfl_amd.paillier) must never import it.

Parity pinning: every function below is checked against the golden vectors in
tests/golden/*.json, which were produced by running the reference's own code
(`/root/reference/python/common/crypto/paillier`, gmpy2 2.0.8 / GMP 6.2.1) via
tests/golden/gen_golden.py. Pure Python ints only (no gmpy2 here).

Reference paths are relative to /root/reference/python.
"""
import math
from fractions import Fraction  # noqa: F401  (kept for callers that want exact values)

MANT_DIG = 53


# --------------------------------------------------------------------------- keys
def l_function(x, p):
    """common/crypto/paillier/context.py:190-191"""
    return (x - 1) // p


def derive_private(p, q, h_pow_n=None):
    """PaillierContext.init with p, q (context.py:28-71)."""
    n = p * q
    k = {"p": p, "q": q, "n": n}
    k["q_inverse_p"] = pow(q, -1, p)                                  # :43
    k["p_square"] = p * p                                             # :44
    k["q_square"] = q * q                                             # :45
    k["q2_inverse_p2"] = pow(k["q_square"], -1, k["p_square"])       # :46
    k["hp"] = pow(l_function(pow(n + 1, p - 1, k["p_square"]), p), -1, p)  # :47,193-194
    k["hq"] = pow(l_function(pow(n + 1, q - 1, k["q_square"]), q), -1, q)  # :48
    k["phi_p2"] = p * (p - 1)                                         # :49
    k["phi_q2"] = q * (q - 1)                                         # :50
    k["ep"] = n % k["phi_p2"]                                         # :51
    k["eq"] = n % k["phi_q2"]                                         # :52
    _common(k, h_pow_n)
    if h_pow_n:
        k["h_pow_n_modp2"] = h_pow_n % k["p_square"]                 # :63
        k["h_pow_n_modq2"] = h_pow_n % k["q_square"]                 # :64
    k["private"] = True
    return k


def derive_public(n, h_pow_n=None):
    """PaillierContext.init with n only (context.py:54-56)."""
    k = {"n": n, "private": False}
    _common(k, h_pow_n)
    return k


def _common(k, h_pow_n):
    n = k["n"]
    if h_pow_n:                                                       # :58-61
        k["h_pow_n"] = h_pow_n
        k["djn_exp_bound"] = 2 ** (n.bit_length() // 2)
        k["djn_on"] = True
    else:
        k["djn_on"] = False
    k["n_square"] = n * n                                             # :68
    k["max_value_for_positive"] = n // 3                              # :69
    k["min_value_for_negative"] = n - k["max_value_for_positive"]     # :70


def to_public(k):
    """context.py:105-121 (DJN h_pow_n survives to_public, not serialize)."""
    return derive_public(k["n"], k.get("h_pow_n"))


# ------------------------------------------------------------------------- encode
def cal_exponent_float(x, precision):
    """encoder.py:29-46 for a float element (paillier.py:279)."""
    if precision is None:
        return math.frexp(x)[1] - MANT_DIG
    return -math.ceil(math.log2(10) * precision)


def cal_exponent_int(precision):
    """encoder.py:29-46 for an int element."""
    if precision is None:
        return 0
    return -math.ceil(math.log2(10) * precision)


def encode(k, x, e):
    """encoder.py:48-54: round(x * (1 << -e)) % n; raises like the reference.

    For floats `x * (1 << -e)` converts the shift to float (OverflowError at
    >= 2**1024, ValueError for a negative shift), multiplies exactly (power of
    two) and round() is round-half-even; inf -> OverflowError, nan -> ValueError.
    """
    return round(x * (1 << -e)) % k["n"]


def encode_element(k, x, precision, max_exponent=None):
    """Paillier._encrypt_single encode part (paillier.py:279-282)."""
    if isinstance(x, int):
        e = cal_exponent_int(precision)
    else:
        e = cal_exponent_float(x, precision)
    if max_exponent is not None:
        e = min(e, max_exponent)
    return encode(k, x, e), e


# ------------------------------------------------------------------------ encrypt
def raw_encrypt(k, m):
    """paillier.py:283"""
    return (k["n"] * m + 1) % k["n_square"]


def crt(mp, mq, p, q, q_inverse, n):
    """utils.py:38-43"""
    u = ((mp - mq) * q_inverse) % p
    return (mq + u * q) % n


def obfuscator(k, rand):
    """PaillierCiphertext.obfuscate (paillier.py:189-230) given the drawn a / r."""
    n2 = k["n_square"]
    if k["djn_on"]:
        if k["private"]:
            mp = pow(k["h_pow_n_modp2"], rand % k["phi_p2"], k["p_square"])   # :207
            mq = pow(k["h_pow_n_modq2"], rand % k["phi_q2"], k["q_square"])   # :208
            return crt(mp, mq, k["p_square"], k["q_square"], k["q2_inverse_p2"], n2)
        return pow(k["h_pow_n"], rand, n2)                                    # :212
    if k["private"]:
        mp = pow(rand % k["p_square"], k["ep"], k["p_square"])                # :225
        mq = pow(rand % k["q_square"], k["eq"], k["q_square"])                # :226
        return crt(mp, mq, k["p_square"], k["q_square"], k["q2_inverse_p2"], n2)
    return pow(rand, k["n"], n2)                                              # :230


def obfuscate(k, c, rand):
    """paillier.py:231"""
    return (c * obfuscator(k, rand)) % k["n_square"]


def encrypt_m(k, m, rand=None):
    """(n*m+1) mod n^2, then obfuscate with the given draw (None = no obfuscation)."""
    c = raw_encrypt(k, m)
    return c if rand is None else obfuscate(k, c, rand)


# ------------------------------------------------------------------------ decrypt
def decrypt_raw(k, c):
    """Paillier._decrypt_single arithmetic (paillier.py:347-365) -> encoded m."""
    p, q = k["p"], k["q"]
    mp = l_function(pow(c, p - 1, k["p_square"]), p) * k["hp"] % p
    mq = l_function(pow(c, q - 1, k["q_square"]), q) * k["hq"] % q
    return crt(mp, mq, p, q, k["q_inverse_p"], k["n"])


def signed_value(k, m):
    """decode_single sign handling (encoder.py:57-61)."""
    if m >= k["min_value_for_negative"]:
        return m - k["n"]
    if m > k["max_value_for_positive"]:
        raise OverflowError("Overflow detected during decoding encrypted number.")
    return m


def _rne53_scaled(v, e):
    """float(gmpy2.mul(mpz(v), 2.0**e)) for e < 0 (encoder.py:63).

    2.0**e is a Python float (0.0 below 2**-1074). gmpy2's mpfr product is the
    exact product rounded to 53 bits (unbounded exponent); float() then maps
    it to a double (overflow -> inf, subnormal -> second rounding).
    """
    twoe = 2.0 ** e
    if twoe == 0.0 or v == 0:
        return math.copysign(0.0, -1.0 if v < 0 else 1.0) if twoe == 0.0 else 0.0
    s = -1.0 if v < 0 else 1.0
    a = -v if v < 0 else v
    bl = a.bit_length()
    if bl > 53:
        sh = bl - 53
        qv = a >> sh
        rem = a & ((1 << sh) - 1)
        half = 1 << (sh - 1)
        if rem > half or (rem == half and (qv & 1)):
            qv += 1
        a, shift = qv, sh
    else:
        shift = 0
    exp2 = shift + e
    top = a.bit_length() + exp2          # value in [2^(top-1), 2^top)
    if top > 1024:
        return s * math.inf
    if top <= -1021:                     # subnormal: second rounding (RNE)
        return s * _ldexp_rne(a, exp2)
    return s * math.ldexp(float(a), exp2)


def _ldexp_rne(a, exp2):
    """Round a * 2**exp2 (a int > 0) to the double subnormal grid, RNE."""
    sh = -1074 - exp2                    # bits to drop
    if sh <= 0:
        return math.ldexp(float(a), exp2)
    qv = a >> sh
    rem = a & ((1 << sh) - 1)
    half = 1 << (sh - 1)
    if rem > half or (rem == half and (qv & 1)):
        qv += 1
    return math.ldexp(float(qv), -1074)


def decode_origin(k, m, e):
    """decode_single output (encoder.py:57-64): float for e<0, int for e>=0."""
    v = signed_value(k, m)
    if e < 0:
        return _rne53_scaled(v, e)
    return v * (1 << e)


def int_to_double_gmpy(v):
    """float(mpz) under gmpy2 2.0.8: truncation toward zero (measured in the
    fixture interpreter); OverflowError above the double range."""
    a = -v if v < 0 else v
    bl = a.bit_length()
    if bl > 1024:
        raise OverflowError("'mpz' too large to convert to float")
    if bl > 53:
        a = (a >> (bl - 53)) << (bl - 53)
    return -float(a) if v < 0 else float(a)


def decode_float32(k, m, e):
    """Paillier.decrypt(..., dtype='float') element: astype(np.float32) of the
    decode_single output (paillier.py:396-398) -> double, then RNE to float32."""
    import numpy as np
    o = decode_origin(k, m, e)
    d = o if isinstance(o, float) else int_to_double_gmpy(o)
    with np.errstate(over="ignore"):
        return float(np.float32(d))


# ------------------------------------------------------------------ homomorphic
def raw_mul(k, c, s, n_private=None):
    """PaillierCiphertext._raw_mul for 0 <= s < n (paillier.py:156-187).

    Both branches (CRT / public) produce the same residue; this is the public
    form: inv(c)^(n-s) for s >= min_neg else c^s, mod n^2.
    """
    n2 = k["n_square"]
    if s >= k["min_value_for_negative"]:
        return pow(pow(c, -1, n2), k["n"] - s, n2)
    return pow(c, s, n2)


def decrease_exponent(k, c, e_from, e_to):
    """paillier.py:79-86"""
    return raw_mul(k, c, 1 << (e_from - e_to))


def add_ct(k, c1, e1, c2, e2):
    """paillier.py:106-123 -> (raw, exponent)."""
    if e1 > e2:
        return (decrease_exponent(k, c1, e1, e2) * c2) % k["n_square"], e2
    if e1 < e2:
        return (c1 * decrease_exponent(k, c2, e2, e1)) % k["n_square"], e1
    return (c1 * c2) % k["n_square"], e1


def encode_scalar(k, s):
    """__mul__ scalar encoding: precision=None (paillier.py:138-139)."""
    if isinstance(s, int):
        e = 0
    else:
        e = math.frexp(s)[1] - MANT_DIG
    return encode(k, s, e), e


def mul_ct(k, c, e, s):
    """paillier.py:134-145 -> (raw, exponent)."""
    ks, es = encode_scalar(k, s)
    return raw_mul(k, c, ks), e + es


def add_scalar(k, c, e, s):
    """paillier.py:95-102: encrypt(s, precision=None, obfuscation=False) then add."""
    m, es = encode_scalar(k, s)
    return add_ct(k, c, e, raw_encrypt(k, m), es)


def sum_ct(k, raws, exps):
    """Order-free homomorphic sum (A.9): prod c_i^(2^(e_i-e_min)) mod n^2."""
    emin = min(exps)
    acc = 1
    n2 = k["n_square"]
    for c, e in zip(raws, exps):
        acc = acc * pow(c, 1 << (e - emin), n2) % n2
    return acc, emin


# ------------------------------------------------------------------ packing
def embed_ref(p_list, interval=1 << 128, precision=64):
    """algorithm/core/paillier_acceleration.py:21-32, element by element."""
    out = []
    for i in range(len(p_list[0])):
        x = int(p_list[0][i] * (1 << precision))
        for j in range(len(p_list) - 1):
            x = x * interval + int(p_list[j + 1][i] * (1 << precision))
        out.append(x)
    return out


def umbed_ref(a, num, interval=1 << 128, precison=64):
    """algorithm/core/paillier_acceleration.py:35-59 -> num lists of float32."""
    import numpy as np
    out = [[0] * len(a) for _ in range(num)]
    for i, x in enumerate(a):
        res = [0] * num
        b = x % interval
        if abs(b) > interval // 2:
            b = b - interval
        a2 = (x - b) // interval
        res[-1] = b / (1 << precison)
        for k in range(num - 1):
            b = a2 % interval
            if abs(b) > interval // 2:
                b = b - interval
            a2 = (a2 - b) // interval
            res[-k - 2] = b / (1 << precison)
        t = np.array(res).astype(np.float32)
        for j in range(num):
            out[j][i] = t[j]
    return out


def unpack_ref(x, num, interval=1 << 128, precison=64):
    """algorithm/core/paillier_acceleration.py:62-81."""
    res = [0] * num
    b = x % interval
    if abs(b) > interval // 2:
        b = b - interval
    a = (x - b) // interval
    res[-1] = float(b / (1 << precison))
    for i in range(num - 1):
        b = a % interval
        if abs(b) > interval // 2:
            b = b - interval
        a = (a - b) // interval
        res[-i - 2] = float(b / (1 << precison))
    return res
