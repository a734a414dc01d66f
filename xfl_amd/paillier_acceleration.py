"""Drop-in for python/algorithm/core/paillier_acceleration.py: packing several
fixed-point values into one Paillier plaintext (SecureBoost grad/hess,
decision_tree_label_trainer.py:108-119) and unpacking decrypted sums.

Same functions, arguments and results as the reference:
  embed(p_list, interval=2^128, precision=64)   paillier_acceleration.py:21-32
      x = int(p0 * 2^precision) * interval^(k-1) + ... (int() truncates toward 0)
  umbed(a, num, interval=2^128, precison=64)    :35-59  centred base-`interval`
      digits, each / 2^precision (correctly rounded true division) -> float32
  unpack(x, num, ...)                           :62-81  one value, Python floats

embed is vectorised: for the reference's (interval, precision) the scaled
integers int(v * 2^precision) are formed exactly from each float's mantissa
and exponent (numpy, no per-element Python float arithmetic), then the packed
Python ints are assembled; umbed / unpack work on Python ints exactly as the
reference does (their inputs are decrypted Python ints).
"""
from typing import List

import numpy as np


def _scaled_ints(v: np.ndarray, precision: int) -> List[int]:
    """[int(x * (1 << precision)) for x in v] for a float array, exactly:
    x * 2^p is exact in binary floating point (a power-of-two scale, no
    overflow for |x| < 2^(1024-p)), int() truncates toward zero."""
    v = np.asarray(v, dtype=np.float64)
    if not np.all(np.isfinite(v)):
        raise OverflowError("cannot convert float infinity to integer")
    mant, exp = np.frexp(v)  # v = mant * 2^exp, 0.5 <= |mant| < 1
    m53 = (mant * (1 << 53)).astype(np.int64)  # exact 53-bit signed mantissa
    sh = exp.astype(np.int64) - 53 + precision  # v * 2^p = m53 * 2^sh
    out = []
    for m, s in zip(m53.tolist(), sh.tolist()):
        if s >= 0:
            out.append(m << s)
        else:
            a = (-m if m < 0 else m) >> (-s)  # truncation toward zero
            out.append(-a if m < 0 else a)
    return out


def embed(p_list: List[np.ndarray], interval: int = (1 << 128), precision: int = 64):
    """paillier_acceleration.py:21-32"""
    cols = [_scaled_ints(p, precision) for p in p_list]
    out = [0] * len(cols[0])
    for i in range(len(out)):
        x = cols[0][i]
        for c in cols[1:]:
            x = x * interval + c[i]
        out[i] = x
    return np.array(out)


def _centred_digits(x, num: int, interval: int):
    res = [0] * num
    b = x % interval
    if abs(b) > interval // 2:
        b = b - interval
    a = (x - b) // interval
    res[-1] = b
    for i in range(num - 1):
        b = a % interval
        if abs(b) > interval // 2:
            b = b - interval
        a = (a - b) // interval
        res[-i - 2] = b
    return res


def umbed(a: np.ndarray, num: int, interval: int = (1 << 128), precison: int = 64) -> List[list]:
    """paillier_acceleration.py:35-59 (argument name `precison` as in the reference)."""
    scale = 1 << precison
    out = [[0] * len(a) for _ in range(num)]
    for i in range(len(a)):
        digits = _centred_digits(a[i], num, interval)
        temp = np.array([d / scale for d in digits]).astype(np.float32)
        for j in range(num):
            out[j][i] = temp[j]
    return out


def unpack(x: float, num: int, interval: int = (1 << 128), precison: int = 64) -> List[list]:
    """paillier_acceleration.py:62-81"""
    scale = 1 << precison
    return [float(d / scale) for d in _centred_digits(x, num, interval)]
