# Portions mirror the API of XFL (python/common/crypto/paillier), Copyright 2022
# The XFL Authors, licensed under the Apache License, Version 2.0
# (http://www.apache.org/licenses/LICENSE-2.0): the method names, arguments and
# spec formulas of the drop-in interface follow that file.
"""PaillierEncoder — drop-in for python/common/crypto/paillier/encoder.py.

Scalar helpers with the reference semantics (encoder.py:26-64). Array
encoding/decoding of the hot path runs on the GPU (k_encode_f64, k_decode);
these scalar forms serve single-element operations and host-side decode of
`out_origin=True` results.
"""
import math
import sys
from typing import Optional, Union

import numpy as np


def _rne53_times_pow2(v: int, e: int) -> float:
    """float(gmpy2.mul(mpz(v), 2.0**e)) for e < 0 (encoder.py:63).

    2.0**e is a Python float (0.0 below 2**-1074); the mpfr product is the
    exact product rounded to 53 bits with unbounded exponent; float() then maps
    it to a double (overflow -> inf, subnormal range rounded again).
    """
    twoe = 2.0 ** e
    if twoe == 0.0:
        return -0.0 if v < 0 else 0.0
    if v == 0:
        return 0.0
    neg = v < 0
    a = -v if neg else v
    bl = a.bit_length()
    shift = 0
    if bl > 53:
        shift = bl - 53
        q = a >> shift
        rem = a & ((1 << shift) - 1)
        half = 1 << (shift - 1)
        if rem > half or (rem == half and (q & 1)):
            q += 1
        a = q
    ex = shift + e
    top = a.bit_length() + ex
    if top > 1024:
        r = math.inf
    elif top <= -1021:
        sh = -1074 - ex
        if sh > 0:
            q = a >> sh
            rem = a & ((1 << sh) - 1)
            half = 1 << (sh - 1)
            if rem > half or (rem == half and (q & 1)):
                q += 1
            r = math.ldexp(float(q), -1074)
        else:
            r = math.ldexp(float(a), ex)
    else:
        r = math.ldexp(float(a), ex)
    return -r if neg else r


class PaillierEncoder(object):
    _MANT_DIG = sys.float_info.mant_dig

    @classmethod
    def cal_exponent(cls, data: Union[int, float, np.ndarray], precision: Optional[int] = None):
        """encoder.py:29-46"""
        if precision is None:
            if isinstance(data, np.ndarray):
                exponent = np.frexp(data)[1] - cls._MANT_DIG
            elif isinstance(data, (np.int32, np.int64, int, np.int16)):
                exponent = 0
            elif isinstance(data, (np.float32, np.float64, float, np.float16,)):
                exponent = math.frexp(data)[1] - cls._MANT_DIG
            else:
                raise TypeError(f"Precision type {type(precision)} not supported.")
        else:
            exponent = -math.ceil(math.log2(10) * precision)
        return exponent

    @classmethod
    def encode_single(cls, context, data, exponent: int) -> int:
        """encoder.py:48-54"""
        return round(data * (1 << -exponent)) % context.n

    @classmethod
    def decode_single(cls, context, data: int, exponent: int):
        """encoder.py:56-64: float (mpfr semantics) for exponent < 0, exact int otherwise."""
        data = int(data)
        if data >= context.min_value_for_negative:
            data -= context.n
        elif data > context.max_value_for_positive:
            raise OverflowError("Overflow detected during decoding encrypted number.")
        if exponent < 0:
            return _rne53_times_pow2(data, exponent)
        return data * (1 << exponent)


def int_to_float_gmpy(v: int) -> float:
    """float() of the mpz an integer decode returns (gmpy2 2.0.8 truncates)."""
    a = -v if v < 0 else v
    bl = a.bit_length()
    if bl > 1024:
        raise OverflowError("'mpz' too large to convert to float")
    if bl > 53:
        a = (a >> (bl - 53)) << (bl - 53)
    return -float(a) if v < 0 else float(a)
