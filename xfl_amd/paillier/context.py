# Portions mirror the API of XFL (python/common/crypto/paillier), Copyright 2022
# The XFL Authors, licensed under the Apache License, Version 2.0
# (http://www.apache.org/licenses/LICENSE-2.0): the method names, arguments and
# spec formulas of the drop-in interface follow that file.
"""PaillierContext — drop-in for python/common/crypto/paillier/context.py.

Same constructor/init/generate/serialize surface and attribute names as the
reference (context.py:27-194). Key material is plain Python ints; the
device-resident key (constants + fixed-base tables, include/xhe.h
xhe_key_create) is built lazily on first use and cached per context.
"""
import math
import os
import pickle
import secrets
import threading
import warnings
from typing import Optional

from .utils import getprimeover, invert

SUPPORTED_DEVICE_BITS = (2048, 3072, 4096, 8192)
_KEY_LOCK = threading.Lock()


def device_key_bits(n):
    """Key size class of n for the device kernels (bitlen(n) in {K-1, K})."""
    bl = n.bit_length()
    for k in SUPPORTED_DEVICE_BITS:
        if k - 2 <= bl <= k:
            return k
    raise NotImplementedError(f"device Paillier supports {SUPPORTED_DEVICE_BITS}-bit keys, got n of {bl} bits")


class PaillierContext(object):
    def init(self, p: Optional[int] = None, q: Optional[int] = None, n: Optional[int] = None,
             djn_h_pow_n: Optional[int] = None):
        """context.py:28-71"""
        if n is None and (p is None or q is None):
            raise ValueError("Insufficient parameters.")
        self._dev = {}
        if p is not None and q is not None:
            p, q = int(p), int(q)
            self.__p = p
            self.__q = q
            self.__n = p * q
            if n is not None and self.__n != n:
                warnings.warn(f"Input n {n} not equal to p * q {self.__n}, use p * q instead.")
            self.q_inverse_p = invert(q, p)
            self.p_square = p * p
            self.q_square = q * q
            self.q2_inverse_p2 = invert(self.q_square, self.p_square)
            self.hp = self._h_function(p, self.p_square)
            self.hq = self._h_function(q, self.q_square)
            self.phi_p2 = p * (p - 1)
            self.phi_q2 = q * (q - 1)
            self.ep = self.__n % self.phi_p2
            self.eq = self.__n % self.phi_q2
            self.__is_private = True
        else:
            self.__n = int(n)
            self.__is_private = False

        if djn_h_pow_n:
            self.h_pow_n = int(djn_h_pow_n)
            self.djn_exp_bound = pow(2, self.__n.bit_length() // 2)
            self.djn_on = True
            if self.__is_private:
                self.h_pow_n_modp2 = self.h_pow_n % self.p_square
                self.h_pow_n_modq2 = self.h_pow_n % self.q_square
        else:
            self.djn_on = False

        self.n_square = pow(self.__n, 2)
        self.max_value_for_positive = self.__n // 3
        self.min_value_for_negative = self.__n - self.max_value_for_positive
        return self

    @classmethod
    def generate(cls, key_bit_size: int = 2048, djn_on: bool = False):
        """context.py:73-84"""
        p, q = cls._generate_paillier_private_key(key_bit_size, djn_on)
        if djn_on:
            n = p * q
            x = secrets.SystemRandom().getrandbits(n.bit_length())
            x |= 1 << (n.bit_length() - 1)
            h = -pow(x, 2)
            from . import _gmp
            n2 = n * n
            h_pow_n = _gmp.powmod(h % n2, n, n2) if _gmp.available() else pow(h, n, n2)
            return PaillierContext().init(p, q, djn_h_pow_n=h_pow_n)
        return PaillierContext().init(p, q)

    @property
    def p(self):
        return self.__p if self.__is_private else None

    @property
    def q(self):
        return self.__q if self.__is_private else None

    @property
    def n(self):
        return self.__n

    def is_private(self):
        return self.__is_private

    def _copy_public_from(self, other):
        """context.py:105-114"""
        self._dev = {}
        self.__n = other.n
        self.__is_private = False
        self.n_square = other.n_square
        self.max_value_for_positive = other.max_value_for_positive
        self.min_value_for_negative = other.min_value_for_negative
        self.djn_on = other.djn_on
        if self.djn_on:
            self.h_pow_n = other.h_pow_n
            self.djn_exp_bound = other.djn_exp_bound

    def to_public(self):
        if not self.__is_private:
            return self
        pub_context = PaillierContext()
        pub_context._copy_public_from(self)
        return pub_context

    @staticmethod
    def _generate_paillier_private_key(n_length: int = 2048, djn_on: bool = False, seed: Optional[int] = None):
        """context.py:123-150 (DJN keys need gcd(p-1, q-1) = 2)."""
        p, q = None, None
        if djn_on:
            def f(x, y):
                return (x == y) or (math.gcd(p - 1, q - 1) != 2)
        else:
            def f(x, y):
                return x == y
        while f(p, q):
            p = getprimeover(n_length // 2)
            q = getprimeover(n_length // 2)
        return p, q

    def serialize(self, save_private_key: bool = True):
        """context.py:152-157 — pickle of (p, q) or (n,)."""
        if save_private_key and self.__is_private:
            return pickle.dumps((self.__p, self.__q))
        return pickle.dumps((self.__n,))

    @classmethod
    def deserialize_from(cls, data: bytes):
        """context.py:159-168 (returns, does not raise, ValueError for bad input)."""
        from ..compat import loads  # accepts gmpy2 mpz pickles from reference peers
        unpickled_data = loads(data)
        if len(unpickled_data) == 1:
            return PaillierContext().init(n=int(unpickled_data[0]))
        elif len(unpickled_data) == 2:
            return PaillierContext().init(p=int(unpickled_data[0]), q=int(unpickled_data[1]))
        return ValueError("The unpickled data should be a tuple contains 1 or 2 big integers.")

    def __eq__(self, other):
        if id(self) == id(other):
            return True
        if self.p != other.p or self.q != other.q or self.n != other.n:
            return False
        return True

    def __hash__(self):
        if self.__is_private:
            return hash((self.__p, self.__q))
        return hash(self.__n)

    def __str__(self):
        if self.__is_private:
            return f"PaillierContext: p = {int(self.__p)}, q = {int(self.__q)}, n = {int(self.__n)}"
        return f"PaillierContext: n = {int(self.__n)}"

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_dev"] = {}
        return st

    def _l_function(self, x, p):
        return (x - 1) // p

    def _h_function(self, x, xsquare):
        return invert(self._l_function(pow(self.__n + 1, x - 1, xsquare), x), x)

    # ------------------------------------------------------------ device
    # Fixed-base table window (DJN private keys, include/xhe.h xhe_key_create):
    # a wider window means fewer products per encryption but exponentially
    # larger tables (2048-bit key: win 16 = 2 x 1.28 GB, 45 -> 64 products per
    # prime; win 20 = 2 x 16.6 GB, 52; win 22 = 2 x 59.9 GB, 47). The tables
    # are rebuilt per key (keys are regenerated per fit(), label_trainer.py:137),
    # so the window follows the volume a key has encrypted: 16 first, 20 after
    # WIN_STEPS[0] elements, 22 after WIN_STEPS[1] - each step only when the
    # new tables leave WIN_MARGIN bytes of the device free. $XHE_WIN_BITS or
    # set_device_window() pin a window instead.
    WIN_STEPS = ((0, 16), (8_000_000, 20), (64_000_000, 22))
    WIN_MARGIN = 32 << 30

    def set_device_window(self, win_bits):
        """Pin the fixed-base window: an int w, or '23s' / (23 | XHE_WIN_SPLIT)
        for the split layout (None: back to the volume policy). Cached device
        keys are rebuilt on next use."""
        from .._native import parse_win
        self._win_pinned = None if win_bits is None else parse_win(win_bits)
        self._dev = {}

    def _wanted_window(self):
        """(window bits w, split layout) this context's tables should have."""
        from .._native import XHE_WIN_SPLIT, parse_win
        pinned = getattr(self, "_win_pinned", None) or parse_win(os.environ.get("XHE_WIN_BITS", "0") or 0)
        if pinned:
            return pinned & 0xFF, bool(pinned & XHE_WIN_SPLIT)
        vol = getattr(self, "_volume", 0)
        return max(w for thr, w in self.WIN_STEPS if vol >= thr), False

    @staticmethod
    def _key_fits(k, want):
        """a built key serves a wanted (w, split) when its window is at least w
        and its layout is the one asked for"""
        return k.win_bits >= want[0] and getattr(k, "win_split", False) == want[1]

    def note_encrypt_volume(self, count: int):
        """Called by the batched encryptions: the policy's element counter."""
        self._volume = getattr(self, "_volume", 0) + int(count)

    def device_key(self, device=None):
        """Device-resident key for this context on `device` (default: the
        process's own GPU, own_device(); built once, cached; rebuilt with
        wider tables when the window policy asks for them)."""
        if device is None:
            device = self.own_device()
        dev = getattr(self, "_dev", None)
        if dev is None:
            dev = self._dev = {}
        k = dev.get(device)
        fixed_base = self.__is_private and self.djn_on
        if k is not None and (not fixed_base or self._key_fits(k, self._wanted_window())):
            return k
        with _KEY_LOCK:
            k = dev.get(device)
            want = self._wanted_window() if fixed_base else (0, False)
            if k is not None and (not fixed_base or self._key_fits(k, want)):
                return k
            from .._native import XHE_WIN_SPLIT, DeviceKey, device_free_bytes, table_bytes
            bits = device_key_bits(self.__n)
            h = self.h_pow_n if self.djn_on else None
            win, split = want
            flag = XHE_WIN_SPLIT if split else 0
            if fixed_base:
                have = table_bytes(bits, k.win_bits | (XHE_WIN_SPLIT if k.win_split else 0)) if k is not None else 0
                free = device_free_bytes(device)
                while win > 16 and free is not None and table_bytes(bits, win | flag) + self.WIN_MARGIN > free + have:
                    win -= 2
                if k is not None and self._key_fits(k, (win, split)):
                    return k
                dev.pop(device, None)
                k = None  # free the old tables before building the new ones
            if self.__is_private:
                k = DeviceKey(bits, self.__n, self.__p, self.__q, h, device=device, win_bits=win | flag if win else 0)
            else:
                k = DeviceKey(bits, self.__n, None, None, h, device=device)
            dev[device] = k
        return k

    @staticmethod
    def own_device():
        """The GPU this process works on: $LOCAL_RANK (one rank per GPU, as
        torch.distributed launches it) modulo the visible GPUs, else 0."""
        from .._native import visible_devices
        lr = os.environ.get("LOCAL_RANK", "").strip()
        return int(lr) % visible_devices() if lr.isdigit() else 0

    @staticmethod
    def shard_devices(num_cores: int = -1):
        """GPUs a batch is spread over (the reference spreads it over
        get_core_num(num_cores) processes, paillier.py:321-332,388-394):
        $XHE_DEVICES (comma-separated ids, may repeat; "all") if set; else
        num_cores = k > 1 -> k GPUs starting at the process's own; else
        (the default -1, or 1) the process's own GPU only. Fanning a default
        call out over every GPU would give every rank of a multi-process job
        a key - and, for a private DJN key, its fixed-base tables - on every
        GPU of the node."""
        spec = os.environ.get("XHE_DEVICES", "").strip()
        if spec and spec != "all":
            return [int(d) for d in spec.split(",") if d.strip()]
        from .._native import visible_devices
        n = visible_devices()
        if spec == "all":
            return list(range(n))
        own = PaillierContext.own_device()
        k = 1 if num_cores is None or num_cores < 1 else min(int(num_cores), n)
        return [(own + i) % n for i in range(k)]
