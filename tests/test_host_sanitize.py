"""CPU: the native host code under AddressSanitizer + UndefinedBehaviorSanitizer.

* wire.hpp's pickle parser reads bytes received from a remote party
  (Paillier.ciphertext_from, paillier.py:260-271). tests/native/host_fuzz.cpp
  decodes the reference's own wire bytes and CPython pickles of the same
  object graph at protocols 2-5, then every truncation, seeded random byte
  flips, opcode substitutions, inflated length/count fields and hand-made
  malformed inputs: each must decode or be rejected with an error, never
  touch memory out of bounds (the sanitizers abort the run otherwise).
* hostbn.hpp's key-setup arithmetic (context.py:28-71 constants) against
  Python ints on random and edge operands, under the same sanitizers.
"""
import os
import pickle
import random
import subprocess

import numpy as np
import pytest

from tests.conftest import FIXTURES, ROOT, hx, load_fixture

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("hostfuzz") / "host_fuzz")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", *SAN, os.path.join(HERE, "native", "host_fuzz.cpp"),
                    os.path.join(ROOT, "xfl_amd", "csrc", "wire_abi.cpp"), "-o", exe], check=True)
    return exe


def _env():
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must come first in the child
    return env


def _seeds(tmp_path):
    from xfl_amd import compat
    from xfl_amd.paillier.paillier import RawCiphertext
    compat._register_alias()
    paths = []
    for fx in FIXTURES:
        g = load_fixture(fx)
        p = tmp_path / f"ref_{fx}.bin"
        p.write_bytes(bytes.fromhex(g["ops"]["wire_a4"]))  # the reference's own bytes (gmpy2 values)
        paths.append(str(p))
    g = load_fixture(FIXTURES[0])
    raws = [hx(r) for r in g["ops"]["a"]["raw"][:5]]
    exps = g["ops"]["a"]["exp"][:5]
    arr = np.empty(5, dtype=object)
    for i, (r, e) in enumerate(zip(raws, exps)):
        arr[i] = RawCiphertext(r, e)
    for proto in (2, 3, 4, 5):
        p = tmp_path / f"cpython_p{proto}.bin"
        p.write_bytes(pickle.dumps(arr.reshape(5, 1), protocol=proto))
        paths.append(str(p))
    return paths


def test_wire_decoder_fuzz_under_sanitizers(harness, tmp_path):
    seeds = _seeds(tmp_path)
    r = subprocess.run([harness, "wire", *seeds], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith(f"seeds {len(seeds)} "), r.stdout
    rejected = int(r.stdout.split()[-1])
    assert rejected > 1000  # the mutants were exercised, not silently accepted


def test_zstd_raw_frames_under_sanitizers(harness):
    r = subprocess.run([harness, "zstd"], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    frames, refused = int(r.stdout.split()[2]), int(r.stdout.split()[4])
    assert frames == 10 and refused > 1000, r.stdout


def test_hostbn_under_sanitizers(harness):
    rng = random.Random(5)
    cases = []
    for fx in FIXTURES:
        k = load_fixture(fx)["key"]
        n, p = hx(k["n"]), hx(k["p"])
        n2 = n * n
        ebits = 16 if n.bit_length() <= 2048 else 4  # BigU powmod is bit-serial: keep the sanitized run short
        for _ in range(2):
            a, b = rng.randrange(n2), rng.randrange(n2)
            cases += [("add", a, b, 1), ("sub", max(a, b), min(a, b), 1), ("mul", a, b, 1), ("mod", a * b, 0, n2),
                      ("mulmod", a, b, n2), ("powmod", a, rng.randrange(1 << ebits), n2), ("modinv", a % p or 1, 0, p),
                      ("words_inv", a, 0, n2)]
        cases += [("mod", n2 - 1, 0, n2), ("mod", n2, 0, n2), ("mulmod", 0, n2 - 1, n2), ("sub", n2, n2, 1),
                  ("words_inv", p * 3, 0, n2), ("ninv", 28, 0, p), ("ninv", 27, 0, n2)]
    inp = "".join(f"{op} {a:x} {b:x} {m:x}\n" for op, a, b, m in cases)
    r = subprocess.run([harness, "bn"], input=inp, capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    out = r.stdout.split()
    assert len(out) == len(cases)
    for (op, a, b, m), got in zip(cases, out):
        if op == "add":
            want = a + b
        elif op == "sub":
            want = a - b
        elif op == "mul":
            want = a * b
        elif op == "mod":
            want = a % m
        elif op == "mulmod":
            want = a * b % m
        elif op == "powmod":
            want = pow(a, b, m)
        elif op == "modinv":
            want = pow(a, -1, m)
        elif op == "ninv":  # -m^-1 mod 2^W
            w = a
            want = (-pow(m, -1, 1 << w)) % (1 << w)
        else:  # words_inv
            try:
                want = pow(a, -1, m)
            except ValueError:
                assert got == "none"
                continue
        assert int(got, 16) == want, (op, got)
