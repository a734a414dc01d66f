"""The opt-in whole-wave digit kernels (k_djn_wavedig, k_dec_wavedig;
$XHE_WAVEDIG=1, read once per process): the golden encrypt/decrypt parity
tests and the arbitrary-residue decrypt rerun in a child process with them
switched on."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_wavedig_kernels_bit_exact():
    env = dict(os.environ, XHE_WAVEDIG="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "tests/test_gpu_parity.py::test_encrypt_bit_exact",
                        "tests/test_gpu_parity.py::test_decrypt_bit_exact",
                        "tests/test_gpu_parity.py::test_decrypt_arbitrary_residues",
                        "tests/test_gpu_parity.py::test_decrypt_shapes_bit_exact",
                        "-k", "2048 or arbitrary"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
