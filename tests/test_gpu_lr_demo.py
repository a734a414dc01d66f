"""BASELINE config 1: the vertical-LR 2-party HE round (label_trainer.py:193-259,
trainer.py:127-178) through the drop-in API on WDBC, every decrypted noised
gradient compared bit for bit with the plaintext-side restatement of the same
homomorphic operations (tools/lr_he_demo.py)."""
import pytest

from tests.conftest import FIXTURES, hx, load_fixture

pytestmark = pytest.mark.gpu


def test_lr_he_rounds_bit_exact():
    """One full epoch: 399 training rows = 6 batches of 64 and the 15-row
    last batch (its mat-vec, noise add and decrypt run other shapes)."""
    from tools.lr_he_demo import run
    from xfl_amd.paillier import PaillierContext
    k = load_fixture(FIXTURES[0])["key"]
    priv = PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=hx(k["h_pow_n"]))
    rec = run(epochs=1, check=True, key=priv, per_batch=True)
    assert rec["batches"] == 7 and rec["checked_bit_exact"] == 7
    assert [b["rows"] for b in rec["batch_ms"]] == [64] * 6 + [15]
