"""Drop-in replacement for XFL's python/common/crypto/paillier package."""
from .context import PaillierContext  # noqa: F401
from .encoder import PaillierEncoder  # noqa: F401
from .paillier import Paillier, PaillierCiphertext, RawCiphertext  # noqa: F401
from .array import PaillierArray  # noqa: F401
