"""xfl_amd — MI355X-native Paillier hot path for XFL."""
__version__ = "0.1.0"
