# Fixture-generation stand-in for the `zstd` module (not installed in the
# generator's interpreter). Identity "compression": it only changes the
# compression=True byte framing, never the arithmetic being recorded.
def compress(b):
    return b


def decompress(b):
    return b
