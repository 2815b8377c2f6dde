"""PyCrypto-compatible subset of ``Crypto.Util.number``."""


def size(N):
    """Bit length of N (PyCrypto: ``size(0) == 0``)."""
    return int(N).bit_length()


def bytes_to_long(s):
    return int.from_bytes(bytes(s), "big")


def long_to_bytes(n, blocksize=0):
    n = int(n)
    b = n.to_bytes(max(1, (n.bit_length() + 7) // 8), "big") if n else b"\0"
    if blocksize and len(b) % blocksize:
        b = b"\0" * (blocksize - len(b) % blocksize) + b
    return b


def getPrime(N, randfunc=None):
    import random
    import sympy
    r = random.Random(N)
    while True:
        x = r.getrandbits(N) | (1 << (N - 1)) | 1
        if sympy.isprime(x):
            return x
