"""PyCrypto-compatible ``Crypto.Hash.SHA256`` (hashlib)."""
import hashlib

digest_size = 32
block_size = 64


class _H(object):
    digest_size = 32
    block_size = 64

    def __init__(self, data=None):
        self._h = hashlib.sha256()
        if data is not None:
            self.update(data)

    def update(self, data):
        self._h.update(data)

    def digest(self):
        return self._h.digest()

    def hexdigest(self):
        return self._h.hexdigest()

    def copy(self):
        c = _H()
        c._h = self._h.copy()
        return c

    def new(self, data=None):
        return _H(data)


def new(data=None):
    return _H(data)
