"""PyCrypto-compatible ``Crypto.Hash.HMAC`` (stdlib hmac over sha256)."""
import hashlib
import hmac as _hmac


class _HMAC(object):
    def __init__(self, key, msg=None, digestmod=None):
        self._m = _hmac.new(bytes(key), None, hashlib.sha256)
        if msg is not None:
            self._m.update(msg)

    def update(self, msg):
        self._m.update(msg)

    def digest(self):
        return self._m.digest()

    def hexdigest(self):
        return self._m.hexdigest()


def new(key, msg=None, digestmod=None):
    return _HMAC(key, msg, digestmod)
