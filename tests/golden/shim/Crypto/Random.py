"""Deterministic stand-in for ``Crypto.Random``.

The golden generator pushes the exact byte strings that the reference should
draw (f_key, alpha_key, state IV, challenge key, ...) with ``push``; ``read``
pops them in order and checks the requested length.  With an empty queue it
falls back to a seeded SHA-256 counter stream, so runs are reproducible.
"""
import hashlib

_queue = []
_ctr = [0]
_seed = [b"heartbeat-golden"]


def push(*items):
    _queue.extend(bytes(x) for x in items)


def reseed(seed):
    _seed[0] = bytes(seed)
    _ctr[0] = 0
    del _queue[:]


def _stream(n):
    out = b""
    while len(out) < n:
        out += hashlib.sha256(_seed[0] + _ctr[0].to_bytes(8, "big")).digest()
        _ctr[0] += 1
    return out[:n]


class _RNG(object):
    def read(self, n):
        if _queue:
            x = _queue.pop(0)
            assert len(x) == n, "queued %d bytes, reference asked for %d" % (len(x), n)
            return x
        return _stream(n)


def new(*a, **k):
    return _RNG()


def get_random_bytes(n):
    return _RNG().read(n)
