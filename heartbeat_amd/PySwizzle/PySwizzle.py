"""Drop-in for heartbeat.PySwizzle (heartbeat/PySwizzle/PySwizzle.py) whose
encode / prove / verify run on an MI355X through libhbswizzle.so.

Same class names, constructor arguments, method signatures, defaults,
``todict`` schemas and error messages as the reference:

    Challenge(chunks, v_max, key)                 PySwizzle.py:33-64
    Tag()  .sigma                                 PySwizzle.py:67-91
    State(f_key, alpha_key, chunks=0, ...)        PySwizzle.py:94-195
    Proof() .mu .sigma                            PySwizzle.py:198-224
    PySwizzle(sectors=10, key=None, prime=None, primebits=1024)
        encode(file) -> (Tag, State)              PySwizzle.py:279-314
        gen_challenge(state) -> Challenge         PySwizzle.py:316-331
        prove(file, chal, tag) -> Proof           PySwizzle.py:333-370
        verify(proof, chal, state) -> bool        PySwizzle.py:372-395

Tags produced by encode keep their fixed-width big-endian image (``Tag.raw``)
so prove can hand them to the GPU without converting 2^27 Python ints; the
``sigma`` list is materialised on first access.
"""
import ctypes
import hashlib
import hmac as _hmac
import os

import numpy as np

from .. import _native, multi
from .._filebuf import FileBuffer
from ..exc import HeartbeatError
from ..util import KeyedPRF, hb_decode, hb_encode

__all__ = ["KeyedPRF", "Challenge", "Tag", "State", "Proof", "PySwizzle", "getPrime"]

AES_BLOCK = 16


def _random_bytes(n):
    return os.urandom(n)


# ---------------------------------------------------------------- primes
_SMALL_PRIMES = [q for q in range(3, 2000, 2) if all(q % d for d in range(3, int(q ** 0.5) + 1, 2))]


def _is_probable_prime(n, rounds=40):
    if n < 2:
        return False
    if n in (2, 3):
        return True
    if n % 2 == 0:
        return False
    for q in _SMALL_PRIMES:
        if n % q == 0:
            return n == q
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = 2 + int.from_bytes(os.urandom((n.bit_length() + 7) // 8 + 8), "big") % (n - 3)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def getPrime(bits):
    """A random prime of exactly `bits` bits (Crypto.Util.number.getPrime)."""
    if bits < 2:
        raise HeartbeatError("prime size must be at least 2 bits")
    while True:
        x = int.from_bytes(os.urandom((bits + 7) // 8), "big")
        x &= (1 << bits) - 1
        x |= (1 << (bits - 1)) | 1
        if _is_probable_prime(x):
            return x


# ---------------------------------------------------------------- data types
class Challenge(object):
    """A challenge: check `chunks` blocks drawn with `key`, coefficients < v_max."""

    def __init__(self, chunks, v_max, key):
        self.chunks = chunks
        self.v_max = v_max
        self.key = key

    def todict(self):
        return {"chunks": self.chunks, "v_max": self.v_max, "key": hb_encode(self.key)}

    @staticmethod
    def fromdict(dict):
        return Challenge(dict["chunks"], dict["v_max"], hb_decode(dict["key"]))


class Tag(object):
    """The file tag: one value sigma_i < p per block."""

    def __init__(self):
        self._sigma = list()
        self._raw = None      # fixed-width big-endian image from encode
        self._width = 0

    @classmethod
    def _from_raw(cls, raw, width):
        t = cls()
        t._sigma = None
        t._raw = raw
        t._width = width
        return t

    @property
    def sigma(self):
        if self._sigma is None:
            w, raw = self._width, bytes(self._raw)
            self._sigma = [int.from_bytes(raw[i:i + w], "big") for i in range(0, len(raw), w)]
        return self._sigma

    @sigma.setter
    def sigma(self, value):
        self._sigma = value
        self._raw = None
        self._width = 0

    def __len__(self):
        if self._sigma is None:
            return len(self._raw) // self._width
        return len(self._sigma)

    def raw(self, p):
        """Fixed-width big-endian image of the tag values (mod p when a value
        does not fit the width -- equal in every use, which is mod p)."""
        w = _native.width_of(p)
        if self._raw is not None and self._width == w and self._sigma is None:
            return self._raw
        top = 1 << (8 * w)
        return b"".join((s if 0 <= s < top else s % p).to_bytes(w, "big") for s in self.sigma)

    def __getstate__(self):
        # the encode image is a memoryview over the GPU output array: pickle bytes
        d = dict(self.__dict__)
        if d.get("_raw") is not None:
            d["_raw"] = bytes(d["_raw"])
        return d

    def todict(self):
        return {"sigma": self.sigma}

    @staticmethod
    def fromdict(dict):
        self = Tag()
        self.sigma = dict["sigma"]
        return self


class State(object):
    """PRF keys of the tagged file, encrypted and signed for storage on the
    server (PySwizzle.py:94-195)."""

    def __init__(self, f_key, alpha_key, chunks=0, encrypted=False, iv=None, hmac=None, key=None):
        self.f_key = f_key
        self.alpha_key = alpha_key
        self.chunks = chunks
        self.encrypted = encrypted
        self.iv = b"" if iv is None else iv
        if hmac is None and key is not None:
            self.hmac = self.get_hmac(key)
        else:
            self.hmac = hmac

    def todict(self):
        return {"f_key": hb_encode(self.f_key),
                "alpha_key": hb_encode(self.alpha_key),
                "chunks": self.chunks,
                "encrypted": self.encrypted,
                "iv": hb_encode(self.iv),
                "hmac": hb_encode(self.hmac)}

    @staticmethod
    def fromdict(dict):
        return State(hb_decode(dict["f_key"]), hb_decode(dict["alpha_key"]), dict["chunks"],
                     dict["encrypted"], hb_decode(dict["iv"]), hb_decode(dict["hmac"]))

    def get_hmac(self, key):
        """HMAC-SHA256 over iv | str(chunks) | f_key | alpha_key | str(encrypted)."""
        if isinstance(key, str):
            key = key.encode("latin-1")
        h = _hmac.new(bytes(key), None, hashlib.sha256)
        h.update(self.iv)
        h.update(str(self.chunks).encode())
        h.update(self.f_key)
        h.update(self.alpha_key)
        h.update(str(self.encrypted).encode())
        return h.digest()

    def encrypt(self, key):
        """AES-CFB8 encrypt both keys with a fresh IV, then sign."""
        if self.encrypted:
            return
        self.iv = _random_bytes(AES_BLOCK)
        nf = len(self.f_key)
        ct = _native.aes_cfb8(_kb(key), self.iv, bytes(self.f_key) + bytes(self.alpha_key), True)
        self.f_key, self.alpha_key = ct[:nf], ct[nf:]
        self.encrypted = True
        self.hmac = self.get_hmac(key)

    def decrypt(self, key):
        """Check the signature, then decrypt the keys."""
        if self.get_hmac(key) != self.hmac:
            raise HeartbeatError("Signature invalid on state.")
        if not self.encrypted:
            return
        nf = len(self.f_key)
        pt = _native.aes_cfb8(_kb(key), self.iv, bytes(self.f_key) + bytes(self.alpha_key), False)
        self.f_key, self.alpha_key = pt[:nf], pt[nf:]
        self.encrypted = False
        self.hmac = self.get_hmac(key)


def _kb(key):
    return key.encode("latin-1") if isinstance(key, str) else bytes(key)


class Proof(object):
    """Proof of storage: mu_j per sector and sigma."""

    def __init__(self):
        self.mu = list()
        self.sigma = None

    def todict(self):
        return {"mu": self.mu, "sigma": self.sigma}

    @staticmethod
    def fromdict(dict):
        self = Proof()
        self.mu = dict["mu"]
        self.sigma = dict["sigma"]
        return self


# ---------------------------------------------------------------- scheme
class PySwizzle(object):
    """Shacham-Waters private proof of storage, GPU-backed."""

    def __init__(self, sectors=10, key=None, prime=None, primebits=1024):
        self.key = _random_bytes(32) if key is None else key
        self.prime = getPrime(primebits) if prime is None else prime
        self.sectors = sectors
        self.sectorsize = self.prime.bit_length() // 8

    def todict(self):
        return {"key": hb_encode(self.key), "prime": self.prime, "sectors": self.sectors}

    @staticmethod
    def fromdict(dict):
        return PySwizzle(dict["sectors"], hb_decode(dict["key"]), dict["prime"])

    def get_public(self):
        """A copy without the private key (a fresh random key is drawn)."""
        return PySwizzle(self.sectors, None, self.prime)

    # -- helpers
    def _check(self):
        if self.sectorsize < 1:
            raise HeartbeatError("prime must be at least 2^8 (sector size of at least one byte)")
        if int(self.sectors) < 1:
            raise HeartbeatError("sectors must be positive")

    def encode(self, file):
        """Tag every block of `file` (from its current position to EOF)."""
        self._check()
        p = int(self.prime)
        state = State(_random_bytes(32), _random_bytes(32))
        tag, nblocks = encode_file(p, int(self.sectors), state.f_key, state.alpha_key, file)
        state.chunks = nblocks
        state.encrypt(self.key)
        return (tag, state)

    def gen_challenge(self, state):
        """Challenge every block once on average (chunks = #blocks, v_max = p)."""
        state.decrypt(self.key)
        return Challenge(state.chunks, self.prime, _random_bytes(32))

    def prove(self, file, chal, tag):
        """mu_j = sum v_i m_{idx_i,j} mod p, sigma = sum v_i tag[idx_i] mod p."""
        self._check()
        p = int(self.prime)
        S = int(self.sectors)
        w = _native.width_of(p)
        ntags = len(tag)
        chunks = int(chal.chunks)
        proof = Proof()
        if chunks <= 0:
            proof.mu = [0] * S
            proof.sigma = 0
            return proof
        if ntags == 0:
            raise HeartbeatError("tag is empty")
        tags_raw = tag.raw(p)
        key = _kb(chal.key)
        vmax = _native.be(int(chal.v_max))
        # absolute offsets from the start of the file, as the reference's
        # file.seek(pos) before every read (PySwizzle.py:353-355)
        fb = FileBuffer(file, from_start=True)
        try:
            tarr = np.frombuffer(tags_raw, dtype=np.uint8)
            proof.mu, proof.sigma = multi.prove_shards(p, S, key, chunks, vmax, tarr.ctypes.data, ntags,
                                                       fb.addr, fb.len, 0, multi.devices())
        finally:
            fb.restore()
            fb.close()
        return proof

    def verify(self, proof, chal, state):
        """True iff proof.sigma == sum v_i F(idx_i) + sum alpha_j mu_j mod p."""
        state.decrypt(self.key)
        self._check()
        p = int(self.prime)
        S = int(self.sectors)
        w = _native.width_of(p)
        chunks = int(chal.chunks)
        if chunks > 0 and int(state.chunks) <= 0:
            raise HeartbeatError("state has no chunks")
        mu = list(proof.mu)
        if len(mu) < S:
            raise HeartbeatError("proof has fewer than %d mu values" % S)
        mub = b"".join((int(m) % p).to_bytes(w, "big") for m in mu[:S])
        vmax = _native.be(int(chal.v_max)) if chunks > 0 else b"\x01"
        rhs = ctypes.create_string_buffer(w)
        ctx = multi.primary_context()
        pb = _native.be(p)
        fk, ak, ck = _kb(state.f_key), _kb(state.alpha_key), _kb(chal.key)
        with ctx.lock:
            ctx.check(_native.lib().hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, len(fk),
                                                  int(state.chunks), ck, len(ck), max(chunks, 0),
                                                  vmax, len(vmax), mub, rhs))
        return proof.sigma == int.from_bytes(rhs.raw, "big")

    @staticmethod
    def tag_type():
        return Tag

    @staticmethod
    def state_type():
        return State

    @staticmethod
    def challenge_type():
        return Challenge

    @staticmethod
    def proof_type():
        return Proof


# Host buffers whose bytes hb_encode page-locks read-only in windows
# (HB_HOST_REGISTER) instead of staging them through the runtime's pageable
# copies, by FileBuffer kind: all of them.  A 4 GiB real file through
# encode_file: 38.2 vs 31.1 GiB/s (registered vs pageable, best of 3), a
# BytesIO 47.7 vs 43.1, one box (profiles/r05/f/bench_c3_nocpu.log; the
# caller-pinned raw rate 48.9); the medians of 5 in a standalone probe 40.7 vs
# 30.4 for the file (profiles/r05/f/probe2.log).  bench.py's host_path
# measures both ways in every default run.
REGISTER_KINDS = ("mmap", "bytesio", "bytes", "read")
# hb_encode page-locks only host buffers of at least this many bytes (below
# it the windows cost more than they save, hb_runtime.cpp); a smaller mapped
# file is prefaulted instead (MAP_POPULATE), as without registration
HOST_REGISTER_MIN = 32 << 20


def encode_file(p, sectors, f_key, alpha_key, file, devices=None, register=None):
    """GPU encode of a file object / buffer: (Tag, number of blocks).  Files of
    at least 2 x multi.MIN_SHARD_BYTES are sharded by block range over
    `devices` (default: multi.devices(), every visible GPU).  `register`
    forces (True) or forbids (False) the windowed read-only page-locking of
    the host bytes (HB_HOST_REGISTER); None: REGISTER_KINDS decides."""
    w = _native.width_of(p)
    ss = p.bit_length() // 8
    C = ss * sectors
    fk, ak = _kb(f_key), _kb(alpha_key)
    if len(fk) != len(ak):
        raise HeartbeatError("f_key and alpha_key must have the same length")
    if register is False or (register is None and "mmap" not in REGISTER_KINDS):
        populate = True
    else:
        populate = HOST_REGISTER_MIN
    fb = FileBuffer(file, populate=populate)
    try:
        nblocks = fb.len // C + 1
        # the tags land in the array the Tag keeps: no zero fill, no copy of
        # the image (a bytes-like buffer to Tag)
        out = np.empty(nblocks * w, dtype=np.uint8)
        reg = fb.kind in REGISTER_KINDS if register is None else bool(register)
        multi.encode_shards(p, sectors, fk, ak, fb.addr, fb.len, nblocks, out.ctypes.data,
                            _native.HB_HOST_REGISTER if reg else 0, multi.devices(devices))
        fb.consume()
    finally:
        fb.close()
    return Tag._from_raw(memoryview(out), w), nblocks


# The reference's module path (heartbeat/PySwizzle/PySwizzle.py): pickles of
# these objects name heartbeat.PySwizzle.PySwizzle, which the repo's
# heartbeat/ package re-exports them from, so they load under either package.
for _c in (Challenge, Tag, State, Proof, PySwizzle):
    _c.__module__ = "heartbeat.PySwizzle.PySwizzle"
del _c
