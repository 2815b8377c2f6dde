"""The cxx extension's Swizzle scheme (``heartbeat.Swizzle``), GPU-backed.

Mirrors the Python surface of the PyCXX module cxx/Swizzle.hxx:43-762 over the
HIP kernels' cxx mode (``HB_PRF_CXX``): the cxx prf (cxx/prf.hxx:97-176,
CFB-128 over SHA256(LE32 i), at most 81 tries) in encode
(shacham_waters_private.cxx:638-702), prove (:731-789, check_all and unsigned
int sector offsets) and verify (:791-842).  Tags differ from PySwizzle's for
equal keys.

Object surface (Swizzle.hxx:63-311): every type -- ``Swizzle``, ``Tag``,
``State``, ``Challenge``, ``Proof`` -- is constructible without arguments and
has ``__getstate__`` (its binary serialization), ``__setstate__(state)``,
``__reduce__`` (pickle), ``todict()`` (base64 TEXT of the binary form),
static ``fromdict(text)`` and equality by serialized bytes; the ordering
comparisons raise NotImplementedError.  ``State`` adds
``encrypt(k_enc, k_mac[, convergent])``, ``decrypt(k_enc, k_mac)`` and
``keysize()`` (Swizzle.hxx:335-432).  Errors are HeartbeatError with the
reference's messages.

Binary formats follow shacham_waters_private.cxx:38-594, 844-976: u32 fields
written as ``PutWord32(htonl(x))`` and integers as ``u32 MinEncodedSize`` +
big-endian bytes.  With Crypto++'s default big-endian PutWord32 the double swap
makes every u32 LITTLE-endian on x86; that byte order, and the
formats as a whole, are parity unpinned -- Crypto++ is absent here and no
reference test pins the bytes.  The State's raw form is
``[sig_len][n, iv_len, iv, enc_len, AES-256-CFB128(k_enc, iv,
[f_key_len, f_key, alpha_key_len, alpha_key])][mac_len][HMAC-SHA256(k_mac,
signed part)]`` (:169-306).
"""
import base64
import binascii
import ctypes
import hashlib
import hmac as _hmac
import struct

import numpy as np

from . import _native, multi
from ._filebuf import FileBuffer
from .exc import HeartbeatError
from .PySwizzle.PySwizzle import _kb, _random_bytes, getPrime

__all__ = ["Swizzle", "Tag", "State", "Challenge", "Proof"]

# shacham_waters_private.hxx:193 / Swizzle.hxx:494-508: the Python API fixes a
# 1024-bit prime (Crypto++ draws it below 2^1024; here exactly 1024 bits)
PRIME_BITS = 1024
KEY_SIZE = 32            # shacham_waters_private_data::key_size
MAX_RAW_SIZE = 2048      # state::max_raw_size
_FLAG_PUBLIC = 0x01


# ---------------------------------------------------------------- wire helpers
def _u32(x):
    return struct.pack("<I", int(x) & 0xffffffff)


def _min_encoded(x):
    """Crypto++ Integer::Encode(bt, MinEncodedSize()): unsigned big-endian,
    at least one byte, after its u32 length."""
    x = int(x)
    n = max(1, (x.bit_length() + 7) // 8)
    return _u32(n) + x.to_bytes(n, "big")


class _Reader(object):
    def __init__(self, data):
        self.b = bytes(data)
        self.i = 0

    def u32(self, err):
        if self.i + 4 > len(self.b):
            raise HeartbeatError(err)
        v = struct.unpack_from("<I", self.b, self.i)[0]
        self.i += 4
        return v

    def take(self, n, err):
        if self.i + n > len(self.b):
            raise HeartbeatError(err)
        v = self.b[self.i:self.i + n]
        self.i += n
        return v

    def integer(self, err):
        n = self.u32(err)
        # safe_integer (shacham_waters_private.hxx:58-75): the stream must hold n bytes
        return int.from_bytes(self.take(n, "Unable to decode integer."), "big")


class _Serializable(object):
    """PyBytesStateAccessiblePyClass (Swizzle.hxx:125-311)."""

    def _serialize(self):
        raise NotImplementedError

    def _deserialize(self, data):
        raise NotImplementedError

    def __getstate__(self):
        return self._serialize()

    def __setstate__(self, *args):
        if len(args) != 1:
            raise HeartbeatError("__setstate__ only takes one argument: state")
        try:
            self._deserialize(bytes(args[0]))
        except HeartbeatError:
            raise
        except Exception as e:   # noqa: BLE001 -- the reference maps std::exception
            raise HeartbeatError(str(e))

    def __reduce__(self):
        return (type(self), (), self.__getstate__())

    def todict(self):
        return base64.b64encode(self._serialize()).decode("utf-8")

    @classmethod
    def fromdict(cls, text):
        obj = cls()
        try:
            raw = base64.b64decode(text.encode("utf-8") if isinstance(text, str) else bytes(text))
        except (binascii.Error, ValueError, AttributeError, TypeError) as e:
            raise HeartbeatError(str(e))
        obj.__setstate__(raw)
        return obj

    def __eq__(self, other):
        if type(other) is not type(self):
            return False
        return self._serialize() == other._serialize()

    def __ne__(self, other):
        return not self == other

    __hash__ = None

    def __lt__(self, other):
        raise NotImplementedError("Less than operator is not implemented.")

    def __le__(self, other):
        raise NotImplementedError("Less than or equal to operator is not implemented.")

    def __gt__(self, other):
        raise NotImplementedError("Greater than operator is not implemented.")

    def __ge__(self, other):
        raise NotImplementedError("Greater than or equal to operator is not implemented.")


# ---------------------------------------------------------------- data types
class Tag(_Serializable):
    """File tag: one sigma per block (tag::serialize :38-54)."""

    def __init__(self):
        self._sigma = []
        self._raw = None
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

    def __len__(self):
        if self._sigma is None:
            return len(self._raw) // self._width
        return len(self._sigma)

    def raw(self, p):
        """Fixed-width big-endian image (the GPU prove's input)."""
        w = _native.width_of(p)
        if self._raw is not None and self._width == w and self._sigma is None:
            return self._raw
        top = 1 << (8 * w)
        return b"".join((s if 0 <= s < top else s % p).to_bytes(w, "big") for s in self.sigma)

    def _serialize(self):
        out = [_u32(len(self))]
        if self._sigma is None:
            w, raw = self._width, self._raw
            for i in range(0, len(raw), w):
                v = bytes(raw[i:i + w]).lstrip(b"\0") or b"\0"
                out.append(_u32(len(v)) + v)
        else:
            out.extend(_min_encoded(s) for s in self._sigma)
        return b"".join(out)

    def _deserialize(self, data):
        r = _Reader(data)
        n = r.u32("Unable to get sigma count.")
        sig = [r.integer("Unable to get sigma size.") for _ in range(n)]
        self._sigma, self._raw, self._width = sig, None, 0


class State(_Serializable):
    """Encrypted and signed file state: n (blocks), f_key, alpha_key
    (state, shacham_waters_private.cxx:80-458)."""

    def __init__(self):
        self.n = 0
        self.f_key = b""
        self.alpha_key = b""
        self._raw = None
        self.encrypted = False

    @property
    def chunks(self):
        return self.n

    def keysize(self):
        return KEY_SIZE

    @staticmethod
    def _key(k):
        try:
            k = _kb(k)
        except (TypeError, AttributeError, UnicodeEncodeError):
            raise HeartbeatError("Invalid encryption key.")
        if len(k) != KEY_SIZE:
            raise HeartbeatError("Encryption key must be %d bytes in length.  Use keysize() to retrieve "
                                 "the key size." % KEY_SIZE)
        return k

    def encrypt(self, *args):
        """encrypt(k_enc, k_mac[, convergent]) -- encrypt_and_sign (:169-306);
        convergent encryption uses a zero IV."""
        if len(args) < 2:
            raise HeartbeatError("encrypt() takes at least two arguments: the encryption key and the mac key "
                                 "and an optional argument a bool, whether to use convergent encryption")
        k_enc, k_mac = self._key(args[0]), self._key(args[1])
        convergent = len(args) > 2 and bool(args[2])
        iv = b"\0" * 16 if convergent else _random_bytes(16)
        plain = _u32(len(self.f_key)) + bytes(self.f_key) + _u32(len(self.alpha_key)) + bytes(self.alpha_key)
        enc = _native.aes_cfb128(k_enc, iv, plain, True)
        sig = _u32(self.n) + _u32(len(iv)) + iv + _u32(len(enc)) + enc
        mac = _hmac.new(k_mac, sig, hashlib.sha256).digest()
        self._raw = _u32(len(sig)) + sig + _u32(len(mac)) + mac
        self.encrypted = True

    def _check_sig_and_decrypt(self, k_enc, k_mac):
        """check_sig_and_decrypt (:308-438): False on a bad signature."""
        if not self.encrypted:
            raise HeartbeatError("in shacham_waters_private_data::state::check_sig_and_decrypt, data must be "
                                 "encrypted before decryption and checking signature.")
        r = _Reader(self._raw)
        sig = r.take(r.u32("Unable to get signed data size."), "Incorrect size transferred.")
        msz = r.u32("Unable to get mac size.")
        if msz != 32:
            return False
        mac = r.take(msz, "Incorrect size transferred.")
        if not _hmac.compare_digest(_hmac.new(k_mac, sig, hashlib.sha256).digest(), mac):
            return False
        s = _Reader(sig)
        self.n = s.u32("Unable to get n.")
        iv = s.take(s.u32("Unable to get iv size."), "Unable to get iv.")
        enc = s.take(s.u32("Unable to get encrypted size."), "Unable to get encrypted data.")
        plain = _native.aes_cfb128(k_enc, iv, enc, False)
        p = _Reader(plain)
        self.f_key = p.take(p.u32("Unable to get key size."), "Key corrupted.")
        self.alpha_key = p.take(p.u32("Unable to get key size."), "Key corrupted.")
        return True

    def decrypt(self, *args):
        """decrypt(k_enc, k_mac): restores the keys on success; a bad
        signature leaves the state as it is (Swizzle.hxx:383-406 ignores the
        result of check_sig_and_decrypt)."""
        if len(args) != 2:
            raise HeartbeatError("decrypt() takes two arguments: the encryption key and the mac key.")
        self._check_sig_and_decrypt(self._key(args[0]), self._key(args[1]))

    def _serialize(self):
        if not self.encrypted:
            raise HeartbeatError("in shacham_waters_private_data::serialize, state must be encrypted prior "
                                 "to serialization.")
        return _u32(len(self._raw)) + self._raw

    def _deserialize(self, data):
        r = _Reader(data)
        n = r.u32("Unable to get raw size of state.")
        if n > MAX_RAW_SIZE:
            raise HeartbeatError("Reported size of encrypted state is too large.")
        self._raw = r.take(n, "Raw data incorrect size.")
        self.encrypted = True
        # public_interpretation (:440-458): n is readable without the keys
        pr = _Reader(self._raw)
        pr.u32("Unable to get n.")
        self.n = pr.u32("Unable to get n.")
        self.f_key = b""
        self.alpha_key = b""

    def _copy(self):
        s = State()
        s.n, s.f_key, s.alpha_key = self.n, self.f_key, self.alpha_key
        s._raw, s.encrypted = self._raw, self.encrypted
        return s


class Challenge(_Serializable):
    """l (indices to check), key, v_max (challenge :460-525)."""

    def __init__(self, chunks=0, v_max=0, key=b""):
        self.chunks = chunks
        self.v_max = v_max
        self.key = key

    def _serialize(self):
        k = bytes(self.key)
        return _u32(self.chunks) + _u32(len(k)) + k + _min_encoded(self.v_max)

    def _deserialize(self, data):
        r = _Reader(data)
        self.chunks = r.u32("Unable to read l.")
        ks = r.u32("Unable to read key size.")
        if ks > KEY_SIZE:
            raise HeartbeatError("Invalid key size.")
        self.key = r.take(ks, "Key corrupted.")
        self.v_max = r.integer("Unable to read B size.")


class Proof(_Serializable):
    """mu_j and sigma (proof :527-594)."""

    def __init__(self):
        self.mu = []
        self.sigma = 0

    def _serialize(self):
        return _u32(len(self.mu)) + b"".join(_min_encoded(m) for m in self.mu) + _min_encoded(self.sigma)

    def _deserialize(self, data):
        r = _Reader(data)
        n = r.u32("Unable to retrieve proof mu count.")
        self.mu = [r.integer("Unable to retrieve integer size.") for _ in range(n)]
        self.sigma = r.integer("Unable to read sigma size.")


# ---------------------------------------------------------------- scheme
class Swizzle(_Serializable):
    """Shacham-Waters private proof of storage with the cxx extension's prf
    (shacham_waters_private.hxx:125-229; Python type Swizzle.hxx:475-735).
    Serialization keeps the reference's fields (flags, keys unless public,
    sectors, sector size, p; :844-976): check_fraction is not part of it, so a
    deserialized object has the constructor default 1.0, as in the reference."""

    def __init__(self, check_fraction=1.0, sectors=10, initialize=True, prime=None):
        self.check_fraction = float(check_fraction)
        self.sectors = int(sectors)
        self.public = False
        self.k_enc = b"\0" * KEY_SIZE
        self.k_mac = b"\0" * KEY_SIZE
        self.prime = 0 if prime is None else int(prime)
        if initialize:
            # init (:596-624): random keys, a random prime, sector size BitCount/8
            self.k_enc = _random_bytes(KEY_SIZE)
            self.k_mac = _random_bytes(KEY_SIZE)
            if prime is None:
                self.prime = getPrime(PRIME_BITS)
        self.sectorsize = self.prime.bit_length() // 8   # _p.BitCount()/8 (:621)

    # -- serialisation (:844-976)
    def __reduce__(self):
        # the reference reduces to (type, (), state): a default-constructed
        # object whose fields __setstate__ then replaces; constructing it
        # uninitialized skips drawing a prime that is thrown away
        return (Swizzle, (1.0, 10, False), self.__getstate__())

    @classmethod
    def fromdict(cls, text):
        obj = cls(initialize=False)
        try:
            raw = base64.b64decode(text.encode("utf-8") if isinstance(text, str) else bytes(text))
        except (binascii.Error, ValueError, AttributeError, TypeError) as e:
            raise HeartbeatError(str(e))
        obj.__setstate__(raw)
        return obj

    def _serialize(self):
        out = [bytes([_FLAG_PUBLIC if self.public else 0])]
        if not self.public:
            out += [_u32(KEY_SIZE), bytes(self.k_enc), _u32(KEY_SIZE), bytes(self.k_mac)]
        out += [_u32(self.sectors), _u32(self.sectorsize), _min_encoded(self.prime)]
        return b"".join(out)

    def _deserialize(self, data):
        r = _Reader(data)
        f = r.take(1, "Unable to retrieve heartbeat flags.")[0]
        self.public = bool(f & _FLAG_PUBLIC)
        if not self.public:
            for attr in ("k_enc", "k_mac"):
                if r.u32("Unable to retrieve key size.") != KEY_SIZE:
                    raise HeartbeatError("Incompatible key sizes.")
                setattr(self, attr, r.take(KEY_SIZE, "Key corrupted."))
        self.sectors = r.u32("Unable to read sector count.")
        self.sectorsize = r.u32("Unable to read sector size.")
        self.prime = r.integer("Unable to read p size.")

    def get_public(self):
        """A copy with the keys zeroed (get_public, :626-636)."""
        s = Swizzle(self.check_fraction, self.sectors, initialize=False, prime=self.prime)
        s.sectorsize = self.sectorsize
        s.public = True
        return s

    def _check(self):
        if self.sectorsize < 1:
            raise HeartbeatError("prime must be at least 2^8 (sector size of at least one byte)")
        if self.sectors < 1:
            raise HeartbeatError("sectors must be positive")

    # -- scheme
    def encode(self, file):
        """(Tag, State) of every block of `file` from its position to EOF
        (encode :638-702); the state is encrypted and signed."""
        self._check()
        p = self.prime
        w = _native.width_of(p)
        C = self.sectorsize * self.sectors
        state = State()
        state.f_key = _random_bytes(KEY_SIZE)
        state.alpha_key = _random_bytes(KEY_SIZE)
        fb = FileBuffer(file)
        try:
            nblocks = fb.len // C + 1
            out = np.empty(nblocks * w, dtype=np.uint8)
            multi.encode_shards(p, self.sectors, state.f_key, state.alpha_key, fb.addr, fb.len, nblocks,
                                out.ctypes.data, _native.HB_PRF_CXX, multi.devices())
            fb.consume()
        finally:
            fb.close()
        state.n = nblocks
        state.encrypt(self.k_enc, self.k_mac)
        return Tag._from_raw(memoryview(out), w), state

    def gen_challenge(self, state):
        """l = (unsigned int)(check_fraction * n) indices, v limit p (:704-729)."""
        s = state._copy()   # `state s = s_enc` (:706)
        if s.encrypted and not s._check_sig_and_decrypt(self.k_enc, self.k_mac):
            raise HeartbeatError("Signature check or decryption failed in generating challenge.  "
                                 "State of remote file cannot be verified.")
        l = int(self.check_fraction * int(s.n)) & 0xffffffff
        return Challenge(l, self.prime, _random_bytes(KEY_SIZE))

    def prove(self, file, chal, tag):
        """mu_j, sigma over the challenged blocks (:731-789)."""
        self._check()
        p = self.prime
        S = self.sectors
        ntags = len(tag)
        if ntags == 0:
            raise HeartbeatError("tag is empty")
        proof = Proof()
        chunks = int(chal.chunks)
        if chunks <= 0:
            proof.mu = [0] * S
            proof.sigma = 0
            return proof
        tarr = np.frombuffer(tag.raw(p), dtype=np.uint8)
        key = _kb(chal.key)
        vmax = _native.be(int(chal.v_max))
        # absolute offsets from the start of the file, as the reference's
        # f.seek(pos) before every read (shacham_waters_private.cxx:763-764)
        fb = FileBuffer(file, from_start=True)
        try:
            proof.mu, proof.sigma = multi.prove_shards(p, S, key, chunks, vmax, tarr.ctypes.data, ntags,
                                                       fb.addr, fb.len, _native.HB_PRF_CXX, multi.devices())
        finally:
            fb.restore()
            fb.close()
        return proof

    def verify(self, proof, chal, state):
        """sigma == sum v_i f(idx_i) + sum alpha(j) mu_j mod p (:791-842);
        False when the state does not authenticate or mu has the wrong length,
        None for arguments of the wrong types (Swizzle.hxx:704-707)."""
        if not (isinstance(proof, Proof) and isinstance(chal, Challenge) and isinstance(state, State)):
            return None
        s = state._copy()   # `state s = s_enc` (:796)
        if s.encrypted and not s._check_sig_and_decrypt(self.k_enc, self.k_mac):
            return False
        self._check()
        p = self.prime
        S = self.sectors
        w = _native.width_of(p)
        mu = list(proof.mu)
        if len(mu) != S:
            return False
        chunks = max(int(chal.chunks), 0)
        if chunks and int(s.n) <= 0:
            raise HeartbeatError("state has no chunks")
        mub = b"".join((int(m) % p).to_bytes(w, "big") for m in mu)
        vmax = _native.be(int(chal.v_max)) if chunks else b"\x01"
        rhs = ctypes.create_string_buffer(w)
        ctx = multi.primary_context()
        pb = _native.be(p)
        fk, ak, ck = _kb(s.f_key), _kb(s.alpha_key), _kb(chal.key)
        with ctx.lock:
            ctx.check(_native.lib().hb_cxx_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, len(fk),
                                                      int(s.n), ck, len(ck), chunks, vmax,
                                                      len(vmax), mub, rhs))
        return int(proof.sigma) == int.from_bytes(rhs.raw, "big")

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


# The extension module's path (cxx/Swizzle.hxx:738, imported as
# heartbeat.Swizzle): pickles name heartbeat.Swizzle.<type>, which the repo's
# heartbeat/ package re-exports.
for _c in (Swizzle, Tag, State, Challenge, Proof):
    _c.__module__ = "heartbeat.Swizzle"
del _c
