"""The cxx extension's Swizzle scheme (``heartbeat.Swizzle``), GPU-backed.

Mirrors the Python surface of cxx/Swizzle.hxx:475-508 (``Swizzle(check_fraction=
1.0, sectors=10, *, initialize=True)`` with encode / gen_challenge / prove /
verify / get_public / todict / fromdict) over the HIP kernels' cxx mode
(``HB_PRF_CXX``): the cxx prf (cxx/prf.hxx:97-176, CFB-128 over SHA256(LE32 i),
at most 81 tries) in encode (shacham_waters_private.cxx:638-702), prove
(:731-789, check_all and unsigned int block offsets) and verify (:791-842).
Tags differ from PySwizzle's for equal keys.

Parity unpinned: Crypto++ is absent here and no reference test pins cxx values
(SURVEY.md 8c); the GPU results are pinned to the oracle's OpenSSL restatement.
Not reproduced: the Crypto++ binary / base64 wire formats of Tag, State,
Challenge and Proof (this module's objects use PySwizzle's dict forms) and the
State's encrypt-and-sign layout (State here is PySwizzle's AES-CFB8 + HMAC
state, keyed by k_enc).
"""
import ctypes

import numpy as np

from . import _native, multi
from ._filebuf import FileBuffer
from .exc import HeartbeatError
from .PySwizzle.PySwizzle import Challenge, Proof, State, Tag, _kb, _random_bytes, getPrime
from .util import hb_decode, hb_encode

__all__ = ["Swizzle", "Tag", "State", "Challenge", "Proof"]

# shacham_waters_private.hxx:193 / Swizzle.hxx:494-508: the Python API fixes a
# 1024-bit prime (Crypto++ draws it below 2^1024; here exactly 1024 bits)
PRIME_BITS = 1024


class Swizzle(object):
    """Shacham-Waters private proof of storage with the cxx extension's prf."""

    def __init__(self, check_fraction=1.0, sectors=10, initialize=True, prime=None):
        self.check_fraction = float(check_fraction)
        self.sectors = int(sectors)
        self.public = False
        if initialize:
            self.k_enc = _random_bytes(32)
            self.k_mac = _random_bytes(32)
            self.prime = getPrime(PRIME_BITS) if prime is None else int(prime)
        else:
            self.k_enc = b"\0" * 32
            self.k_mac = b"\0" * 32
            self.prime = 0 if prime is None else int(prime)
        self.sectorsize = self.prime.bit_length() // 8   # _p.BitCount()/8 (:621)

    # -- serialisation (dict form; the Crypto++ binary format is not reproduced)
    def todict(self):
        return {"check_fraction": self.check_fraction, "sectors": self.sectors, "prime": self.prime,
                "public": self.public, "k_enc": hb_encode(self.k_enc), "k_mac": hb_encode(self.k_mac)}

    @staticmethod
    def fromdict(d):
        s = Swizzle(d["check_fraction"], d["sectors"], initialize=False, prime=d["prime"])
        s.public = bool(d.get("public", False))
        s.k_enc = hb_decode(d["k_enc"])
        s.k_mac = hb_decode(d["k_mac"])
        return s

    def __eq__(self, other):
        return isinstance(other, Swizzle) and self.todict() == other.todict()

    def __ne__(self, other):
        return not self == other

    def get_public(self):
        """A copy with the keys zeroed (shacham_waters_private.cxx:626-636)."""
        s = Swizzle(self.check_fraction, self.sectors, initialize=False, prime=self.prime)
        s.public = True
        return s

    def _check(self):
        if self.sectorsize < 1:
            raise HeartbeatError("prime must be at least 2^8 (sector size of at least one byte)")
        if self.sectors < 1:
            raise HeartbeatError("sectors must be positive")

    # -- scheme
    def encode(self, file):
        """Tags of every block of `file` from its position to EOF, and the
        encrypted State (shacham_waters_private.cxx:638-702)."""
        self._check()
        p = self.prime
        w = _native.width_of(p)
        C = self.sectorsize * self.sectors
        state = State(_random_bytes(32), _random_bytes(32))
        fb = FileBuffer(file)
        try:
            nblocks = fb.len // C + 1
            out = np.empty(nblocks * w, dtype=np.uint8)
            multi.encode_shards(p, self.sectors, state.f_key, state.alpha_key, fb.addr, fb.len, nblocks,
                                out.ctypes.data, _native.HB_PRF_CXX, multi.devices())
            fb.consume()
        finally:
            fb.close()
        state.chunks = nblocks
        state.encrypt(self.k_enc)
        return Tag._from_raw(out.tobytes(), w), state

    def gen_challenge(self, state):
        """l = (unsigned int)(check_fraction * n) indices, v limit p (:704-729)."""
        state = State.fromdict(state.todict())   # `state s = s_enc` (:706)
        try:
            state.decrypt(self.k_enc)
        except HeartbeatError:
            raise HeartbeatError("Signature check or decryption failed in generating challenge.  "
                                 "State of remote file cannot be verified.")
        l = int(self.check_fraction * int(state.chunks)) & 0xffffffff
        return Challenge(l, self.prime, _random_bytes(32))

    def prove(self, file, chal, tag):
        """mu_j, sigma over the challenged blocks (:731-789)."""
        self._check()
        p = self.prime
        S = self.sectors
        w = _native.width_of(p)
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
        False when the state does not decrypt or mu has the wrong length."""
        state = State.fromdict(state.todict())   # `state s = s_enc` (:796)
        try:
            state.decrypt(self.k_enc)
        except HeartbeatError:
            return False
        self._check()
        p = self.prime
        S = self.sectors
        w = _native.width_of(p)
        mu = list(proof.mu)
        if len(mu) != S:
            return False
        chunks = max(int(chal.chunks), 0)
        if chunks and int(state.chunks) <= 0:
            raise HeartbeatError("state has no chunks")
        mub = b"".join((int(m) % p).to_bytes(w, "big") for m in mu)
        vmax = _native.be(int(chal.v_max)) if chunks else b"\x01"
        rhs = ctypes.create_string_buffer(w)
        ctx = _native.context()
        pb = _native.be(p)
        fk, ak, ck = _kb(state.f_key), _kb(state.alpha_key), _kb(chal.key)
        with ctx.lock:
            ctx.check(_native.lib().hb_cxx_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, len(fk),
                                                      int(state.chunks), ck, len(ck), chunks, vmax,
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
