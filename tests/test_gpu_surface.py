"""GPU tests of the drop-in under the reference's names, and of two launch
boundaries of the small-input encode and the fused prove.

* The reference tests' flows (tests_unit_heartbeat.py:34-58,
  tests_unit_pyswpriv.py:94-106) through ``import heartbeat`` /
  ``from heartbeat import PySwizzle`` -- encode, prove, verify on the GPU --
  and a native error caught as ``heartbeat.exc.HeartbeatError``.
* The one-launch F + alpha quad kernel (hb_prf_pair_kernel) at the edge of
  its wave positions: ceil(nb/16) + ceil(S/16) can exceed the grid's 16 G
  positions by one; alpha then runs in its own launch (hb_runtime.cpp).
* A fused prove right after a fused verify on the same context, whose
  polled token word held the verify's mu (hb_runtime.cpp, finish_sums).
"""
import hashlib
import importlib
import io
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)


def _num_cus():
    from heartbeat_amd import _native
    return _native.context().num_cus()


def _prime(bits, seed):
    import random
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(seed)
    while True:
        p = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(p):
            return p


def test_reference_usage_through_heartbeat_names():
    """tests_unit_heartbeat.py:34-58 (Heartbeat = the cxx Swizzle) and
    tests_unit_pyswpriv.py:94-106, verbatim imports, on the GPU."""
    import heartbeat
    from heartbeat import Heartbeat, PySwizzle
    from heartbeat.exc import HeartbeatError

    beat = Heartbeat()
    assert isinstance(beat, heartbeat.Swizzle.Swizzle)
    public_beat = beat.get_public()
    with open(os.path.join(GOLDEN, "files", "test.txt"), "rb") as fh:
        (tag, state) = beat.encode(fh)
    challenge = beat.gen_challenge(state)
    with open(os.path.join(GOLDEN, "files", "test.txt"), "rb") as fh:
        proof = public_beat.prove(fh, challenge, tag)
    assert beat.verify(proof, challenge, state)

    memfile = io.BytesIO(os.urandom(10))
    beat = PySwizzle.PySwizzle(10)
    (tag, state) = beat.encode(memfile)
    chal = beat.gen_challenge(state)
    memfile.seek(0)
    proof = beat.prove(memfile, chal, tag)
    assert beat.verify(proof, chal, state)
    assert type(tag).__module__ == "heartbeat.PySwizzle.PySwizzle"

    # an error raised by the native library surfaces as the reference's class
    with pytest.raises(HeartbeatError, match="AES key must be either 16, 24, or 32 bytes long"):
        PySwizzle.KeyedPRF(b"k" * 17, 1000).eval(3)
    with pytest.raises(heartbeat.exc.HeartbeatError):
        PySwizzle.PySwizzle(2, b"k", 1 << 4099 | 1).encode(io.BytesIO(b"x" * 100))


@pytest.mark.parametrize("S,short", [(1, 1), (10, 10), (3, 3), (16, 0)])
def test_small_encode_alpha_at_the_position_limit(oracle, S, short):
    """nb = 256 #CUs - short blocks with S sectors: nb + S <= 256 #CUs picks the
    placed one-launch path; ceil(nb/16) + ceil(S/16) is 16 #CUs + 1 for the
    first three cases.  A previous encode with another alpha key leaves its
    alpha_j R mod p in the context's buffer, so a skipped alpha would show as
    wrong tags.  Reference: PySwizzle.py:279-314."""
    from heartbeat_amd import _native as nat
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    nb = 256 * _num_cus() - short
    p = P256
    C = 32 * S
    nbytes = (nb - 1) * C + 5
    data = np.random.default_rng(S).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"pos-f").digest(), hashlib.sha256(b"pos-a").digest()
    pys.encode_file(p, S, fk, hashlib.sha256(b"other alpha").digest(), io.BytesIO(data[:C * 40]))
    tag, n = pys.encode_file(p, S, fk, ak, io.BytesIO(data))
    assert n == nb
    w = nat.width_of(p)
    raw = bytes(tag.raw(p))
    got = [int.from_bytes(raw[i:i + w], "big") for i in range(0, len(raw), w)]
    assert got == oracle.encode(p, S, fk, ak, data, nthreads=8)


def test_fused_prove_after_fused_verify_small_top_limb(oracle):
    """A 249-bit prime (top limb < 2^25; 31-byte sectors, S = 16: C and the
    32-byte tags 16-byte aligned, so the uploaded small file is proved by
    the fused launch): prove, verify, prove ... on one context with the same
    S; every proof equals the oracle's and verifies.  The prove's polled
    token word (the verify's top limb of mu_{S-1} in the pinned results
    buffer) is cleared before its launch, so a stale value cannot pass for
    the token.  Reference: PySwizzle.py:333-395."""
    from heartbeat_amd.PySwizzle import Challenge, PySwizzle
    p = _prime(249, 249)
    S = 16
    data = np.random.default_rng(232).integers(0, 256, 200000, dtype=np.uint8).tobytes()
    beat = PySwizzle(S, b"k" * 32, p)
    tag, state = beat.encode(io.BytesIO(data))
    for r in range(12):
        key = hashlib.sha256(b"tok-%d" % r).digest()
        chal = Challenge(300 + r, p, key)
        proof = beat.prove(io.BytesIO(data), chal, tag)
        mu, sg = oracle.prove(p, S, key, 300 + r, p, tag.sigma, data)
        assert proof.mu == mu and proof.sigma == sg, r
        assert beat.verify(proof, chal, state), r
