"""The cxx extension's object surface without a GPU: construction, pickle,
__getstate__/__setstate__, todict/fromdict (base64 of the binary form),
equality by serialized bytes, State.encrypt/decrypt/keysize and the
exception messages -- the reference's tests/tests_unit_swpriv.py:43-187
(TestSubClasses, TestSwizzle.test_exceptions), minus the parts that encode a
file (tests/test_gpu_swizzle.py).  Wire bytes: parity unpinned (Crypto++
absent); the layout follows shacham_waters_private.cxx."""
import os
import pickle
import struct

import pytest

from heartbeat_amd.exc import HeartbeatError

P1024 = None


@pytest.fixture(scope="module")
def sw():
    from heartbeat_amd import Swizzle as m
    return m


@pytest.fixture(scope="module")
def beat1(sw):
    return sw.Swizzle()


def assign_and_compare_states(item1, item2):
    state1 = item1.__getstate__()
    item2.__setstate__(state1)
    assert state1 == item2.__getstate__()


def test_comparison(sw, beat1):
    beat2 = pickle.loads(pickle.dumps(beat1))
    beat3 = sw.Swizzle(prime=beat1.prime)
    assert beat1 == beat2
    assert beat1 != beat3
    assert beat1.get_public() == beat1.get_public()
    assert sw.Challenge() == sw.Challenge()
    assert sw.Tag() == sw.Tag()
    assert sw.Proof() == sw.Proof()
    s1, s2 = sw.State(), sw.State()
    key = os.urandom(s1.keysize())
    s1.encrypt(key, key, True)
    s2.encrypt(key, key, True)
    assert s1 == s2                       # convergent encryption: equal bytes
    s3 = sw.State()
    s3.encrypt(key, key)                  # random IV
    assert s1 != s3
    assert sw.Tag() != sw.Proof()
    with pytest.raises(NotImplementedError):
        sw.Tag() < sw.Tag()


def test_get_set_state(sw):
    assign_and_compare_states(sw.Challenge(), sw.Challenge())
    assign_and_compare_states(sw.Tag(), sw.Tag())
    assign_and_compare_states(sw.Proof(), sw.Proof())
    s1, s2 = sw.State(), sw.State()
    key = os.urandom(s1.keysize())
    s1.encrypt(key, key, True)
    st = s1.__getstate__()
    s2.__setstate__(st)
    s2.decrypt(key, key)
    s2.encrypt(key, key, True)
    assert s2.__getstate__() == st


def test_serialization(sw, beat1):
    d = beat1.todict()
    assert isinstance(d, str)
    assert sw.Swizzle.fromdict(d) == beat1
    with pytest.raises(HeartbeatError):
        sw.Swizzle.fromdict("invalid object")
    for T in (sw.Swizzle.challenge_type(), sw.Swizzle.tag_type(), sw.Swizzle.proof_type()):
        obj = T()
        assert T.fromdict(obj.todict()) == obj
        with pytest.raises(HeartbeatError):
            T.fromdict("invalid object")
    s1 = sw.State()
    key = os.urandom(s1.keysize())
    s1.encrypt(key, key, True)
    sw.Swizzle.state_type().fromdict(s1.todict())
    with pytest.raises(HeartbeatError):
        sw.Swizzle.state_type().fromdict("invalid object")


def test_exceptions(sw):
    """tests_unit_swpriv.py:155-187, the exact messages."""
    state = sw.State()
    with pytest.raises(HeartbeatError) as ex:
        state.__setstate__()
    assert ex.value.message == "__setstate__ only takes one argument: state"
    with pytest.raises(HeartbeatError) as ex:
        state.encrypt()
    assert ex.value.message == ("encrypt() takes at least two arguments: the encryption key and the mac key "
                                "and an optional argument a bool, whether to use convergent encryption")
    with pytest.raises(HeartbeatError) as ex:
        state.decrypt()
    assert ex.value.message == "decrypt() takes two arguments: the encryption key and the mac key."
    with pytest.raises(HeartbeatError) as ex:
        state.encrypt(None, None)
    assert ex.value.message == "Invalid encryption key."
    n = state.keysize()
    with pytest.raises(HeartbeatError) as ex:
        state.encrypt(os.urandom(n - 1), os.urandom(n - 1))
    assert ex.value.message == ("Encryption key must be %d bytes in length.  Use keysize() to retrieve the key "
                                "size." % n)
    with pytest.raises(HeartbeatError):
        sw.State().__getstate__()        # must be encrypted prior to serialization


def test_state_wire_layout_and_tamper(sw):
    """encrypt_and_sign's raw layout (shacham_waters_private.cxx:169-306) and
    the signature check of check_sig_and_decrypt (:308-438)."""
    s = sw.State()
    s.n = 12345
    s.f_key, s.alpha_key = os.urandom(32), os.urandom(32)
    ke, km = os.urandom(32), os.urandom(32)
    s.encrypt(ke, km, True)
    raw = s.__getstate__()
    (raw_sz,) = struct.unpack_from("<I", raw, 0)
    (sig_sz,) = struct.unpack_from("<I", raw, 4)
    n, iv_sz = struct.unpack_from("<II", raw, 8)
    assert (n, iv_sz) == (12345, 16) and raw[16:32] == b"\0" * 16
    (enc_sz,) = struct.unpack_from("<I", raw, 32)
    assert enc_sz == 4 + 32 + 4 + 32 and sig_sz == 4 + 4 + 16 + 4 + enc_sz
    assert raw_sz == 4 + sig_sz + 4 + 32
    t = sw.State.fromdict(s.todict())
    assert t.n == 12345 and t.f_key == b""       # public interpretation: n only
    t.decrypt(ke, km)
    assert (t.f_key, t.alpha_key) == (s.f_key, s.alpha_key)
    bad = bytearray(raw)
    bad[40] ^= 1
    u = sw.State()
    u.__setstate__(bytes(bad))
    u.decrypt(ke, km)                          # bad MAC: ignored, keys stay unknown
    assert u.f_key == b""
    beat = sw.Swizzle(initialize=False)
    beat.k_enc, beat.k_mac = ke, km
    with pytest.raises(HeartbeatError):
        beat.gen_challenge(u)


def test_proof_and_challenge_layout(sw):
    pr = sw.Proof()
    pr.mu = [0, 1, 256]
    pr.sigma = 2 ** 64
    b = pr.__getstate__()
    assert b == (struct.pack("<I", 3) + struct.pack("<I", 1) + b"\0" + struct.pack("<I", 1) + b"\1" +
                 struct.pack("<I", 2) + b"\1\0" + struct.pack("<I", 9) + b"\1" + b"\0" * 8)
    ch = sw.Challenge(7, 255, b"k" * 32)
    assert ch.__getstate__() == struct.pack("<II", 7, 32) + b"k" * 32 + struct.pack("<I", 1) + b"\xff"
    big = struct.pack("<II", 7, 33) + b"k" * 33 + struct.pack("<I", 1) + b"\xff"
    with pytest.raises(HeartbeatError) as ex:
        sw.Challenge().__setstate__(big)
    assert ex.value.message == "Invalid key size."
