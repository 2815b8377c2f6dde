"""heartbeat_amd.Swizzle, the cxx extension's scheme object (cxx/Swizzle.hxx,
cxx/shacham_waters_private.cxx:638-842), through the GPU cxx mode.  Flows
follow the reference's tests/tests_unit_swpriv.py (round trips, public copies,
tampered files, serialisation); values are checked against the oracle's cxx
restatement.  Parity unpinned (Crypto++ absent).
"""
import hashlib
import io

import pytest

from test_gpu_cxx import P1024, _cxx_prove_want

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sw():
    from heartbeat_amd import Swizzle as m
    return m


DATA = b"".join(hashlib.sha256(b"swz%d" % i).digest() for i in range(400)) + b"tail!"


@pytest.mark.parametrize("frac", [1.0, 0.3])
def test_round_trip(sw, oracle, frac):
    beat = sw.Swizzle(frac, 10, prime=P1024)
    tag, state = beat.encode(io.BytesIO(DATA))
    assert len(tag) == len(DATA) // (10 * 128) + 1
    # tags are the cxx encode of the state's keys
    st = sw.State.fromdict(state.todict())
    st.decrypt(beat.k_enc, beat.k_mac)
    assert tag.sigma == oracle.cxx_encode(P1024, 10, st.f_key, st.alpha_key, DATA)
    chal = beat.gen_challenge(state)
    assert chal.chunks == int(frac * len(tag))
    proof = beat.get_public().prove(io.BytesIO(DATA), chal, tag)
    want = _cxx_prove_want(oracle, P1024, 10, chal.key, chal.chunks, P1024, len(tag),
                           lambda k: tag.sigma[k], lambda off, n: DATA[off:off + n])
    assert (proof.mu, proof.sigma) == want
    assert beat.verify(proof, chal, state)
    # state untouched by gen_challenge / verify (the reference copies it)
    assert state.encrypted


def test_tampered_file_fails(sw):
    beat = sw.Swizzle(1.0, 10, prime=P1024)
    tag, state = beat.encode(io.BytesIO(DATA))
    chal = beat.gen_challenge(state)
    bad = bytearray(DATA)
    bad[1000] ^= 1
    proof = beat.prove(io.BytesIO(bytes(bad)), chal, tag)
    assert not beat.verify(proof, chal, state)


def test_wrong_key_and_mu_length(sw):
    beat = sw.Swizzle(1.0, 10, prime=P1024)
    tag, state = beat.encode(io.BytesIO(DATA))
    chal = beat.gen_challenge(state)
    proof = beat.prove(io.BytesIO(DATA), chal, tag)
    other = sw.Swizzle(1.0, 10, prime=P1024)
    assert not other.verify(proof, chal, state)          # state does not decrypt
    proof.mu = proof.mu[:-1]
    assert not beat.verify(proof, chal, state)           # p.mu().size() != _sectors


def test_serialisation(sw):
    beat = sw.Swizzle(0.5, 7, prime=P1024)
    assert sw.Swizzle.fromdict(beat.todict()) == beat
    pub = beat.get_public()
    assert pub.public and pub.k_enc == b"\0" * 32 and pub != beat


def test_size_bound_and_wire_round_trip(sw):
    """tests_unit_swpriv.py:189-204: the binary tag is at most
    0.104 * |file| + 4 bytes (1024-bit prime, 10 sectors); every object
    survives pickle / todict round trips after a real encode/prove."""
    import pickle
    beat = sw.Swizzle(1.0, 10, prime=P1024)
    data = DATA * 40
    tag, state = beat.encode(io.BytesIO(data))
    assert len(tag.__getstate__()) <= len(data) * 0.104 + 4
    chal = beat.gen_challenge(state)
    proof = beat.prove(io.BytesIO(data), chal, tag)
    for obj in (beat, tag, state, chal, proof):
        assert pickle.loads(pickle.dumps(obj)) == obj
        assert type(obj).fromdict(obj.todict()) == obj
    # the client / server exchange through the wire forms
    tag2 = sw.Tag.fromdict(tag.todict())
    chal2 = sw.Challenge.fromdict(chal.todict())
    proof2 = beat.get_public().prove(io.BytesIO(data), chal2, tag2)
    assert proof2 == proof
    assert beat.verify(sw.Proof.fromdict(proof2.todict()), chal, sw.State.fromdict(state.todict()))
    assert beat.verify(proof, chal, "not a state") is None


def test_heartbeat_alias_is_swizzle():
    import heartbeat_amd
    from heartbeat_amd import Swizzle as m
    assert heartbeat_amd.Heartbeat is m.Swizzle
