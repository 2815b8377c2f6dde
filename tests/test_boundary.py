"""CPU-side checks of the drop-in boundary: the C-ABI library loads and
exports every symbol include/hbswizzle.h declares; host-side API logic
(State encryption/HMAC, todict/fromdict, KeyedPRF.pad, error behaviour)
matches the reference (tests/tests_unit_pyswpriv.py:43-87 in the reference);
without a GPU the compute entry points fail loudly."""
import io
import json
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "hbswizzle.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hb_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from heartbeat_amd import _native
    L = _native.lib()
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
    bound = {n for n, _, _ in _native.SIGNATURES}
    assert set(syms) == bound
    assert L.hb_abi_version() == 1


def test_width_and_block_count():
    from heartbeat_amd import _native
    L = _native.lib()
    p = (1 << 256) - 189
    pb = p.to_bytes(32, "big")
    assert L.hb_width(pb, 32) == 32
    assert L.hb_block_count(pb, 32, 16, 0) == 1
    assert L.hb_block_count(pb, 32, 16, 511) == 1
    assert L.hb_block_count(pb, 32, 16, 512) == 2
    p255 = int(json.load(open(os.path.join(ROOT, "tests/golden/primes.json")))["p255"], 16)
    assert L.hb_width(p255.to_bytes(32, "big"), 32) == 32


def test_keyedprf_pad():
    from heartbeat_amd.PySwizzle import KeyedPRF
    d = b"test data 0"
    assert KeyedPRF.pad(d, 15) == d + b"\0\0\0\0"
    assert KeyedPRF.pad(d, 7) == d[0:7]


def test_state_encryption_matches_reference(golden_encode, monkeypatch):
    """State.encrypt with the reference's IV reproduces its encrypted state
    and HMAC byte for byte (PySwizzle.py:149-195)."""
    import importlib
    mod = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    from heartbeat_amd.PySwizzle import State
    for c in golden_encode["cases"][:20]:
        iv = bytes.fromhex(c["state_iv"])
        monkeypatch.setattr(mod, "_random_bytes", lambda n, iv=iv: iv if n == 16 else os.urandom(n))
        st = State(bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]), c["ntags"])
        st.encrypt(bytes.fromhex(c["state_key"]))
        assert st.todict() == c["state"]
        back = State.fromdict(json.loads(json.dumps(st.todict())))
        back.decrypt(bytes.fromhex(c["state_key"]))
        assert back.f_key == bytes.fromhex(c["f_key"])
        assert back.alpha_key == bytes.fromhex(c["alpha_key"])


def test_state_tamper_detected():
    from heartbeat_amd import HeartbeatError
    from heartbeat_amd.PySwizzle import State
    state = State(os.urandom(32), os.urandom(32), 100)
    k = os.urandom(32)
    state.encrypt(k)
    state.encrypt(k)
    state.chunks = 10
    with pytest.raises(HeartbeatError) as ex:
        state.decrypt(k)
    assert ex.value.message == "Signature invalid on state."
    k = os.urandom(32)
    state = State(os.urandom(32), os.urandom(32), 100, False, None, None, k)
    assert state.hmac == state.get_hmac(k)


def test_short_key_state():
    from heartbeat_amd.PySwizzle import PySwizzle, State
    beat = PySwizzle(10, b"test pass phrase", prime=(1 << 256) - 189)
    assert beat.key == b"test pass phrase"
    s = State(b"f" * 32, b"a" * 32, 3)
    s.encrypt(beat.key)
    s.decrypt(beat.key)
    assert s.f_key == b"f" * 32


def test_todict_roundtrips():
    from heartbeat_amd.PySwizzle import Challenge, Proof, PySwizzle, Tag
    beat = PySwizzle(16, b"k" * 32, prime=(1 << 256) - 189)
    b2 = PySwizzle.fromdict(json.loads(json.dumps(beat.todict())))
    assert (b2.key, b2.prime, b2.sectors, b2.sectorsize) == (beat.key, beat.prime, 16, 32)
    ch = Challenge(7, 12345, b"c" * 32)
    assert Challenge.fromdict(json.loads(json.dumps(ch.todict()))).todict() == ch.todict()
    t = Tag()
    t.sigma = [1, 2, 3]
    assert Tag.fromdict(json.loads(json.dumps(t.todict()))).sigma == [1, 2, 3]
    raw = Tag._from_raw(bytes([0, 1, 0, 2]), 2)
    assert raw.sigma == [1, 2] and len(raw) == 2
    pr = Proof()
    pr.mu, pr.sigma = [4, 5], 6
    assert Proof.fromdict(pr.todict()).todict() == pr.todict()
    assert PySwizzle.tag_type() is Tag and PySwizzle.proof_type() is Proof


def test_get_prime():
    import importlib
    m = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    _is_probable_prime, getPrime = m._is_probable_prime, m.getPrime
    p = getPrime(128)
    assert p.bit_length() == 128 and _is_probable_prime(p)
    assert not _is_probable_prime((1 << 61) + 1)
    assert _is_probable_prime((1 << 61) - 1)


def test_no_gpu_fails_loudly():
    """Without a GPU the hot path raises; it never computes on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from heartbeat_amd import HeartbeatError
    from heartbeat_amd.PySwizzle import KeyedPRF, PySwizzle
    with pytest.raises(HeartbeatError):
        KeyedPRF(b"k" * 32, 1000).eval(1)
    beat = PySwizzle(4, b"k" * 32, prime=(1 << 256) - 189)
    with pytest.raises(HeartbeatError):
        beat.encode(io.BytesIO(b"hello"))
    from heartbeat_amd.Swizzle import Swizzle
    sw = Swizzle(1.0, 4, prime=(1 << 256) - 189)
    with pytest.raises(HeartbeatError):
        sw.encode(io.BytesIO(b"hello"))


def test_pyswizzle_tag_image_pickles_and_compares():
    """encode returns the tag image as a memoryview over its output array
    (no copy); the Tag still pickles, deep-copies and converts like the
    reference's list-of-ints Tag (PySwizzle.py:67-91)."""
    import copy
    import pickle

    import numpy as np

    from heartbeat_amd.PySwizzle.PySwizzle import Tag
    arr = np.frombuffer(bytes(range(96)), dtype=np.uint8).copy()
    t = Tag._from_raw(memoryview(arr), 32)
    want = [int.from_bytes(bytes(range(k, k + 32)), "big") for k in (0, 32, 64)]
    assert t.raw(2 ** 255 + 95) == bytes(range(96))
    assert pickle.loads(pickle.dumps(t)).sigma == want
    assert copy.deepcopy(t).sigma == want
    assert len(t) == 3 and t.todict() == {"sigma": want}


def test_product_build_is_not_an_experiment_build():
    """The wrong-tag instruction-count switches (HB_EXP_*, hb_lane.hpp) cannot
    reach libhbswizzle.so: the in-tree library reports a product build, the
    headers refuse the switches without HB_EXPERIMENT_BUILD, and the product
    Makefile refuses HB_EXP flags for libhbswizzle.so."""
    import subprocess
    from heartbeat_amd import _native
    assert _native.lib().hb_build_flags() & _native.HB_BUILD_EXPERIMENT == 0
    csrc = os.path.join(ROOT, "heartbeat_amd", "csrc")
    src = '#include "hb_lane.hpp"\nint main() { return 0; }\n'
    for flag in ("-DHB_EXP_NO_MAC", "-DHB_EXP_NO_SHA", "-DHB_EXP_MAC_NOLOAD", "-DHB_EXP_MFMA_NOLOAD"):
        r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-x", "c++", "-I", csrc, flag, "-"],
                           input=src.encode(), capture_output=True)
        assert r.returncode != 0 and b"experiment builds only" in r.stderr, flag
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-x", "c++", "-I", csrc, "-DHB_EXP_NO_MAC",
                        "-DHB_EXPERIMENT_BUILD", "-"], input=src.encode(), capture_output=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(["make", "-n", "-C", csrc, "EXTRA=-DHB_EXP_NO_MAC -DHB_EXPERIMENT_BUILD"],
                       capture_output=True)
    assert r.returncode != 0 and b"not libhbswizzle.so" in r.stderr
