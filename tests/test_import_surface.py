"""The drop-in under the reference's own names, without a GPU: the import lines
of the reference's tests run unchanged against the repo's ``heartbeat``
package, every name is the GPU build's object, errors are one class, and
pickles name ``heartbeat.*`` paths (heartbeat/__init__.py:28-36,
heartbeat/PySwizzle/__init__.py:28)."""
import os
import pickle
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# The reference tests' import lines, verbatim:
#   tests/tests_unit_pyswpriv.py:38-39, tests/tests_unit_swpriv.py:38-39,
#   tests/tests_unit_heartbeat.py:30-32
REFERENCE_IMPORTS = """
from heartbeat.exc import HeartbeatError
from heartbeat import PySwizzle
from heartbeat import Swizzle
import heartbeat
from heartbeat import Heartbeat
"""


def test_reference_import_lines_run_in_a_fresh_interpreter(tmp_path):
    """A fresh interpreter outside the repo (only PYTHONPATH points at it), so
    no module cached by this session hides a broken import."""
    check = REFERENCE_IMPORTS + """
import heartbeat_amd
assert Heartbeat is heartbeat.Swizzle.Swizzle is Swizzle.Swizzle
assert HeartbeatError is heartbeat_amd.HeartbeatError is heartbeat.exc.HeartbeatError
assert PySwizzle.PySwizzle is heartbeat_amd.PySwizzle.PySwizzle
assert PySwizzle.KeyedPRF is heartbeat.util.KeyedPRF is heartbeat_amd.util.KeyedPRF
for name in ("KeyedPRF", "Challenge", "Tag", "State", "Proof", "PySwizzle"):
    assert getattr(PySwizzle, name) is getattr(heartbeat_amd.PySwizzle, name), name
for name in ("Swizzle", "State", "Tag", "Challenge", "Proof"):
    assert getattr(Swizzle, name) is getattr(heartbeat_amd.Swizzle, name), name
assert heartbeat.__version__ == "0.1.4" and PySwizzle.__version__ == "0.1.4"
print("ok")
"""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", check], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"


def test_one_exception_class():
    import heartbeat
    import heartbeat_amd
    from heartbeat.exc import HeartbeatError
    from heartbeat import PySwizzle

    assert HeartbeatError.__module__ == "heartbeat.exc"
    st = PySwizzle.State(b"f" * 32, b"a" * 32, 5, key=b"k" * 32)
    # an error raised inside heartbeat_amd is caught by the reference's except clause
    with pytest.raises(heartbeat.exc.HeartbeatError, match="Signature invalid on state."):
        st.decrypt(b"wrong key")
    try:
        st.decrypt(b"wrong key")
    except heartbeat_amd.exc.HeartbeatError as e:
        assert type(e) is HeartbeatError
        assert e.message == str(e) == "Signature invalid on state."


def test_pickles_name_reference_paths():
    from heartbeat import PySwizzle, Swizzle

    t = PySwizzle.Tag()
    t.sigma = [1, 2, 3]
    c = PySwizzle.Challenge(7, 11, b"k" * 32)
    for obj, mod in ((t, b"heartbeat.PySwizzle.PySwizzle"), (c, b"heartbeat.PySwizzle.PySwizzle"),
                     (Swizzle.Challenge(), b"heartbeat.Swizzle")):
        blob = pickle.dumps(obj)
        assert mod in blob and b"heartbeat_amd" not in blob
        back = pickle.loads(blob)
        assert type(back) is type(obj)
    assert pickle.loads(pickle.dumps(t)).sigma == [1, 2, 3]
    assert pickle.loads(pickle.dumps(c)).todict() == c.todict()


def test_reference_pickle_paths_load_here():
    """A pickle written under the reference's paths (protocol 2, as the
    reference package would write it) loads into this build's classes."""
    from heartbeat import PySwizzle

    blob = (b"\x80\x02cheartbeat.PySwizzle.PySwizzle\nChallenge\nq\x00)\x81q\x01}q\x02"
            b"(X\x06\x00\x00\x00chunksq\x03K\x05X\x05\x00\x00\x00v_maxq\x04K\x0bX\x03\x00\x00\x00keyq\x05"
            b"C\x02abq\x06ub.")
    c = pickle.loads(blob)
    assert type(c) is PySwizzle.Challenge
    assert (c.chunks, c.v_max, c.key) == (5, 11, b"ab")


def test_merkle_names():
    import heartbeat
    from heartbeat.Merkle import DEFAULT_CHUNK_SIZE, MerkleHelper
    import heartbeat_amd.Merkle

    assert MerkleHelper is heartbeat_amd.Merkle.MerkleHelper and DEFAULT_CHUNK_SIZE == 8192
    with pytest.raises(AttributeError, match="outside this build's scope"):
        heartbeat.Merkle.Merkle
