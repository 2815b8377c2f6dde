"""heartbeat -- the reference's import surface over the MI355X build.

Reference callers keep their imports unchanged (heartbeat/__init__.py:28-36,
tests/tests_unit_pyswpriv.py:38-39, tests_unit_swpriv.py:38-39,
tests_unit_heartbeat.py:30-32):

    import heartbeat
    from heartbeat import Heartbeat, PySwizzle, Swizzle
    from heartbeat.exc import HeartbeatError

Every name here is the object the GPU-backed package ``heartbeat_amd``
defines: this package holds no logic of its own.  Classes carry the
reference's module paths (``heartbeat.PySwizzle.PySwizzle.Tag``,
``heartbeat.Swizzle.State``, ``heartbeat.exc.HeartbeatError`` ...), so pickles
name ``heartbeat.*`` and ``except heartbeat.exc.HeartbeatError`` catches every
error the library raises.  The Merkle tree scheme and OneHash stay outside
this build's scope; ``heartbeat.Merkle`` carries MerkleHelper.
"""
__version__ = "0.1.4"

import heartbeat.Swizzle    # NOQA
import heartbeat.Merkle     # NOQA
import heartbeat.PySwizzle  # NOQA
from .exc import HeartbeatError  # NOQA


Heartbeat = heartbeat.Swizzle.Swizzle
