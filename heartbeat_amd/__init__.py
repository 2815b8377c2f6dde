"""heartbeat_amd -- MI355X-native Swizzle (Shacham-Waters private PDP)
encode/prove hot path behind the heartbeat API.

    import heartbeat_amd.PySwizzle as PySwizzle     # drop-in for heartbeat.PySwizzle
    from heartbeat_amd import HeartbeatError

Compute runs in hand-written HIP kernels for gfx950 (libhbswizzle.so, C ABI in
include/hbswizzle.h); see DESIGN.md.  ``heartbeat_amd.Swizzle.Swizzle`` mirrors
the C++ extension's ``heartbeat.Swizzle`` objects over the kernels' cxx mode
(parity unpinned); as in the reference package (heartbeat/__init__.py:28-36)
``Heartbeat`` is that Swizzle class.  The Merkle / OneHash schemes are outside
this build's scope.
"""
__version__ = "0.1.4"

from . import PySwizzle  # NOQA
from . import Swizzle  # NOQA
from .exc import HeartbeatError  # NOQA
from .util import KeyedPRF  # NOQA

Heartbeat = Swizzle.Swizzle
