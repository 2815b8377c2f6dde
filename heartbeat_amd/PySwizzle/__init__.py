"""heartbeat_amd.PySwizzle: GPU-backed drop-in for heartbeat.PySwizzle
(reference re-export list: heartbeat/PySwizzle/__init__.py:28)."""
from .PySwizzle import KeyedPRF, Challenge, Tag, State, Proof, PySwizzle  # NOQA

__version__ = "0.1.4"
