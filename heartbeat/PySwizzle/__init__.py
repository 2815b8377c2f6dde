"""heartbeat.PySwizzle (reference heartbeat/PySwizzle/__init__.py:28).  As
there, ``heartbeat.PySwizzle.PySwizzle`` is the class once the package is
imported; the module stays reachable as sys.modules entry (pickles use it)."""
from .PySwizzle import KeyedPRF, Challenge, Tag, State, Proof, PySwizzle  # NOQA

__version__ = "0.1.4"
