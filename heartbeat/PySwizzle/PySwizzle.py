"""heartbeat.PySwizzle.PySwizzle (reference heartbeat/PySwizzle/PySwizzle.py):
the scheme's classes from heartbeat_amd.PySwizzle.PySwizzle, whose encode /
prove / verify run on the GPU."""
from ..util import KeyedPRF  # NOQA  (as the reference module: heartbeat.util)
from heartbeat_amd.PySwizzle.PySwizzle import (  # NOQA
    Challenge, Proof, PySwizzle, State, Tag, encode_file, getPrime)

__all__ = ["KeyedPRF", "Challenge", "Tag", "State", "Proof", "PySwizzle", "getPrime"]
