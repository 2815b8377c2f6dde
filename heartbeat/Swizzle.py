"""heartbeat.Swizzle: the cxx extension module's names (cxx/Swizzle.hxx:734-762:
Swizzle, State, Tag, Challenge, Proof), GPU-backed in heartbeat_amd.Swizzle."""
from heartbeat_amd.Swizzle import Challenge, Proof, State, Swizzle, Tag  # NOQA

__all__ = ["Swizzle", "State", "Tag", "Challenge", "Proof"]
