"""heartbeat.Merkle: the part of the reference subpackage this build covers,
MerkleHelper (heartbeat/Merkle/Merkle.py:447-515) with GPU chunk positions
and leaves.  The Merkle tree scheme itself (Merkle, MerkleTree and its
Challenge/Tag/State/Proof) is outside the build's scope (SURVEY.md 2 row 13,
DESIGN.md 1): asking for it raises an AttributeError that says so."""
from .Merkle import DEFAULT_BUFFER_SIZE, DEFAULT_CHUNK_SIZE, MerkleHelper  # NOQA

__version__ = "0.1.4"
# the submodule stays in sys.modules (pickles name heartbeat.Merkle.Merkle);
# the package attribute is the reference's Merkle CLASS, which is out of scope
del Merkle  # NOQA

_OUT_OF_SCOPE = ("Merkle", "MerkleTree", "Challenge", "Tag", "State", "Proof")


def __getattr__(name):
    if name in _OUT_OF_SCOPE:
        raise AttributeError("heartbeat.Merkle.%s: the Merkle tree scheme is outside this build's scope "
                             "(only MerkleHelper is provided; DESIGN.md 1)" % name)
    raise AttributeError("module 'heartbeat.Merkle' has no attribute %r" % name)
