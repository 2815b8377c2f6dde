"""The Merkle scheme's use of KeyedPRF (heartbeat/Merkle/Merkle.py:447-515):
MerkleHelper with GPU chunk positions and leaves.  The Merkle tree scheme
itself is out of scope."""
from .Merkle import DEFAULT_BUFFER_SIZE, DEFAULT_CHUNK_SIZE, MerkleHelper  # NOQA
