"""heartbeat.Merkle.Merkle: MerkleHelper from heartbeat_amd.Merkle.Merkle."""
from heartbeat_amd.Merkle.Merkle import DEFAULT_BUFFER_SIZE, DEFAULT_CHUNK_SIZE, MerkleHelper  # NOQA

__all__ = ["DEFAULT_CHUNK_SIZE", "DEFAULT_BUFFER_SIZE", "MerkleHelper"]
