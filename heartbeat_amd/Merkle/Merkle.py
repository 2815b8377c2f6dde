"""MerkleHelper (heartbeat/Merkle/Merkle.py:447-515) over the GPU KeyedPRF.

The Merkle scheme picks, for every challenge seed, the chunk of the file that
the challenge checks: ``KeyedPRF(seed, filesz - chunksz + 1).eval(0)``
(Merkle.py:502-503), and its leaf is HMAC-SHA256(seed, chunk)
(:505-515).  ``Merkle.encode`` does this for 256 seeds of an HMAC chain
(:357-361).  Here the positions of any number of seeds come from ONE kernel
launch (``hb_merkle_offsets``: a lane per seed, each expanding its own AES
key schedule), and for device-resident files the leaves too
(``hb_merkle_chunk_hmacs``: a lane per chunk).  Host files are hashed on the
host, reading the chunk through the file object as the reference does: the
bytes are already there, and one SHA-256 stream is serial.

The tree, the Challenge/Tag/State/Proof containers and the Merkle class are
the reference's other scheme and out of scope.
"""
import ctypes
import hashlib
import hmac

import numpy as np

from .. import _native, multi
from ..exc import HeartbeatError

DEFAULT_CHUNK_SIZE = 8192     # Merkle.py:38
DEFAULT_BUFFER_SIZE = 65536   # Merkle.py:39


def _seed_block(seeds):
    seeds = [bytes(s) for s in seeds]
    n = len(seeds)
    if n == 0:
        return b"", 0, 0
    sl = len(seeds[0])
    if any(len(s) != sl for s in seeds):
        raise HeartbeatError("seeds of one batch must have one length")
    return b"".join(seeds), sl, n


class MerkleHelper(object):
    """Helper functions of the Merkle scheme (Merkle.py:447-515)."""

    @staticmethod
    def get_next_seed(key, seed):
        """HMAC-SHA256(key, seed): the next seed of the chain (Merkle.py:451-460)."""
        return hmac.new(key, seed, hashlib.sha256).digest()

    @staticmethod
    def seed_chain(key, seed, n):
        """The n leaf seeds Merkle.encode derives from the state seed
        (Merkle.py:357-361): s_1 = next(key, seed), s_{k+1} = next(key, s_k)."""
        out = []
        s = seed
        for _ in range(n):
            s = MerkleHelper.get_next_seed(key, s)
            out.append(s)
        return out

    @staticmethod
    def get_file_hash(file, seed, bufsz=DEFAULT_BUFFER_SIZE):
        """HMAC-SHA256(seed, rest of the file) (Merkle.py:462-478): a host read loop."""
        h = hmac.new(seed, None, hashlib.sha256)
        while True:
            buffer = file.read(bufsz)
            h.update(buffer)
            if len(buffer) != bufsz:
                break
        return h.digest()

    @staticmethod
    def chunk_offsets(seeds, filesz, chunksz=DEFAULT_CHUNK_SIZE):
        """Chunk positions KeyedPRF(seed, filesz - chunk + 1).eval(0) of many
        seeds, chunk = min(chunksz, filesz) (Merkle.py:500-503), in one GPU
        launch.  Seeds are AES keys: 16, 24 or 32 bytes."""
        blob, sl, n = _seed_block(seeds)
        if n == 0:
            return []
        out = np.zeros(n, dtype=np.uint64)
        ctx = multi.primary_context()
        with ctx.lock:
            ctx.check(_native.lib().hb_merkle_offsets(ctx.h, blob, sl, n, int(filesz), int(chunksz),
                                                      out.ctypes.data))
        return [int(x) for x in out]

    @staticmethod
    def get_chunk_hash(file, seed, filesz=None, chunksz=DEFAULT_CHUNK_SIZE, bufsz=DEFAULT_BUFFER_SIZE):
        """The leaf of one seed (Merkle.py:480-515): HMAC-SHA256(seed, the
        chunksz bytes at KeyedPRF(seed, filesz - chunksz + 1).eval(0)).
        Leaves the file after the chunk, as the reference's reads do."""
        return MerkleHelper.get_chunk_hashes(file, [seed], filesz, chunksz, bufsz)[0]

    @staticmethod
    def get_chunk_hashes(file, seeds, filesz=None, chunksz=DEFAULT_CHUNK_SIZE, bufsz=DEFAULT_BUFFER_SIZE):
        """get_chunk_hash for many seeds: positions in one GPU launch, leaves
        hashed on the host from the file object (seek + reads of bufsz)."""
        if filesz is None:
            file.seek(0, 2)
            filesz = file.tell()
        if filesz < chunksz:
            chunksz = filesz
        offs = MerkleHelper.chunk_offsets(seeds, filesz, chunksz)
        out = []
        for seed, i in zip(seeds, offs):
            file.seek(i)
            h = hmac.new(seed, None, hashlib.sha256)
            left, bs = chunksz, bufsz
            while True:
                if left < bs:
                    bs = left
                buffer = file.read(bs)
                h.update(buffer)
                left -= len(buffer)
                if left == 0:
                    break
                if not buffer:
                    # the reference loops forever here (a filesz larger than the file)
                    raise HeartbeatError("file shorter than filesz")
            out.append(h.digest())
        return out

    @staticmethod
    def device_chunk_hashes(data_ptr, length, seeds, filesz=None, chunksz=DEFAULT_CHUNK_SIZE):
        """Leaves of many seeds over a DEVICE-resident file (hb_device_malloc'd
        pointer, `length` bytes): positions and HMACs both on the GPU.
        Returns (offsets, digests)."""
        filesz = length if filesz is None else int(filesz)
        if filesz < chunksz:
            chunksz = filesz
        offs = MerkleHelper.chunk_offsets(seeds, filesz, chunksz)
        blob, sl, n = _seed_block(seeds)
        if n == 0:
            return [], []
        oarr = np.asarray(offs, dtype=np.uint64)
        dig = ctypes.create_string_buffer(32 * n)
        ctx = multi.primary_context()
        with ctx.lock:
            ctx.check(_native.lib().hb_merkle_chunk_hmacs(ctx.h, blob, sl, n, data_ptr, int(length),
                                                          oarr.ctypes.data, int(chunksz), dig))
        raw = dig.raw
        return offs, [raw[32 * k:32 * (k + 1)] for k in range(n)]


MerkleHelper.__module__ = "heartbeat.Merkle.Merkle"   # the reference's path (repo heartbeat/ package)
