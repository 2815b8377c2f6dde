"""GPU parity of Merkle's KeyedPRF-positioned chunk hashing
(heartbeat/Merkle/Merkle.py:447-515): heartbeat_amd.Merkle's
MerkleHelper (hb_merkle_offsets / hb_merkle_chunk_hmacs) against the golden
leaves of the reference MerkleHelper (tests/golden/merkle_cases.json) and the
oracle restatement (oracle.merkle_chunk_hash) on larger batches."""
import ctypes
import hashlib
import io
import json
import os

import numpy as np
import pytest

from test_oracle import _merkle_file

pytestmark = pytest.mark.gpu

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_cases.json")))


@pytest.fixture(scope="module")
def MH():
    from heartbeat_amd import _native
    _native.context()
    from heartbeat_amd.Merkle import MerkleHelper
    return MerkleHelper


def _dev(data):
    from heartbeat_amd import _native
    ctx = _native.context()
    L = _native.lib()
    p = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, max(1, len(data)), ctypes.byref(p)))
    a = np.frombuffer(data, dtype=np.uint8)
    if len(a):
        ctx.check(L.hb_memcpy(ctx.h, p.value, a.ctypes.data, len(a), 1))
    return p.value


def _free(p):
    from heartbeat_amd import _native
    ctx = _native.context()
    ctx.check(_native.lib().hb_device_free(ctx.h, p))


def test_chunk_hash_golden_host_file(MH):
    """get_chunk_hash / get_chunk_hashes on BytesIO files == the reference."""
    for c in G["cases"]:
        data = _merkle_file(c["file"])
        seeds = [bytes.fromhex(s) for s in c["seeds"]]
        got = MH.get_chunk_hashes(io.BytesIO(data), seeds, None, c["chunksz"])
        assert [x.hex() for x in got] == c["leaves"], (c["file"], c["chunksz"])
        assert MH.get_chunk_hash(io.BytesIO(data), seeds[0], None, c["chunksz"]).hex() == c["leaves"][0]
        if "leaves_explicit_small_buf" in c:
            got2 = [MH.get_chunk_hash(io.BytesIO(data), s, len(data), c["chunksz"], 37).hex() for s in seeds[:4]]
            assert got2 == c["leaves_explicit_small_buf"]


def test_chunk_hash_golden_device_file(MH):
    """Positions and HMACs both on the GPU (device-resident file) == the reference."""
    for c in G["cases"]:
        data = _merkle_file(c["file"])
        seeds = [bytes.fromhex(s) for s in c["seeds"]]
        p = _dev(data)
        try:
            offs, digs = MH.device_chunk_hashes(p, len(data), seeds, None, c["chunksz"])
        finally:
            _free(p)
        assert [x.hex() for x in digs] == c["leaves"], (c["file"], c["chunksz"])


def test_merkle_encode_batch_vs_oracle(MH, oracle):
    """Merkle.encode's 256 leaves (a seed chain, Merkle.py:357-361) over a
    1 MiB device-resident file, plus 1,000 seeds with 100-byte chunks: the
    GPU offsets and leaves == the oracle's."""
    data = hashlib.sha256(b"m").digest() * (1 << 15) + b"tail-bytes"
    key, seed = b"K" * 32, b"S" * 32
    p = _dev(data)
    try:
        for n, chunksz in ((256, 8192), (1000, 100), (64, len(data))):
            seeds = MH.seed_chain(key, seed, n)
            offs, digs = MH.device_chunk_hashes(p, len(data), seeds, None, chunksz)
            want = [oracle.merkle_chunk(s, len(data), chunksz)[0] for s in seeds]
            assert offs == want
            assert [d.hex() for d in digs] == [oracle.merkle_chunk_hash(data, s, None, chunksz).hex()
                                               for s in seeds]
    finally:
        _free(p)


def test_chunk_past_end_rejected(MH):
    from heartbeat_amd.exc import HeartbeatError
    data = b"x" * 1000
    p = _dev(data)
    try:
        with pytest.raises(HeartbeatError):
            MH.device_chunk_hashes(p, len(data), MH.seed_chain(b"k" * 32, b"s" * 32, 16), 5000, 100)
    finally:
        _free(p)
