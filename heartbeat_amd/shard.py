"""Block-range sharding of one Swizzle encode over N GPUs (one process each).

Blocks are independent (tag_i depends on the global block index i, block i's
bytes and the keys; PySwizzle.py:296-309), so rank r encodes a contiguous
block range with ``block_base`` = its first block and the tags of all ranks
concatenate, in rank order, to the single-device tags.  No collective is needed
in the data path.
"""


def block_range(nblocks, rank, world):
    """[b0, b1) of `nblocks` for `rank` of `world` (contiguous, balanced)."""
    return nblocks * rank // world, nblocks * (rank + 1) // world


def shard_plan(file_len, block_bytes, rank, world):
    """This rank's piece of a whole-file encode of `file_len` bytes.

    Returns dict(b0, nblocks, byte_off, byte_len): the rank passes the bytes
    [byte_off, byte_off + byte_len) with block_base = b0 and nblocks blocks to
    hb_encode.  The whole file has file_len // block_bytes + 1 tags (the last
    one covers the partial or empty tail block, PySwizzle.py:304-309); it falls
    in the last rank's range.
    """
    total = file_len // block_bytes + 1
    b0, b1 = block_range(total, rank, world)
    off = b0 * block_bytes
    end = min(b1 * block_bytes, file_len)
    return {"b0": b0, "nblocks": b1 - b0, "byte_off": off, "byte_len": max(0, end - off),
            "total_blocks": total}
