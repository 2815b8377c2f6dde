"""configs[3] on one GPU ("emulating shards sequentially"): the
256 GiB file, 512-byte blocks (256-bit prime, 16 sectors), sharded over 8
ranks by heartbeat_amd.shard.shard_plan exactly as `bench.py --gpus 8` does,
run as eight sequential ~32 GiB shard launches on one device.

One resident 32 GiB buffer is refilled per shard with that shard's SplitMix64
stream (the bench's per-rank seed), encoded with block_base = the shard's first
block; the last shard carries the ragged end, i.e. the PRF-only tail block of
a file whose length is a multiple of the block size (PySwizzle.py:304-309).
For every shard the first and last 1,000 tags and 1,250 random ones equal the
oracle (oracle/swizzle_oracle.c) on the host copy of the same stream.
Bar: bit-exact.  Reference: PySwizzle.py:296-309 (block i's tag depends on
i, its bytes and the keys only), SURVEY.md 8(e)."""
import ctypes
import hashlib

import numpy as np
import pytest

from conftest import splitmix_bytes

pytestmark = pytest.mark.gpu

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
GIB = 1 << 30


def test_configs3_eight_shards_sequential_on_one_gpu(oracle):
    from heartbeat_amd import _native as nat
    from heartbeat_amd.shard import shard_plan
    ctx = nat.context()
    L = nat.lib()
    p, S, C, w, world = P256, 16, 512, 32, 8
    file_len = 256 * GIB
    plans = [shard_plan(file_len, C, g, world) for g in range(world)]
    total = plans[0]["total_blocks"]
    assert total == file_len // C + 1
    assert sum(pl["nblocks"] for pl in plans) == total
    assert plans[-1]["byte_off"] + plans[-1]["byte_len"] == file_len
    max_len = max(pl["byte_len"] for pl in plans)
    max_nb = max(pl["nblocks"] for pl in plans)
    assert max_len <= 33 * GIB
    fk = hashlib.sha256(b"hb-bench-f").digest()
    ak = hashlib.sha256(b"hb-bench-alpha").digest()
    pb = nat.be(p)
    dptr, tptr = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, max_len, ctypes.byref(dptr)))
    ctx.check(L.hb_device_malloc(ctx.h, max_nb * w, ctypes.byref(tptr)))
    try:
        rng = np.random.default_rng(3)
        tail_seen = False
        for g, pl in enumerate(plans):
            seed = 0x5EED0000 + 3 + g
            n, nb, b0 = pl["byte_len"], pl["nblocks"], pl["b0"]
            ctx.check(L.hb_fill_random(ctx.h, dptr, n, seed))
            tries = ctypes.c_uint64()
            ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, b0, dptr, n, nb, tptr, 3,
                                  ctypes.byref(tries)))
            assert tries.value >= nb
            runs = [(0, 1000), (nb - 1000, 1000)] + [(int(b), 1) for b in rng.integers(0, nb, 1250)]
            for r0, k in runs:
                got = np.empty(k * w, dtype=np.uint8)
                ctx.check(L.hb_memcpy(ctx.h, got.ctypes.data, tptr.value + r0 * w, k * w, 2))
                lo, hi = r0 * C, min((r0 + k) * C, n)
                data = splitmix_bytes(seed, lo, max(0, hi - lo))
                want = oracle.encode(p, S, fk, ak, data, block_base=b0 + r0, nblocks=k)
                assert got.tobytes() == b"".join(t.to_bytes(w, "big") for t in want), (g, r0)
            if g == world - 1:
                # the file's last tag: block 2^29 has no bytes (PRF only)
                assert b0 + nb - 1 == file_len // C and nb * C > n
                tail_seen = True
        assert tail_seen
    finally:
        ctx.check(L.hb_device_free(ctx.h, dptr))
        ctx.check(L.hb_device_free(ctx.h, tptr))
