"""configs[4] at its own index width: PySwizzle.prove on
the 64 GiB, 16-sector, 256-bit file with a 10,000-index challenge, i.e.
N = 2^27 + 1 tags, so the index KeyedPRF draws from a 28-bit range with
nb = 4 digest bytes (PySwizzle.py:344, util.py:83-96) -- wider than every
other GPU prove test (<= 24 bits).

The oracle needs only the challenged blocks: the host mirror of the file is a
64 GiB zero mapping (virtual; only touched pages are backed) into which the
challenged blocks are regenerated from the SplitMix64 stream the device was
filled with (hb_fill_random == conftest.splitmix_bytes), and the tags are the
device's, downloaded.  Checked: hb_prove (device-resident) == oracle.prove;
hb_prove_range over [0, 5000) and [5000, 10000) summed mod p == the whole
proof; hb_verify_rhs(proof) == sigma; the challenge reaches past block 2^26
(the 28-bit range is exercised, not just declared).

A second case runs the host-gather path (mode 2 of hb_wsum_kernel) at a 26-bit
index range: configs[1]'s 1 GiB, 1-sector file (2^25 + 1 tags), file and tags
in host memory.  Bar: bit-exact.  Reference: PySwizzle.py:333-370, 372-395.
"""
import ctypes
import hashlib

import numpy as np
import pytest

from conftest import splitmix_bytes

pytestmark = pytest.mark.gpu

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
GIB = 1 << 30


def _ints(raw, w, n):
    return [int.from_bytes(raw[j * w:(j + 1) * w], "big") for j in range(n)]


def _oracle_prove(oracle, p, S, key, chunks, vmax, nb, tags_addr, data_addr, length):
    w = 32
    pb = p.to_bytes(w, "big")
    vb = vmax.to_bytes(w, "big")
    mu = ctypes.create_string_buffer(w * S)
    sg = ctypes.create_string_buffer(w)
    rc = oracle.lib().hbo_prove(pb, len(pb), S, key, len(key), chunks, vb, len(vb), nb,
                                ctypes.cast(tags_addr, ctypes.c_char_p), w, data_addr, length, mu, sg)
    assert rc == 0
    return _ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")


def _sparse_mirror(seed, length, C, blocks):
    """A `length`-byte host array holding the SplitMix64 bytes of `blocks` only."""
    host = np.zeros(length, dtype=np.uint8)          # calloc: untouched pages stay unbacked
    for b in sorted(set(blocks)):
        lo, hi = b * C, min((b + 1) * C, length)
        if hi > lo:
            host[lo:hi] = np.frombuffer(splitmix_bytes(seed, lo, hi - lo), dtype=np.uint8)
    return host


def test_configs4_prove_at_28_bit_index_width(oracle):
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p, S, C, w = P256, 16, 512, 32
    length = 64 * GIB
    nb = length // C + 1
    assert nb == (1 << 27) + 1 and nb.bit_length() == 28   # configs[4]'s N, nb = 4 digest bytes
    seed = 0x5EED0000 + 3                                    # bench.py c5's stream
    fk = hashlib.sha256(b"hb-bench-f").digest()
    ak = hashlib.sha256(b"hb-bench-alpha").digest()
    key = hashlib.sha256(b"hb-bench-challenge").digest()
    chunks = 10000
    pb = nat.be(p)
    dptr, tptr = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, length, ctypes.byref(dptr)))
    ctx.check(L.hb_device_malloc(ctx.h, nb * w, ctypes.byref(tptr)))
    try:
        ctx.check(L.hb_fill_random(ctx.h, dptr, length, seed))
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, dptr, length, nb, tptr, 3, None))
        mu = ctypes.create_string_buffer(w * S)
        sg = ctypes.create_string_buffer(w)
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), tptr, nb, dptr, length, 3,
                             mu, sg))
        gmu, gsg = _ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")
        # the challenged indices (the oracle's index PRF, range N = 2^27 + 1)
        idx = [oracle.prf_eval(key, nb, i) for i in range(chunks)]
        assert max(idx) >= 1 << 26, "the 28-bit index range is not exercised"
        host = _sparse_mirror(seed, length, C, idx)
        tags = np.empty(nb * w, dtype=np.uint8)
        ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data, tptr.value, nb * w, 2))
        omu, osg = _oracle_prove(oracle, p, S, key, chunks, p, nb, tags.ctypes.data, host.ctypes.data, length)
        assert gmu == omu
        assert gsg == osg
        # two halves of the challenge (multi-device prove) add up mod p
        parts = []
        for i0, i1 in ((0, 5000), (5000, chunks)):
            m = ctypes.create_string_buffer(w * S)
            s = ctypes.create_string_buffer(w)
            ctx.check(L.hb_prove_range(ctx.h, pb, len(pb), S, key, 32, chunks, i0, i1, pb, len(pb), tptr, nb,
                                       dptr, length, 3, m, s))
            parts.append((_ints(m.raw, w, S), int.from_bytes(s.raw, "big")))
        assert [(a + b) % p for a, b in zip(parts[0][0], parts[1][0])] == omu
        assert (parts[0][1] + parts[1][1]) % p == osg
        # and the proof verifies (PySwizzle.py:372-395)
        rhs = ctypes.create_string_buffer(w)
        ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, 32, nb, key, 32, chunks, pb, len(pb),
                                  mu.raw, rhs))
        assert int.from_bytes(rhs.raw, "big") == gsg
    finally:
        ctx.check(L.hb_device_free(ctx.h, dptr))
        ctx.check(L.hb_device_free(ctx.h, tptr))


def test_configs1_host_gather_prove_at_26_bit_index_width(oracle):
    """1 GiB, S = 1 (2^25 + 1 tags): file and tags in host memory, the
    challenged blocks gathered on the host (the reference's seek/read per
    index) and summed on the GPU; == the oracle and == the device-resident
    proof."""
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p, S, C, w = P256, 1, 32, 32
    length = GIB
    nb = length // C + 1
    assert nb.bit_length() == 26
    seed = 0x5EED0000 + 2
    key = hashlib.sha256(b"c1-wide-index").digest()
    chunks = 10000
    pb = nat.be(p)
    dptr, tptr = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, length, ctypes.byref(dptr)))
    ctx.check(L.hb_device_malloc(ctx.h, nb * w, ctypes.byref(tptr)))
    try:
        ctx.check(L.hb_fill_random(ctx.h, dptr, length, seed))
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, b"f" * 32, b"a" * 32, 32, 0, dptr, length, nb, tptr, 3,
                              None))
        host = np.empty(length, dtype=np.uint8)
        tags = np.empty(nb * w, dtype=np.uint8)
        ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value, length, 2))
        ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data, tptr.value, nb * w, 2))
        # the full-size configs[1] tags themselves against the oracle: the
        # first and last 1,000 blocks (the PRF-only tail block included) and
        # 10,000 random ones (PySwizzle.py:296-309 at S = 1)
        rng = np.random.default_rng(0xC1)
        picks = sorted(set(range(1000)) | set(range(nb - 1000, nb)) | set(rng.integers(0, nb, 10000).tolist()))
        runs, i = [], 0
        while i < len(picks):
            j = i
            while j + 1 < len(picks) and picks[j + 1] == picks[j] + 1:
                j += 1
            runs.append((picks[i], picks[j] + 1))
            i = j + 1
        for r0, r1 in runs:
            want = oracle.encode(p, S, b"f" * 32, b"a" * 32, host[r0 * C:r1 * C].tobytes(), block_base=r0,
                                 nblocks=r1 - r0, nthreads=4)
            assert tags[r0 * w:r1 * w].tobytes() == b"".join(t.to_bytes(w, "big") for t in want), (r0, r1)
        res = []
        for tp, dp, flags in ((tptr.value, dptr.value, 3), (tags.ctypes.data, host.ctypes.data, 0)):
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), tp, nb, dp, length, flags,
                                 mu, sg))
            res.append((_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")))
        idx = [oracle.prf_eval(key, nb, i) for i in range(chunks)]
        assert max(idx) >= 1 << 24
        want = _oracle_prove(oracle, p, S, key, chunks, p, nb, tags.ctypes.data, host.ctypes.data, length)
        assert res[0] == want
        assert res[1] == want
    finally:
        ctx.check(L.hb_device_free(ctx.h, dptr))
        ctx.check(L.hb_device_free(ctx.h, tptr))
