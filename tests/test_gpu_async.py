"""GPU tests of the asynchronous C-ABI variant ("calls are
synchronous; an async variant takes a hipStream_t"): hb_encode with HB_ASYNC
returns once the encode kernels are enqueued, hb_ctx_wait completes it, and
hb_ctx_set_stream puts the context's kernels on a caller's HIP stream.  Tags must equal the synchronous encode's."""
import ctypes
import hashlib

import pytest

from test_gpu_parity import P256, DevBuf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    from heartbeat_amd import _native
    _native.context()
    return _native


def test_async_encode_equals_sync(nat):
    p, S, L = P256, 16, 16 << 20
    nb = L // 512 + 1
    pb = nat.be(p)
    fk, ak = hashlib.sha256(b"async-f").digest(), hashlib.sha256(b"async-a").digest()
    buf = DevBuf(nat, L)
    tbs = [DevBuf(nat, nb * 32) for _ in range(4)]
    ctx = nat.context()
    L_ = nat.lib()
    try:
        ctx.check(L_.hb_fill_random(ctx.h, buf.p, L, 99))
        tries = ctypes.c_uint64(0)
        ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tbs[0].p, 3, ctypes.byref(tries)))
        # async + explicit wait
        t2 = ctypes.c_uint64(123)
        ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tbs[1].p, 3 | nat.HB_ASYNC,
                               ctypes.byref(t2)))
        assert t2.value == 0                      # filled by hb_ctx_wait, not here
        ctx.check(L_.hb_ctx_wait(ctx.h, ctypes.byref(t2)))
        assert t2.value == tries.value
        # async, then another call on the context settles it implicitly
        ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tbs[2].p, 3 | nat.HB_ASYNC, None))
        got2 = tbs[2].download()
        # on a caller's stream, created with the HIP runtime the library links
        # (this image's torch bundles its own HIP runtime, a separate instance)
        hip = ctypes.CDLL("libamdhip64.so.7")
        st = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(st)) == 0
        ctx.check(L_.hb_ctx_set_stream(ctx.h, st))
        try:
            ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tbs[3].p, 3 | nat.HB_ASYNC,
                                   None))
            assert hip.hipStreamSynchronize(st) == 0
            ctx.check(L_.hb_ctx_wait(ctx.h, None))
        finally:
            ctx.check(L_.hb_ctx_set_stream(ctx.h, None))
            hip.hipStreamDestroy(st)
        want = tbs[0].download()
        assert tbs[1].download() == want and got2 == want and tbs[3].download() == want
        # nothing pending: wait is a no-op
        ctx.check(L_.hb_ctx_wait(ctx.h, None))
        # HB_ASYNC needs device data and tags
        host = ctypes.create_string_buffer(L)
        rc = L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, host, L, nb, tbs[0].p, 2 | nat.HB_ASYNC, None)
        assert rc == -1 and b"HB_ASYNC" in L_.hb_last_error(ctx.h)
    finally:
        buf.free()
        for tb in tbs:
            tb.free()


def test_async_status_and_timing_accumulate(nat, monkeypatch):
    """Two HB_ASYNC encodes before one hb_ctx_wait: the wait reports both
    (tries summed; a failure of the first would be kept), and
    hb_last_kernel_ms completes a pending encode instead of reporting the
    previous operation's time.  (The two-pass engine throughout: on the
    small-input path an 8 MiB and a 2-block encode are both one latency-bound
    PRF chain long, too close to tell apart by time.)"""
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
    p, S, L = P256, 16, 8 << 20
    nb = L // 512 + 1
    pb = nat.be(p)
    fk, ak = hashlib.sha256(b"async2-f").digest(), hashlib.sha256(b"async2-a").digest()
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    ctx = nat.context()
    L_ = nat.lib()
    try:
        ctx.check(L_.hb_fill_random(ctx.h, buf.p, L, 7))
        tries = ctypes.c_uint64(0)
        ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tb.p, 3, ctypes.byref(tries)))
        sync_ms, _ = ctx.last_kernel_ms()
        want = tb.download()
        for _ in range(2):
            ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tb.p, 3 | nat.HB_ASYNC, None))
        t2 = ctypes.c_uint64(0)
        ctx.check(L_.hb_ctx_wait(ctx.h, ctypes.byref(t2)))
        assert t2.value == 2 * tries.value
        # a tiny synchronous PRF batch sets the timing to its own; the async
        # encode after it must be what hb_last_kernel_ms reports
        ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, 512, 2, tb.p, 3, None))
        small_ms, _ = ctx.last_kernel_ms()
        ctx.check(L_.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, buf.p, L, nb, tb.p, 3 | nat.HB_ASYNC, None))
        big_ms, launches = ctx.last_kernel_ms()
        assert big_ms > 2 * small_ms and 0.5 * sync_ms < big_ms < 2 * sync_ms and launches >= 1
        ctx.check(L_.hb_ctx_wait(ctx.h, ctypes.byref(t2)))
        assert t2.value == tries.value
        assert tb.download() == want
    finally:
        buf.free()
        tb.free()


def test_prepare_then_encode_on_a_fresh_context(nat, oracle):
    """hb_ctx_prepare (load the kernels' code objects ahead of the first call)
    on a fresh context, for every supported prime size; an encode afterwards
    on it equals the oracle; > 2048 bits is refused like hb_encode refuses it."""
    from heartbeat_amd.exc import HeartbeatError
    ctx = nat.Context(0)
    try:
        for bits in (8, 255, 256, 512, 1024, 2048):
            ctx.prepare(bits)
        with pytest.raises(HeartbeatError):
            ctx.prepare(2049)
        p, S, L = P256, 16, 1 << 20
        nb = L // 512 + 1
        pb = nat.be(p)
        data = b"".join(hashlib.sha256(b"prep%d" % i).digest() for i in range(L // 32))
        tags = ctypes.create_string_buffer(nb * 32)
        tries = ctypes.c_uint64()
        ctx.check(nat.lib().hb_encode(ctx.h, pb, len(pb), S, b"f" * 32, b"a" * 32, 32, 0, data, L, nb, tags, 0,
                                      ctypes.byref(tries)))
        want = oracle.encode(p, S, b"f" * 32, b"a" * 32, data)
        assert tags.raw == b"".join(t.to_bytes(32, "big") for t in want)
    finally:
        ctx.close()
