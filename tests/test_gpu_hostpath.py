"""The host-memory boundary with HB_HOST_REGISTER (north_star: "a seekable
file-like object in, tag bytes out"): hb_encode page-locks the file bytes
read-only and the tag buffer for writing in windows pinned ahead of the copies
by helper threads.  Checked against the device-resident encode of the same
bytes (itself pinned to the oracle by test_gpu_parity.py):

* a pageable buffer at an odd address, 2 MiB windows (HB_HOST_WINDOW_MIB, a
  test switch) so that chunks straddle many windows, with look-ahead 1 and 5;
* a read-only mmap of a real file through the drop-in API (encode_file with
  register=True, the default for files: REGISTER_KINDS) and PySwizzle.encode
  on the same open file, S = 1 so the tag windows are as large as the file's;
* memory the caller has registered already (the library's registration of
  those windows fails and they are copied as they are).

Reference: PySwizzle.py:279-314 (the encode loop reads the file object
sector by sector), cxx/PythonSeekableFile.hxx:47-54."""
import ctypes
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)


def _device_tags(nat, host, S, fk, ak):
    ctx = nat.context()
    L = nat.lib()
    n = len(host)
    nb = n // (32 * S) + 1
    d, t = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, max(n, 16), ctypes.byref(d)))
    ctx.check(L.hb_device_malloc(ctx.h, nb * 32, ctypes.byref(t)))
    try:
        ctx.check(L.hb_memcpy(ctx.h, d, host.ctypes.data, n, 1))
        pb = nat.be(P256)
        ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, d, n, nb, t, 3, None))
        out = np.empty(nb * 32, dtype=np.uint8)
        ctx.check(L.hb_memcpy(ctx.h, out.ctypes.data, t.value, nb * 32, 2))
        return out.tobytes()
    finally:
        ctx.check(L.hb_device_free(ctx.h, d))
        ctx.check(L.hb_device_free(ctx.h, t))


def test_register_windows_pageable_buffer(monkeypatch):
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    S = 16
    n = (300 << 20) + 12345
    raw = np.random.default_rng(5).integers(0, 256, n + 7, dtype=np.uint8)
    host = raw[7:]                                     # not page aligned
    fk, ak = b"r" * 32, b"w" * 32
    want = _device_tags(nat, host, S, fk, ak)
    nb = n // (32 * S) + 1
    pb = nat.be(P256)
    monkeypatch.setenv("HB_HOST_WINDOW_MIB", "2")
    for ahead in ("1", "5"):
        monkeypatch.setenv("HB_HOST_AHEAD", ahead)
        tags = np.empty(nb * 32 + 3, dtype=np.uint8)[3:]   # odd tag address too
        ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, host.ctypes.data, n, nb, tags.ctypes.data,
                              nat.HB_HOST_REGISTER, None))
        assert tags.tobytes() == want, ahead


def test_register_real_file_through_the_api(tmp_path):
    from heartbeat_amd import _native as nat
    from heartbeat_amd.PySwizzle import PySwizzle
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    assert "mmap" in pys.REGISTER_KINDS
    S = 1
    n = (96 << 20) + 31
    host = np.random.default_rng(6).integers(0, 256, n, dtype=np.uint8)
    path = tmp_path / "f.bin"
    host.tofile(str(path))
    fk, ak = b"f" * 32, b"a" * 32
    want = _device_tags(nat, host, S, fk, ak)
    with open(str(path), "rb") as f:
        for register in (True, None, False):
            f.seek(0)
            tag, nb = pys.encode_file(P256, S, fk, ak, f, register=register)
            assert f.tell() == n
            assert tag.raw(P256) == want, register
        # the reference's API on the same (unrewound, then rewound) file
        beat = PySwizzle(S, b"k" * 32, P256)
        f.seek(0)
        tag, state = beat.encode(f)
        chal = beat.gen_challenge(state)
        proof = beat.prove(f, chal, tag)
        assert beat.verify(proof, chal, state)


def test_register_memory_the_caller_pinned():
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    S = 16
    n = (64 << 20) + 100
    host = np.random.default_rng(7).integers(0, 256, n, dtype=np.uint8)
    fk, ak = b"c" * 32, b"p" * 32
    want = _device_tags(nat, host, S, fk, ak)
    nb = n // (32 * S) + 1
    tags = np.empty(nb * 32, dtype=np.uint8)
    pb = nat.be(P256)
    ctx.check(L.hb_host_register(ctx.h, host.ctypes.data, n))
    try:
        ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, host.ctypes.data, n, nb, tags.ctypes.data,
                              nat.HB_HOST_REGISTER, None))
    finally:
        ctx.check(L.hb_host_unregister(ctx.h, host.ctypes.data))
    assert tags.tobytes() == want
