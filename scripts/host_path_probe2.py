#!/usr/bin/env python3
"""HB_HOST_REGISTER geometry A/B and the cost of page-locking itself: the
drop-in API's real-file encode (encode_file on a read-only mmap, 4 GiB,
S = 16) with window sizes / look-ahead depths set through the test switches
HB_HOST_WINDOW_MIB / HB_HOST_AHEAD, against the pageable path; and
hipHostRegister(ReadOnly) + hipHostUnregister of the same mapping timed
window by window.  Prints one JSON line."""
import ctypes
import hashlib
import json
import mmap
import os
import sys
import tempfile
import time

import numpy as np

os.environ["HB_ENABLE_TEST_SWITCHES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from heartbeat_amd import _native  # noqa: E402

GIB = 1 << 30
P = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)


def main():
    import importlib
    L = _native.lib()
    ctx = _native.context()
    S, C = 16, 512
    n = 4 * GIB
    nb = n // C + 1
    fk, ak = hashlib.sha256(b"hb-bench-f").digest(), hashlib.sha256(b"hb-bench-alpha").digest()
    d = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(d)))
    ctx.check(L.hb_fill_random(ctx.h, d, n, 1234))
    host = np.empty(n, dtype=np.uint8)
    ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, d.value, n, 2))
    ref = np.empty(nb * 32, dtype=np.uint8)
    pb = _native.be(P)
    ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, d, n, nb, ref.ctypes.data, 1, None))
    ctx.check(L.hb_device_free(ctx.h, d))
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    res = {"api": {}, "register": {}}
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp")) as fh:
        host.tofile(fh.name)
        with open(fh.name, "rb") as f:
            # raw page-locking cost of the file mapping, 256 MiB windows
            for populate in (True, False):
                mm = mmap.mmap(f.fileno(), 0, flags=mmap.MAP_SHARED | (mmap.MAP_POPULATE if populate else 0),
                               prot=mmap.PROT_READ)
                a = np.frombuffer(mm, dtype=np.uint8).ctypes.data
                W = 256 << 20
                reg = unreg = 0.0
                for off in range(0, n, W):
                    t = time.perf_counter()
                    rc = hip.hipHostRegister(a + off, W, 8)
                    reg += time.perf_counter() - t
                    assert rc == 0, rc
                for off in range(0, n, W):
                    t = time.perf_counter()
                    hip.hipHostUnregister(a + off)
                    unreg += time.perf_counter() - t
                res["register"]["populate" if populate else "lazy"] = {
                    "register_s": round(reg, 4), "register_gib_s": round(n / GIB / reg, 2),
                    "unregister_s": round(unreg, 4)}
                mm.close()
            configs = [("pageable", None, None), ("256x2", 256, 2), ("128x4", 128, 4), ("512x1", 512, 1),
                       ("256x4", 256, 4)]
            for rep in range(5):
                for name, wmib, ahead in configs:
                    if wmib:
                        os.environ["HB_HOST_WINDOW_MIB"] = str(wmib)
                        os.environ["HB_HOST_AHEAD"] = str(ahead)
                    f.seek(0)
                    t = time.perf_counter()
                    tag, _ = pys.encode_file(P, S, fk, ak, f, register=wmib is not None)
                    dt = time.perf_counter() - t
                    assert tag._raw[:nb * 32] == ref.tobytes()
                    res["api"].setdefault(name, []).append(round(n / GIB / dt, 2))
                    del tag
    # BytesIO (the caller's buffer, touched anonymous memory) both ways, 256 MiB windows
    import io
    os.environ.pop("HB_HOST_WINDOW_MIB", None)
    os.environ.pop("HB_HOST_AHEAD", None)
    bio = io.BytesIO(host.tobytes())
    for rep in range(5):
        for reg in (False, True):
            bio.seek(0)
            t = time.perf_counter()
            tag, _ = pys.encode_file(P, S, fk, ak, bio, register=reg)
            dt = time.perf_counter() - t
            assert tag._raw[:nb * 32] == ref.tobytes()
            res["api"].setdefault("bytesio_" + ("register" if reg else "pageable"), []).append(round(n / GIB / dt, 2))
            del tag
    del bio
    res["api_best"] = {k: max(v) for k, v in res["api"].items()}
    res["api_median"] = {k: sorted(v)[len(v) // 2] for k, v in res["api"].items()}
    # the caller-pinned raw rate on the same box (hb_host_register, not timed)
    tags = np.empty(nb * 32, dtype=np.uint8)
    ctx.check(L.hb_host_register(ctx.h, host.ctypes.data, n))
    ctx.check(L.hb_host_register(ctx.h, tags.ctypes.data, tags.nbytes))
    rates = []
    for _ in range(5):
        t = time.perf_counter()
        ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, host.ctypes.data, n, nb, tags.ctypes.data, 0, None))
        rates.append(round(n / GIB / (time.perf_counter() - t), 2))
    ctx.check(L.hb_host_unregister(ctx.h, tags.ctypes.data))
    ctx.check(L.hb_host_unregister(ctx.h, host.ctypes.data))
    res["raw_pinned"] = rates
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
