#!/usr/bin/env python3
"""Where the API real-file encode loses time against the raw pinned rate
(bench.py host_path): mmap creation with and without MAP_POPULATE, page
faults of a fresh tag buffer, and hb_encode from each kind of source buffer
pageable vs HB_HOST_REGISTER.  4 GiB, S = 16, 256-bit prime.  Prints one JSON
line (seconds; GiB/s where it says so)."""
import ctypes
import hashlib
import json
import mmap
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from heartbeat_amd import _native  # noqa: E402

GIB = 1 << 30
P = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)


def main():
    L = _native.lib()
    ctx = _native.context()
    S, C = 16, 512
    n = 4 * GIB
    nb = n // C + 1
    pb = _native.be(P)
    fk, ak = hashlib.sha256(b"hb-bench-f").digest(), hashlib.sha256(b"hb-bench-alpha").digest()
    d = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(d)))
    ctx.check(L.hb_fill_random(ctx.h, d, n, 1234))
    host = np.empty(n, dtype=np.uint8)
    ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, d.value, n, 2))
    ref = np.empty(nb * 32, dtype=np.uint8)
    ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, d, n, nb, ref.ctypes.data, 1, None))
    ctx.check(L.hb_device_free(ctx.h, d))
    out = {}

    def enc(src_addr, tags, flags):
        t = time.perf_counter()
        ctx.check(L.hb_encode(ctx.h, pb, 32, S, fk, ak, 32, 0, src_addr, n, nb, tags.ctypes.data, flags, None))
        dt = time.perf_counter() - t
        assert np.array_equal(tags, ref)
        return dt

    warm = np.zeros(nb * 32, dtype=np.uint8)
    R = _native.HB_HOST_REGISTER
    enc(host.ctypes.data, warm, 0)
    out["anon_pageable_warm_tags"] = enc(host.ctypes.data, warm, 0)
    out["anon_register_warm_tags"] = enc(host.ctypes.data, warm, R)
    t = time.perf_counter()
    fresh = np.empty(nb * 32, dtype=np.uint8)
    out["np_empty_tags"] = time.perf_counter() - t
    out["anon_pageable_fresh_tags"] = enc(host.ctypes.data, fresh, 0)
    t = time.perf_counter()
    touch = np.empty(nb * 32, dtype=np.uint8)
    touch[::4096] = 0
    out["touch_fresh_tags_256mib"] = time.perf_counter() - t
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp")) as fh:
        host.tofile(fh.name)
        with open(fh.name, "rb") as f:
            fd = f.fileno()
            for populate in (True, False):
                for flags, name in ((0, "pageable"), (R, "register")):
                    t = time.perf_counter()
                    mflags = mmap.MAP_SHARED | (mmap.MAP_POPULATE if populate else 0)
                    mm = mmap.mmap(fd, 0, flags=mflags, prot=mmap.PROT_READ)
                    tm = time.perf_counter() - t
                    arr = np.frombuffer(mm, dtype=np.uint8)
                    key = "file_%s_%s" % ("populate" if populate else "lazy", name)
                    out[key + "_mmap_s"] = tm
                    out[key + "_encode_warm_tags_s"] = enc(arr.ctypes.data, warm, flags)
                    fresh = np.empty(nb * 32, dtype=np.uint8)
                    out[key + "_encode_fresh_tags_s"] = enc(arr.ctypes.data, fresh, flags)
                    del arr
                    mm.close()
        # the drop-in API on the same file, phase by phase (encode_file)
        import importlib
        from heartbeat_amd import multi
        from heartbeat_amd._filebuf import FileBuffer
        pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
        with open(fh.name, "rb") as f:
            for rep in range(3):
                for populate, reg in ((True, False), (False, False), (True, True), (False, True)):
                    ph = {}
                    t0 = time.perf_counter()
                    f.seek(0)
                    fb = FileBuffer(f, populate=populate)
                    t1 = time.perf_counter()
                    tags = np.empty(nb * 32, dtype=np.uint8)
                    multi.encode_shards(P, S, fk, ak, fb.addr, fb.len, nb, tags.ctypes.data,
                                        _native.HB_HOST_REGISTER if reg else 0, multi.devices())
                    t2 = time.perf_counter()
                    fb.consume()
                    fb.close()
                    t3 = time.perf_counter()
                    ph["filebuffer"] = t1 - t0
                    ph["encode_shards"] = t2 - t1
                    ph["consume_close"] = t3 - t2
                    ph["total_gib_s"] = n / GIB / (t3 - t0)
                    assert np.array_equal(tags, ref)
                    out["api_%s_%s_r%d" % ("populate" if populate else "lazy", "register" if reg else "pageable",
                                           rep)] = ph
    out = {k: v for k, v in out.items()}
    phases = {k: {a: round(b, 4) for a, b in v.items()} for k, v in out.items() if isinstance(v, dict)}
    out = {k: v for k, v in out.items() if not isinstance(v, dict)}
    rates = {k.replace("_s", "_gib_s") if k.endswith("_s") else k + "_gib_s": round(n / GIB / v, 2)
             for k, v in out.items() if "encode" in k or k.startswith("anon")}
    print(json.dumps({"seconds": {k: round(v, 4) for k, v in out.items()}, "rates": rates, "api_phases": phases}),
          flush=True)


if __name__ == "__main__":
    main()
