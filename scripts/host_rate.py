"""Host-memory encode rate (PCIe-inclusive) per prime size: hb_encode on a
4 GiB host buffer (pageable and with HB_HOST_REGISTER windows) and the
PySwizzle encode_file API on a BytesIO, split into its phases.  Experiment
script (round 6): why the 1024-bit API row trails the 256-bit one."""
import ctypes
import hashlib
import io
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from heartbeat_amd import _native as nat   # noqa: E402
import bench                               # noqa: E402

GIB = 1 << 30
ctx = nat.context()
L = nat.lib()
pys = __import__("heartbeat_amd.PySwizzle.PySwizzle", fromlist=["encode_file"])
from heartbeat_amd import multi             # noqa: E402
from heartbeat_amd._filebuf import FileBuffer   # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
n0 = int(gib * GIB)
host = np.random.default_rng(1).integers(0, 256, n0, dtype=np.uint8)
fk, ak = hashlib.sha256(b"hr-f").digest(), hashlib.sha256(b"hr-a").digest()
REG = bench._native_flag("HB_HOST_REGISTER")
for bits, S in ((256, 16), (1024, 10)):
    p = bench.seeded_prime(bits)
    pb = nat.be(p)
    w = nat.width_of(p)
    C = (p.bit_length() // 8) * S
    n = n0 // C * C
    nb = n // C
    tags = np.empty(nb * w, dtype=np.uint8)
    ctx.prepare(p.bit_length())
    row = {"prime_bits": bits, "sectors": S, "gib": gib}
    for name, fl in (("raw_pageable", 0), ("raw_register", REG)):
        best = None
        for rep in range(3):
            t0 = time.perf_counter()
            ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, host.ctypes.data, n, nb,
                                  tags.ctypes.data, fl, None))
            dt = time.perf_counter() - t0
            if rep and (best is None or dt < best):
                best = dt
        row[name + "_gib_s"] = round(n / GIB / best, 2)
        row[name + "_kernel_ms"] = round(ctx.last_kernel_ms()[0], 2)
    bio = io.BytesIO(host[:n].tobytes())
    pys.encode_file(p, S, fk, ak, bio)
    best = None
    for rep in range(3):
        bio.seek(0)
        t0 = time.perf_counter()
        tag, _ = pys.encode_file(p, S, fk, ak, bio)
        dt = time.perf_counter() - t0
        del tag
        best = dt if best is None or dt < best else best
    row["api_bytesio_gib_s"] = round(n / GIB / best, 2)
    bio.seek(0)
    t0 = time.perf_counter()
    fb = FileBuffer(bio, populate=False)
    t1 = time.perf_counter()
    tags_out = np.empty((fb.len // C + 1) * w, dtype=np.uint8)
    multi.encode_shards(p, S, fk, ak, fb.addr, fb.len, fb.len // C + 1, tags_out.ctypes.data, REG, multi.devices())
    t2 = time.perf_counter()
    fb.consume()
    fb.close()
    t3 = time.perf_counter()
    row["api_phases_ms"] = {"filebuffer": round((t1 - t0) * 1e3, 2), "encode": round((t2 - t1) * 1e3, 2),
                            "close": round((t3 - t2) * 1e3, 2)}
    del bio
    print(json.dumps(row), flush=True)
