"""Fused vs two-launch device prove on a list of shapes (round-5 bisect of a
fused-sum mismatch): prints, per shape, the launch counts and whether mu and
sigma equal the oracle's.  Experiment script."""
import ctypes
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from heartbeat_amd import _native as nat   # noqa: E402
from oracle import oracle                 # noqa: E402
from test_gpu_fused import _prime, _ints  # noqa: E402

os.environ["HB_ENABLE_TEST_SWITCHES"] = "1"
ctx = nat.context()
L = nat.lib()
for spec in sys.argv[1:]:
    bits, S, n, chunks = (int(x) for x in spec.split(":"))
    p = _prime(bits)
    w = nat.width_of(p)
    data = np.random.default_rng(bits + S).integers(0, 256, n, dtype=np.uint8).tobytes()
    tags = oracle.encode(p, S, b"f" * 32, b"a" * 32, data, nthreads=8)
    traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
    dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, max(n, 16), ctypes.byref(dd)))
    ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
    ctx.check(L.hb_memcpy(ctx.h, dd, np.frombuffer(data, dtype=np.uint8).ctypes.data, n, 1))
    ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
    key = hashlib.sha256(b"bisect").digest()
    want = oracle.prove(p, S, key, chunks, p, tags, data)
    pb = nat.be(p)
    row = {"spec": spec, "ss": p.bit_length() // 8, "tw": w}
    for off in (False, True):
        if off:
            os.environ["HB_NO_PROVE_FUSE"] = "1"
        else:
            os.environ.pop("HB_NO_PROVE_FUSE", None)
        mu = ctypes.create_string_buffer(w * S)
        sg = ctypes.create_string_buffer(w)
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), dt, len(tags), dd, n, 3, mu, sg))
        ms, nl = ctypes.c_double(), ctypes.c_uint32()
        ctx.check(L.hb_last_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(nl)))
        got_mu, got_sg = _ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")
        bad = [j for j in range(S) if got_mu[j] != want[0][j]]
        row["two" if off else "fused"] = {"launches": nl.value, "mu_bad_cols": bad, "sigma_ok": got_sg == want[1],
                                          "sigma_minus_want": hex((got_sg - want[1]) % p)[:24]}
    os.environ.pop("HB_NO_PROVE_FUSE", None)
    ctx.check(L.hb_device_free(ctx.h, dd))
    ctx.check(L.hb_device_free(ctx.h, dt))
    print(row, flush=True)
