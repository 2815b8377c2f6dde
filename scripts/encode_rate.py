"""Device-resident encode rate at other prime sizes than the benchmarked
256-bit one (PySwizzle's default is 1024 bits, S = 10): fill, encode a few
times, report GiB/s of file bytes and the kernel times, and check 200
sampled blocks against the oracle.  Experiment script (round 5)."""
import ctypes
import hashlib
import json
import random
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from heartbeat_amd import _native as nat   # noqa: E402
from oracle import oracle as O            # noqa: E402


def prime(bits):
    if bits == 0:   # "P256": the benchmark's prime (tests/golden/primes.json, E[tries] 1.17)
        return int(json.load(open("tests/golden/primes.json"))["p256"], 16)
    pys = __import__("heartbeat_amd.PySwizzle.PySwizzle", fromlist=["_is_probable_prime"])
    rng = random.Random(5000 + bits)
    while True:
        x = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(x):
            return x


out = []
# bits:S:GiB[:cxx] -- ":cxx" encodes with the cxx Swizzle prf (HB_PRF_CXX;
# its oracle restatement is parity unpinned)
for bits, S, gib, cxx in [(0 if a[0] == "P256" else int(a[0]), int(a[1]), float(a[2]), a[3:] == ["cxx"])
                          for a in (x.split(":") for x in sys.argv[1:])]:
    p = prime(bits)
    w = nat.width_of(p)
    C = (p.bit_length() // 8) * S
    n = int(gib * (1 << 30))
    nb = n // C + 1
    ctx = nat.context()
    L = nat.lib()
    d, t = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(d)))
    ctx.check(L.hb_device_malloc(ctx.h, nb * w, ctypes.byref(t)))
    ctx.check(L.hb_fill_random(ctx.h, d, n, 99))
    fk, ak = hashlib.sha256(b"er-f").digest(), hashlib.sha256(b"er-a").digest()
    pb = nat.be(p)
    ctx.prepare(p.bit_length())
    best = None
    for rep in range(4):
        t0 = time.perf_counter()
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, d, n, nb, t, 3 | (nat.HB_PRF_CXX if cxx else 0),
                              None))
        dt = time.perf_counter() - t0
        kms = ctx.last_kernel_ms()[0]
        if rep and (best is None or dt < best[0]):
            best = (dt, kms, ctx.last_kernel_phases())
    rng = np.random.default_rng(p.bit_length())
    ok = True
    for b in sorted(set(rng.integers(0, nb, 200).tolist()) | {nb - 1}):
        m = min(C, max(0, n - b * C))
        blk = np.empty(max(m, 1), dtype=np.uint8)
        if m:
            ctx.check(L.hb_memcpy(ctx.h, blk.ctypes.data, d.value + b * C, m, 2))
        tg = np.empty(w, dtype=np.uint8)
        ctx.check(L.hb_memcpy(ctx.h, tg.ctypes.data, t.value + b * w, w, 2))
        want = (O.cxx_encode if cxx else O.encode)(p, S, fk, ak, blk.tobytes()[:m], block_base=b, nblocks=1)[0]
        ok = ok and int.from_bytes(tg.tobytes(), "big") == want
    ctx.check(L.hb_device_free(ctx.h, d))
    ctx.check(L.hb_device_free(ctx.h, t))
    out.append({"prime_bits": bits or "P256", "sectors": S, "gib": gib, "prf": "cxx" if cxx else "pyswizzle", "blocks": nb, "gib_s": round(n / (1 << 30) / best[0], 2),
                "wall_ms": round(best[0] * 1e3, 3), "kernel_ms": round(best[1], 3), "phases_ms": best[2], "sample_equal_oracle": ok})
    print(json.dumps(out[-1]), flush=True)
