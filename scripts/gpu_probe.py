#!/usr/bin/env python3
"""Staged GPU probe: runs the C-ABI entry points from simplest to full,
printing (flushed) after each stage, so a fault or hang is localized.
Usage: python scripts/gpu_probe.py [stage ...]"""
import ctypes
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def log(*a):
    print("[probe %.1fs]" % (time.time() - T0), *a, flush=True)


T0 = time.time()


def main():
    import faulthandler
    faulthandler.dump_traceback_later(60, exit=True)
    stages = sys.argv[1:] or ["ctx", "fill", "prf_small", "prf_p256", "encode_small", "prove_small"]
    from heartbeat_amd import _native
    L = _native.lib()
    log("lib loaded")
    ctx = _native.context(0)
    log("ctx ok")
    from oracle import oracle as O
    p = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
    for st in stages:
        log("stage", st)
        if st == "fill":
            from conftest import splitmix_bytes
            n = 1 << 20
            d = ctypes.c_void_p()
            ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(d)))
            ctx.check(L.hb_fill_random(ctx.h, d, n, 42))
            buf = ctypes.create_string_buffer(n)
            ctx.check(L.hb_memcpy(ctx.h, buf, d, n, 2))
            ok = buf.raw == splitmix_bytes(42, 0, n)
            log("fill matches host splitmix:", ok)
            ctx.check(L.hb_device_free(ctx.h, d))
        elif st == "prf_small":
            from heartbeat_amd.util import KeyedPRF
            k = b"k" * 32
            got = KeyedPRF(k, 10000).eval_many([0, 1, 2])
            want = [O.prf_eval(k, 10000, x) for x in (0, 1, 2)]
            log("prf range 10000:", got, want, got == want)
        elif st == "prf_p256":
            from heartbeat_amd.util import KeyedPRF
            k = b"k" * 32
            xs = list(range(100))
            got = KeyedPRF(k, p).eval_many(xs)
            want = [O.prf_eval(k, p, x) for x in xs]
            log("prf range p256 match:", got == want)
        elif st == "encode_small":
            import importlib
            import io
            pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
            data = hashlib.sha256(b"x").digest() * 100
            tag, n = pys.encode_file(p, 16, b"f" * 32, b"a" * 32, io.BytesIO(data))
            want = O.encode(p, 16, b"f" * 32, b"a" * 32, data)
            log("encode small match:", tag.sigma == want, n)
        elif st == "prove_small":
            import io
            from heartbeat_amd.PySwizzle import Challenge, PySwizzle
            data = hashlib.sha256(b"y").digest() * 100
            beat = PySwizzle(16, b"s" * 32, p)
            tag, state = beat.encode(io.BytesIO(data))
            chal = Challenge(20, p, b"c" * 32)
            proof = beat.prove(io.BytesIO(data), chal, tag)
            mu, sg = O.prove(p, 16, b"c" * 32, 20, p, tag.sigma, data)
            log("prove small match:", proof.mu == mu and proof.sigma == sg)
            log("verify:", beat.verify(proof, chal, state))
        log("stage done", st)


if __name__ == "__main__":
    main()
