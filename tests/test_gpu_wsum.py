"""Consecutive weighted sums on ONE context: hb_wsum_kernel's
cross-workgroup protocol must leave its column counters, PRF slots, flag word
and result buffer ready for the next operation whatever that operation is
(hb_kernels.hpp, invariants I1-I4).  One context runs a sequence of proves
and verifies that alternates limb counts (256-bit NL = 8, 1024-bit NL = 32,
2048-bit NL = 64 -- the first 2048-bit sum grows the result buffer, the case
that exposed a broken variant in round 4), column counts (S + 1 = 2, 4, 11,
17; verify = 1), workgroups per column (1 to 40), empty and non-empty files,
device- and host-resident data (the host path's multi-batch accumulate
chain included), and every result is compared with the oracle.

Bar: bit-exact.  Reference: PySwizzle.py:333-370 (prove), 372-395 (verify).
"""
import ctypes
import hashlib

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _primes():
    pr = {k: int(v, 16) for k, v in load_golden("primes.json").items()}
    pos = load_golden("position_cases.json")
    pr["p2048"] = next(int(c["prime"], 16) for c in pos["cases"] if int(c["prime"], 16).bit_length() == 2048)
    return pr


def _ints(raw, w, n):
    return [int.from_bytes(raw[j * w:(j + 1) * w], "big") for j in range(n)]


# (prime, sectors, file bytes, challenge chunks, residency, host batch cap)
SEQUENCE = [
    ("p256", 16, 64 << 10, 3000, "device", None),
    ("p2048", 1, 0, 1, "host", None),           # round 4's failing shape: first 2048-bit sum
    ("p256", 3, 17, 6, "host", None),
    ("p2048", 1, 0, 1, "device", None),
    ("p2048", 2, 1545, 4, "host", None),
    ("p1024", 10, 5000, 777, "device", None),
    ("p256", 1, 0, 1, "device", None),
    ("p2048", 3, 40000, 10000, "device", None),  # 40 workgroups per column
    ("p256", 16, 1 << 20, 7777, "host", "2500"),  # 4 host batches: the accumulate chain
    ("p2048", 1, 300, 9, "host", "4"),           # 3 batches at 2048 bits
    ("p256", 16, 0, 2, "host", None),
    ("p1024", 3, 12345, 5000, "host", "1000"),
    ("p256", 16, 64 << 10, 3000, "device", None),
]


def test_alternating_proves_and_verifies_on_one_context(oracle, monkeypatch):
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    primes = _primes()
    rng = np.random.default_rng(2025)
    monkeypatch.setenv("HB_GATHER_THREADS", "4")
    bufs = []
    try:
        for k, (pname, S, n, chunks, where, batch) in enumerate(SEQUENCE):
            p = primes[pname]
            w = nat.width_of(p)
            C = (p.bit_length() // 8) * S
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            fk, ak = hashlib.sha256(b"ws-f%d" % k).digest(), hashlib.sha256(b"ws-a%d" % k).digest()
            tags = oracle.encode(p, S, fk, ak, data, nthreads=8)
            nb = len(tags)
            assert nb == n // C + 1
            traw = b"".join(t.to_bytes(w, "big") for t in tags)
            key = hashlib.sha256(b"ws-chal%d" % k).digest()
            pb = nat.be(p)
            if batch:
                monkeypatch.setenv("HB_TEST_PROVE_BATCH", batch)
            else:
                monkeypatch.delenv("HB_TEST_PROVE_BATCH", raising=False)
            if where == "device":
                dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
                ctx.check(L.hb_device_malloc(ctx.h, max(n, 16), ctypes.byref(dd)))
                bufs.append(dd)
                ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
                bufs.append(dt)
                if n:
                    hd = np.frombuffer(data, dtype=np.uint8)
                    ctx.check(L.hb_memcpy(ctx.h, dd, hd.ctypes.data, n, 1))
                ht = np.frombuffer(traw, dtype=np.uint8)
                ctx.check(L.hb_memcpy(ctx.h, dt, ht.ctypes.data, len(traw), 1))
                dptr, tptr, flags = dd, dt, 3
            else:
                dptr = ctypes.create_string_buffer(data, max(n, 1))
                tptr = ctypes.create_string_buffer(traw, len(traw))
                flags = 0
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), tptr, nb, dptr, n, flags,
                                 mu, sg))
            omu, osg = oracle.prove(p, S, key, chunks, p, tags, data)
            assert _ints(mu.raw, w, S) == omu, (k, pname, S, n, where)
            assert int.from_bytes(sg.raw, "big") == osg, (k, pname, S, n, where)
            if pname == "p2048" and n == 0:
                assert omu == [0]
            # a verify (one column) between proves
            rhs = ctypes.create_string_buffer(w)
            ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, 32, nb, key, 32, chunks, pb, len(pb),
                                      mu.raw, rhs))
            assert rhs.raw == sg.raw, (k, pname)
            assert oracle.verify(p, S, fk, ak, nb, key, chunks, p, omu, osg)
    finally:
        for b in bufs:
            ctx.check(L.hb_device_free(ctx.h, b))


@pytest.mark.parametrize("pname,S,n,chunks,misalign", [
    ("p256", 16, (8 << 20) + 77, 10000, 0),     # whole-block 16-byte gathers, ragged tail block
    ("p256", 16, (1 << 20) + 5, 3000, 3),       # misaligned file: the file sum (no gather)
    ("p255", 10, 123457, 2000, 0),              # 31-byte sectors, C = 310: the file sum (no gather)
    ("p2048", 3, 40000, 5000, 0),               # 2048-bit: C = 768, partial last block
    ("p256", 1, 0, 5, 0),                       # empty file: every sector past EOF
])
def test_device_gather_equals_file_sum(oracle, monkeypatch, pname, S, n, chunks, misalign):
    """A device-resident prove gathers each challenged block and tag in the
    PRF kernel (hb_gather_block: 16-byte copies for whole blocks, sector by
    sector for the ragged last block and past EOF) and sums the compact buffer;
    the same prove with the gather off (HB_NO_PROVE_GATHER, the sum reads the
    file directly) and the oracle agree.  Layouts the gather does not take
    (misaligned file, C = 310) run the file sum either way.
    Reference: PySwizzle.py:351-368."""
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p = _primes()[pname]
    w = nat.width_of(p)
    C = (p.bit_length() // 8) * S
    rng = np.random.default_rng(n + S)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    fk, ak = b"g" * 32, b"h" * 32
    tags = oracle.encode(p, S, fk, ak, data, nthreads=8)
    nb = len(tags)
    traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
    dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n + 64, ctypes.byref(dd)))
    ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
    try:
        dptr = dd.value + misalign
        if n:
            hd = np.frombuffer(data, dtype=np.uint8)
            ctx.check(L.hb_memcpy(ctx.h, dptr, hd.ctypes.data, n, 1))
        ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
        key = hashlib.sha256(b"gather%d" % n).digest()
        pb = nat.be(p)
        res = []
        for off in (False, True):
            if off:
                monkeypatch.setenv("HB_NO_PROVE_GATHER", "1")
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), dt, nb, dptr, n, 3, mu, sg))
            res.append((_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")))
        monkeypatch.delenv("HB_NO_PROVE_GATHER", raising=False)
        assert res[0] == res[1]
        assert res[0] == oracle.prove(p, S, key, chunks, p, tags, data)
    finally:
        ctx.check(L.hb_device_free(ctx.h, dd))
        ctx.check(L.hb_device_free(ctx.h, dt))
