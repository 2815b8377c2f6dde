"""The fused device prove (round 5, hb_kernels.hpp hb_prove_fused): one launch
in which each workgroup's index waves gather their challenged blocks into LDS,
its v waves store v R mod p there, and summer waves add the terms as both
halves arrive; the last workgroup finishes the sums.  Every case is proved
three times on one context -- fused, with HB_NO_PROVE_FUSE (PRF launch +
hb_wsum_kernel), and fused again -- and each must equal the oracle.  The launch count tells
which path ran (1 = fused): the cases cover the shapes the host admits (48
jobs per workgroup and one more, NL = 8, 16 and 32, 16-byte and byte-wise sector
and tag loads, 2 to 65 columns, empty and ragged files, repeated proves on
one context: the limb sums and counters re-zeroed by each launch's closer).

Bar: bit-exact.  Reference: PySwizzle.py:333-370 (prove)."""
import ctypes
import hashlib
import importlib
import random

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _prime(bits):
    if bits == 256:
        return int(load_golden("primes.json")["p256"], 16)
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(7000 + bits)
    while True:
        x = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(x):
            return x


def _ints(raw, w, n):
    return [int.from_bytes(raw[j * w:(j + 1) * w], "big") for j in range(n)]


# (prime bits, sectors, file bytes, challenge chunks, fused?)
CASES = [
    (256, 16, (16 << 20) + 77, 10000, True),     # configs[4]'s shape at 16 MiB, ragged tail block
    (256, 16, 8 << 20, 12288, True),             # 48 jobs in every workgroup (256 of them)
    (256, 16, 8 << 20, 12289, False),            # one more: the two-launch sum
    (256, 1, (1 << 20) + 5, 3000, True),         # two columns
    (256, 16, 0, 5, True),                       # empty file: every sector past EOF
    (256, 64, 1 << 20, 300, True),               # 65 columns, 3 summer lanes each
    (512, 3, 300000, 4000, True),                # NL = 16, 16-byte sector loads
    (384, 7, 250000, 2500, True),                # NL = 16, 48-byte sectors: byte-wise loads
    (128, 16, 100000, 1000, True),               # NL = 8, 16-byte sectors and tags: byte-wise loads
    (1024, 10, 1 << 20, 820, True),              # NL = 32, PySwizzle's defaults and default challenge
    (1020, 16, 200000, 2000, True),              # NL = 32, 127-byte sectors: byte-wise loads
    (1000, 2, 150000, 3000, False),              # NL = 32, 125-byte sectors and tags: host-layout gather
]


def test_fused_prove_equals_two_launch_sum_and_oracle(oracle, monkeypatch):
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    rng = np.random.default_rng(55)
    for k, (bits, S, n, chunks, fused) in enumerate(CASES):
        p = _prime(bits)
        w = nat.width_of(p)
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        fk, ak = hashlib.sha256(b"fz-f%d" % k).digest(), hashlib.sha256(b"fz-a%d" % k).digest()
        tags = oracle.encode(p, S, fk, ak, data, nthreads=8)
        nb = len(tags)
        traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
        dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
        ctx.check(L.hb_device_malloc(ctx.h, max(n, 16), ctypes.byref(dd)))
        ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
        try:
            if n:
                hd = np.frombuffer(data, dtype=np.uint8)
                ctx.check(L.hb_memcpy(ctx.h, dd, hd.ctypes.data, n, 1))
            ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
            pb = nat.be(p)
            want = oracle.prove(p, S, hashlib.sha256(b"fz-c%d" % k).digest(), chunks, p, tags, data)
            for off in (False, True, False):
                if off:
                    monkeypatch.setenv("HB_NO_PROVE_FUSE", "1")
                else:
                    monkeypatch.delenv("HB_NO_PROVE_FUSE", raising=False)
                key = hashlib.sha256(b"fz-c%d" % k).digest()
                mu = ctypes.create_string_buffer(w * S)
                sg = ctypes.create_string_buffer(w)
                ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), dt, nb, dd, n, 3, mu, sg))
                ms, nl = ctypes.c_double(), ctypes.c_uint32()
                ctx.check(L.hb_last_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(nl)))
                assert nl.value == (1 if fused and not off else 2), (bits, S, n, chunks, off, nl.value)
                got = (_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big"))
                assert got == want, (bits, S, n, chunks, "two-launch" if off else "fused")
        finally:
            monkeypatch.delenv("HB_NO_PROVE_FUSE", raising=False)
            ctx.check(L.hb_device_free(ctx.h, dd))
            ctx.check(L.hb_device_free(ctx.h, dt))


def test_fused_prove_ranges_sum_to_whole(oracle):
    """hb_prove_range halves (the multi-GPU split of a challenge) each run
    fused and add up mod p to the whole proof (PySwizzle.py:351-368)."""
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p = _prime(256)
    w = nat.width_of(p)
    S, n, chunks = 16, 4 << 20, 10000
    data = np.random.default_rng(9).integers(0, 256, n, dtype=np.uint8).tobytes()
    tags = oracle.encode(p, S, b"r" * 32, b"s" * 32, data, nthreads=8)
    traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
    dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(dd)))
    ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
    try:
        ctx.check(L.hb_memcpy(ctx.h, dd, np.frombuffer(data, dtype=np.uint8).ctypes.data, n, 1))
        ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
        pb, key = nat.be(p), hashlib.sha256(b"halves").digest()
        parts = []
        for i0, i1 in ((0, 4321), (4321, chunks)):
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            ctx.check(L.hb_prove_range(ctx.h, pb, len(pb), S, key, 32, chunks, i0, i1, pb, len(pb), dt, len(tags),
                                       dd, n, 3, mu, sg))
            parts.append((_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")))
        mu = [(a + b) % p for a, b in zip(parts[0][0], parts[1][0])]
        assert (mu, (parts[0][1] + parts[1][1]) % p) == oracle.prove(p, S, key, chunks, p, tags, data)
    finally:
        ctx.check(L.hb_device_free(ctx.h, dd))
        ctx.check(L.hb_device_free(ctx.h, dt))


def test_unplaced_queue_engine_prove_equals_oracle(oracle, monkeypatch):
    """With HB_NO_PROVE_PLACE the PRF waves race for the job queue (the
    pre-placement engine) and the sum takes its own launch: same proof."""
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p = _prime(256)
    w = nat.width_of(p)
    S, n, chunks = 16, 2 << 20, 10000
    data = np.random.default_rng(10).integers(0, 256, n, dtype=np.uint8).tobytes()
    tags = oracle.encode(p, S, b"q" * 32, b"u" * 32, data, nthreads=8)
    traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
    dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(dd)))
    ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
    monkeypatch.setenv("HB_NO_PROVE_PLACE", "1")
    try:
        ctx.check(L.hb_memcpy(ctx.h, dd, np.frombuffer(data, dtype=np.uint8).ctypes.data, n, 1))
        ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
        pb, key = nat.be(p), hashlib.sha256(b"queue").digest()
        mu = ctypes.create_string_buffer(w * S)
        sg = ctypes.create_string_buffer(w)
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), dt, len(tags), dd, n, 3, mu, sg))
        ms, nl = ctypes.c_double(), ctypes.c_uint32()
        ctx.check(L.hb_last_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(nl)))
        assert nl.value == 2
        assert (_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")) == oracle.prove(p, S, key, chunks, p, tags, data)
    finally:
        monkeypatch.delenv("HB_NO_PROVE_PLACE", raising=False)
        ctx.check(L.hb_device_free(ctx.h, dd))
        ctx.check(L.hb_device_free(ctx.h, dt))


# (prime bits, sectors, state chunks (blocks), challenge chunks, key bytes, fused?)
VERIFY_CASES = [
    (256, 16, 2 ** 27 + 1, 10000, 32, True),     # configs[4]'s index width and challenge
    (256, 16, 131073, 12288, 32, True),          # 48 jobs in every workgroup
    (256, 16, 131073, 12289, 32, False),         # one more: the launch sequence
    (256, 1, 5, 3, 32, True),                    # tiny: one workgroup pair, alpha of 1 sector
    (256, 100, 4000, 1000, 32, True),            # alpha over several workgroups (100 > 16)
    (512, 3, 9000, 4000, 16, True),              # NL = 16, AES-128 keys (NR = 10)
    (384, 7, 77777, 2500, 24, True),             # NL = 16, AES-192 keys (NR = 12)
    (1024, 4, 5000, 1000, 32, True),             # NL = 32
    (1024, 10, 820, 820, 32, True),              # NL = 32, PySwizzle's defaults (1 MiB file)
    (2048, 4, 5000, 1000, 32, False),            # NL = 64: the launch sequence
]


@pytest.mark.parametrize("bits,S,nchunks,chunks,klen,fused", VERIFY_CASES)
def test_fused_verify_equals_launch_sequence_and_oracle(oracle, monkeypatch, bits, S, nchunks, chunks, klen, fused):
    """PySwizzle.verify's right-hand side sum_i v_i F(idx_i) + sum_j alpha_j
    mu_j (PySwizzle.py:380-395) from one launch (hb_verify_fused_kernel) and
    from the launch sequence (HB_NO_VERIFY_FUSE) for an honest mu (the rhs
    the oracle's verify accepts) and a tampered one (rejected): equal
    bytes either way."""
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p = _prime(bits)
    w = nat.width_of(p)
    rng = random.Random(bits * 1000 + S)
    fk, ak = bytes(rng.getrandbits(8) for _ in range(klen)), bytes(rng.getrandbits(8) for _ in range(klen))
    key = bytes(rng.getrandbits(8) for _ in range(32 if klen == 32 else klen))
    mus = [rng.getrandbits(8 * w) % p for _ in range(S)]
    pb = nat.be(p)
    out = {}
    for off in (False, True):
        if off:
            monkeypatch.setenv("HB_NO_VERIFY_FUSE", "1")
        else:
            monkeypatch.delenv("HB_NO_VERIFY_FUSE", raising=False)
        for tamper in (0, 1):
            m = list(mus)
            m[0] = (m[0] + tamper) % p
            mub = b"".join(x.to_bytes(w, "big") for x in m)
            rhs = ctypes.create_string_buffer(w)
            ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, klen, nchunks, key, len(key), chunks, pb,
                                      len(pb), mub, rhs))
            ms, nl = ctypes.c_double(), ctypes.c_uint32()
            ctx.check(L.hb_last_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(nl)))
            assert nl.value == (1 if fused and not off else 0), (bits, S, chunks, off, nl.value)
            out[(off, tamper)] = (m, int.from_bytes(rhs.raw, "big"))
    monkeypatch.delenv("HB_NO_VERIFY_FUSE", raising=False)
    for tamper in (0, 1):
        assert out[(False, tamper)] == out[(True, tamper)], (bits, S, chunks, tamper)
        m, rhs = out[(False, tamper)]
        # the oracle's verify accepts exactly sigma = rhs
        assert oracle.verify(p, S, fk, ak, nchunks, key, chunks, p, m, rhs)
        assert not oracle.verify(p, S, fk, ak, nchunks, key, chunks, p, m, (rhs + 1) % p)


@pytest.mark.parametrize("bits,S,nbytes,chunks,uploaded", [
    (256, 16, 1 << 20, 2049, True),             # a 1 MiB file and its default challenge: uploaded, fused
    (1024, 10, 1 << 20, 820, True),             # PySwizzle's defaults: uploaded, fused (NL = 32)
    (256, 1, (5 << 20) + 3, 3000, True),        # under 8 MiB: uploaded
    (256, 16, 16 << 20, 10000, False),          # 16 MiB > 2 x 5.1 MB of challenged blocks: host gather
])
def test_host_prove_upload_equals_gather_and_oracle(oracle, monkeypatch, bits, S, nbytes, chunks, uploaded):
    """A prove of a host file small next to its challenge uploads the file
    and proves it device-resident; with HB_NO_PROVE_UPLOAD the challenged
    blocks are gathered on the host.  Both == the oracle, through the C ABI
    from host memory (PySwizzle.py:333-370)."""
    from heartbeat_amd import _native as nat
    ctx = nat.context()
    L = nat.lib()
    p = _prime(bits)
    w = nat.width_of(p)
    data = np.random.default_rng(bits + nbytes).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"up-f%d" % bits).digest(), hashlib.sha256(b"up-a%d" % bits).digest()
    tags = oracle.encode(p, S, fk, ak, data, nthreads=8)
    traw = b"".join(t.to_bytes(w, "big") for t in tags)
    key = hashlib.sha256(b"up-c%d" % nbytes).digest()
    want = oracle.prove(p, S, key, chunks, p, tags, data)
    pb = nat.be(p)
    dbuf = ctypes.create_string_buffer(data, max(nbytes, 1))
    tbuf = ctypes.create_string_buffer(traw, len(traw))
    launches = []
    try:
        for off in (False, True):
            if off:
                monkeypatch.setenv("HB_NO_PROVE_UPLOAD", "1")
            else:
                monkeypatch.delenv("HB_NO_PROVE_UPLOAD", raising=False)
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), tbuf, len(tags), dbuf, nbytes,
                                 0, mu, sg))
            ms, nl = ctypes.c_double(), ctypes.c_uint32()
            ctx.check(L.hb_last_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(nl)))
            launches.append(nl.value)
            assert (_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")) == want, (bits, S, nbytes, off)
    finally:
        monkeypatch.delenv("HB_NO_PROVE_UPLOAD", raising=False)
    if uploaded:
        assert launches[0] == 1      # the fused launch on the uploaded file


def test_concurrent_contexts_fused_proves_and_verifies(oracle):
    """Two contexts on one GPU (heartbeat_amd.multi's repeated-device
    instances), each driven by its own host thread, run fused proves and
    verifies at the same time: each context's counters, limb sums and result
    buffer are its own, and no fused launch waits on another workgroup, so
    the interleaving neither deadlocks nor mixes results.  All == the oracle."""
    import threading
    from heartbeat_amd import _native as nat
    L = nat.lib()
    p = _prime(256)
    w = nat.width_of(p)
    S, n, chunks = 16, 4 << 20, 10000
    data = np.random.default_rng(21).integers(0, 256, n, dtype=np.uint8).tobytes()
    fk, ak = b"x" * 32, b"y" * 32
    tags = oracle.encode(p, S, fk, ak, data, nthreads=8)
    traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
    pb = nat.be(p)
    keys = [hashlib.sha256(b"cc%d" % k).digest() for k in range(6)]
    want = {k: oracle.prove(p, S, key, chunks, p, tags, data) for k, key in enumerate(keys)}
    errors, got = [], {}

    def worker(inst, ks):
        try:
            ctx = nat.context(0, inst)
            dd, dt = ctypes.c_void_p(), ctypes.c_void_p()
            ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(dd)))
            ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
            try:
                ctx.check(L.hb_memcpy(ctx.h, dd, np.frombuffer(data, dtype=np.uint8).ctypes.data, n, 1))
                ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
                for rep in range(5):
                    for k in ks:
                        mu = ctypes.create_string_buffer(w * S)
                        sg = ctypes.create_string_buffer(w)
                        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, keys[k], 32, chunks, pb, len(pb), dt, len(tags),
                                             dd, n, 3, mu, sg))
                        rhs = ctypes.create_string_buffer(w)
                        ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, 32, len(tags), keys[k], 32, chunks,
                                                  pb, len(pb), mu.raw, rhs))
                        got[(inst, rep, k)] = (_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big"),
                                               rhs.raw == sg.raw)
            finally:
                ctx.check(L.hb_device_free(ctx.h, dd))
                ctx.check(L.hb_device_free(ctx.h, dt))
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(i + 1, [0, 1, 2] if i == 0 else [3, 4, 5])) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not errors, errors
    assert len(got) == 2 * 5 * 3
    for (inst, rep, k), (mu, sg, ok) in got.items():
        assert (mu, sg) == want[k] and ok, (inst, rep, k)


def test_fused_sums_after_limb_buffer_growth(oracle):
    """On a fresh context, fused proves whose column counts (and limb widths)
    keep growing the limb-sum buffer, each followed by a fused verify: the
    grown buffer must start at zero wherever the allocator places it (a
    reallocation at the same address once left a stale tail there and a wrong
    sigma).  Each proof == the oracle, each verify accepts it."""
    from heartbeat_amd import _native as nat
    ctx = nat.context(0, 3)
    L = nat.lib()
    rng = np.random.default_rng(77)
    n = 1 << 19
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    dd = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(dd)))
    try:
        ctx.check(L.hb_memcpy(ctx.h, dd, np.frombuffer(data, dtype=np.uint8).ctypes.data, n, 1))
        for k, (bits, S) in enumerate([(256, 1), (256, 2), (256, 5), (1024, 4), (256, 16), (1024, 10), (256, 40),
                                       (256, 64)]):
            p = _prime(bits)
            w = nat.width_of(p)
            fk, ak = hashlib.sha256(b"gr-f%d" % k).digest(), hashlib.sha256(b"gr-a%d" % k).digest()
            tags = oracle.encode(p, S, fk, ak, data, nthreads=8)
            traw = np.frombuffer(b"".join(t.to_bytes(w, "big") for t in tags), dtype=np.uint8)
            dt = ctypes.c_void_p()
            ctx.check(L.hb_device_malloc(ctx.h, len(traw), ctypes.byref(dt)))
            try:
                ctx.check(L.hb_memcpy(ctx.h, dt, traw.ctypes.data, len(traw), 1))
                pb, key = nat.be(p), hashlib.sha256(b"gr-c%d" % k).digest()
                chunks = min(len(tags), 2000)
                mu = ctypes.create_string_buffer(w * S)
                sg = ctypes.create_string_buffer(w)
                ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), dt, len(tags), dd, n, 3,
                                     mu, sg))
                ms, nl = ctypes.c_double(), ctypes.c_uint32()
                ctx.check(L.hb_last_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(nl)))
                assert nl.value == 1, (bits, S, nl.value)
                assert (_ints(mu.raw, w, S), int.from_bytes(sg.raw, "big")) == \
                    oracle.prove(p, S, key, chunks, p, tags, data), (bits, S)
                rhs = ctypes.create_string_buffer(w)
                ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, 32, len(tags), key, 32, chunks, pb, len(pb),
                                          mu.raw, rhs))
                assert rhs.raw == sg.raw, (bits, S)
            finally:
                ctx.check(L.hb_device_free(ctx.h, dt))
    finally:
        ctx.check(L.hb_device_free(ctx.h, dd))
