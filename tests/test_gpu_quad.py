"""GPU parity of the quad PRF engine (hb_kernels.hpp, hb_engine_quad: one
KeyedPRF evaluation per four lanes, DPP-gathered T-table rounds), which runs
every latency-bound KeyedPRF launch (challenges, alpha, batches of up to
num_cus * 256 inputs) against the lane engine (HB_NO_QUAD=1) and the CPU
oracle (pinned to the reference's KATs in tests/test_oracle.py).  The
1,537 reference KATs of test_gpu_parity.py::test_prf_kats already go through
the quad engine; this adds bulk inputs and the prove path."""
import ctypes
import hashlib
import os

import pytest

pytestmark = pytest.mark.gpu

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
P1024 = (1 << 1024) - 105   # odd 1024-bit range: no primality needed for the PRF


class _NoQuad:
    def __enter__(self):
        os.environ["HB_NO_QUAD"] = "1"

    def __exit__(self, *a):
        del os.environ["HB_NO_QUAD"]


@pytest.mark.parametrize("rng", [1, 2, 255, 257, (1 << 27) + 1, 10 ** 6, P256, (1 << 300) - 1, P1024])
@pytest.mark.parametrize("klen", [16, 32])
def test_quad_equals_lane_engine(rng, klen, oracle):
    from heartbeat_amd.util import KeyedPRF
    key = hashlib.sha256(b"quad-%d" % klen).digest()[:klen]
    xs = list(range(0, 3000)) + [2 ** 40 + 7, 2 ** 64 - 1]
    prf = KeyedPRF(key, rng)
    quad = prf.eval_many(xs)
    with _NoQuad():
        lane = prf.eval_many(xs)
    assert quad == lane
    for x in xs[:40] + xs[-2:]:
        assert quad[xs.index(x)] == oracle.prf_eval(key, rng, x)


def test_quad_prove_equals_lane_prove(oracle):
    """A 10,000-index prove (the quad engine runs both challenge PRFs) on a
    device-resident 32 MiB file == the lane-engine prove == the oracle."""
    from heartbeat_amd import _native as nat
    from test_gpu_parity import DevBuf, dev_encode, split_tags
    p, S = P256, 16
    L = 32 << 20
    nb = L // 512 + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 11))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tb.p)
        key = hashlib.sha256(b"quad-chal").digest()
        pb = nat.be(p)
        res = []
        for noquad in (False, True):
            mu = ctypes.create_string_buffer(32 * S)
            sg = ctypes.create_string_buffer(32)
            if noquad:
                os.environ["HB_NO_QUAD"] = "1"
            try:
                ctx.check(nat.lib().hb_prove(ctx.h, pb, 32, S, key, 32, 10000, pb, 32, tb.p, nb, buf.p, L, 3,
                                             mu, sg))
            finally:
                os.environ.pop("HB_NO_QUAD", None)
            res.append((mu.raw, sg.raw))
        assert res[0] == res[1]
        omu, osg = oracle.prove(p, S, key, 10000, p, split_tags(tb.download(), 32), buf.download())
        assert [int.from_bytes(res[0][0][j * 32:(j + 1) * 32], "big") for j in range(S)] == omu
        assert int.from_bytes(res[0][1], "big") == osg
    finally:
        buf.free()
        tb.free()


@pytest.mark.parametrize("prime_name,S,L,chunks", [("p256", 16, 8 << 20, 10000), ("p255", 5, 3 << 20, 3000),
                                                   ("p1024", 10, 4 << 20, 700), ("p61", 4, 1 << 20, 20000),
                                                   ("p256", 16, 1 << 20, 1)])
def test_quad_prove_ranges_vs_oracle(oracle, prime_name, S, L, chunks):
    """Device-resident proves on the quad engine == the lane engine
    (HB_NO_QUAD=1) == the oracle, for several primes / sector counts (aligned
    and byte-path sectors, 61- to 1024-bit), repeated on one context, and over
    index ranges (hb_prove_range, i0 != 0) whose partial sums add up mod p."""
    import json
    from heartbeat_amd import _native as nat
    from test_gpu_parity import DevBuf, dev_encode, split_tags
    primes = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))
    p = int(primes[prime_name], 16)
    w = (p.bit_length() + 7) // 8
    C = (p.bit_length() // 8) * S
    nb = L // C + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * w)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 31 + S))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tb.p)
        key = hashlib.sha256(b"fused-%d" % chunks).digest()
        pb = nat.be(p)

        def prove(i0, i1, lane=False):
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            if lane:
                os.environ["HB_NO_QUAD"] = "1"
            try:
                ctx.check(nat.lib().hb_prove_range(ctx.h, pb, len(pb), S, key, 32, chunks, i0, i1, pb, len(pb),
                                                   tb.p, nb, buf.p, L, 3, mu, sg))
            finally:
                os.environ.pop("HB_NO_QUAD", None)
            return mu.raw, sg.raw

        full = prove(0, chunks)
        assert full == prove(0, chunks, lane=True)
        assert full == prove(0, chunks)
        omu, osg = oracle.prove(p, S, key, chunks, p, split_tags(tb.download(), w), buf.download())
        assert [int.from_bytes(full[0][j * w:(j + 1) * w], "big") for j in range(S)] == omu
        assert int.from_bytes(full[1], "big") == osg
        if chunks > 2:
            cut = chunks // 3
            a, b = prove(0, cut), prove(cut, chunks)
            assert a == prove(0, cut, lane=True) and b == prove(cut, chunks, lane=True)
            mu = [(int.from_bytes(a[0][j * w:(j + 1) * w], "big") + int.from_bytes(b[0][j * w:(j + 1) * w], "big")) % p
                  for j in range(S)]
            assert mu == omu
    finally:
        buf.free()
        tb.free()
