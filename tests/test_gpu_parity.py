"""GPU parity: the HIP path (libhbswizzle.so, through its C ABI) against the
reference's golden vectors and the CPU oracle.

Bar: bit-exact tags / proofs.  Sizes: golden fixtures (every edge case the
reference's semantics have: empty file, 1 byte, ss-1, ss, ss+1, C-1, C, C+1,
3C+17, primes of 20/61/255/256/1024 bits, sectors 1/3/10/16, 16/24/32-byte
PRF keys), the reference's own files (test.txt, test3.txt, regenerated
test6.txt), then 64 MiB device-resident random files compared block for block
with the oracle, plus size-independent properties (shards concatenate, host
path == device path, prove/verify round trips and tamper detection).
"""
import ctypes
import hashlib
import importlib
import io
import json
import os

import numpy as np
import pytest

from conftest import fixture_file, splitmix_bytes

pytestmark = pytest.mark.gpu

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)


@pytest.fixture(scope="module")
def nat():
    from heartbeat_amd import _native
    _native.context()
    return _native


@pytest.fixture(scope="module")
def pys():
    return importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")


class DevBuf(object):
    def __init__(self, nat, n):
        self.nat = nat
        self.ctx = nat.context()
        p = ctypes.c_void_p()
        self.ctx.check(nat.lib().hb_device_malloc(self.ctx.h, n, ctypes.byref(p)))
        self.p = p.value
        self.n = n

    def upload(self, data, off=0):
        a = np.frombuffer(data, dtype=np.uint8)
        if len(a):
            self.ctx.check(self.nat.lib().hb_memcpy(self.ctx.h, self.p + off, a.ctypes.data, len(a), 1))

    def download(self, n=None, off=0):
        n = self.n - off if n is None else n
        out = np.empty(n, dtype=np.uint8)
        if n:
            self.ctx.check(self.nat.lib().hb_memcpy(self.ctx.h, out.ctypes.data, self.p + off, n, 2))
        return out.tobytes()

    def free(self):
        self.ctx.check(self.nat.lib().hb_device_free(self.ctx.h, self.p))


def dev_encode(nat, p, S, fk, ak, dptr, length, nblocks, tags_ptr, block_base=0):
    ctx = nat.context()
    pb = nat.be(p)
    tries = ctypes.c_uint64()
    ctx.check(nat.lib().hb_encode(ctx.h, pb, len(pb), S, fk, ak, len(fk), block_base, dptr, length,
                                  nblocks, tags_ptr, 3, ctypes.byref(tries)))
    return tries.value


def split_tags(raw, w):
    return [int.from_bytes(raw[i:i + w], "big") for i in range(0, len(raw), w)]


# ------------------------------------------------------------------ golden
def test_prf_kats(golden_prf):
    from heartbeat_amd.PySwizzle import KeyedPRF
    for c in golden_prf["cases"]:
        f = KeyedPRF(bytes.fromhex(c["key"]), int(c["range"]))
        assert f.eval_many([int(x) for x in c["xs"]]) == [int(o) for o in c["outs"]], c["range"]


def test_encode_golden_host_path(golden_encode, pys):
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        tag, n = pys.encode_file(p, c["sectors"], bytes.fromhex(c["f_key"]),
                                 bytes.fromhex(c["alpha_key"]), io.BytesIO(bytes.fromhex(c["data"])))
        assert n == c["ntags"]
        assert tag.sigma == [int(t, 16) for t in c["tags"]], c["name"]


@pytest.mark.parametrize("engine", ["small", "two_pass"])
@pytest.mark.parametrize("misalign", [0, 1])
def test_encode_golden_device_path(golden_encode, nat, misalign, engine, monkeypatch):
    """Every golden case through the C ABI from device memory, on the
    small-input path (placed quad PRF + hb_mac_kernel, the default for these
    sizes) and on the two-pass engine (HB_NO_SMALL_ENCODE)."""
    if engine == "two_pass":
        monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        w = nat.width_of(p)
        data = bytes.fromhex(c["data"])
        nt = c["ntags"]
        buf = DevBuf(nat, len(data) + 16)
        tb = DevBuf(nat, nt * w)
        try:
            buf.upload(data, misalign)
            dev_encode(nat, p, c["sectors"], bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]),
                       buf.p + misalign, len(data), nt, tb.p)
            assert split_tags(tb.download(), w) == [int(t, 16) for t in c["tags"]], c["name"]
        finally:
            buf.free()
            tb.free()


def test_prove_verify_golden(golden_encode):
    from heartbeat_amd.PySwizzle import Challenge, PySwizzle, State, Tag
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        beat = PySwizzle(c["sectors"], bytes.fromhex(c["state_key"]), p)
        tag = Tag.fromdict({"sigma": [int(t, 16) for t in c["tags"]]})
        data = bytes.fromhex(c["data"])
        for chn, prn in (("chal", "proof"), ("chal2", "proof2")):
            ch = c[chn]
            chal = Challenge(ch["chunks"], int(ch["v_max"], 16), bytes.fromhex(ch["key"]))
            proof = beat.get_public().prove(io.BytesIO(data), chal, tag)
            assert proof.mu == [int(m, 16) for m in c[prn]["mu"]], c["name"]
            assert proof.sigma == int(c[prn]["sigma"], 16), c["name"]
            state = State.fromdict(c["state"])
            assert beat.verify(proof, chal, state)
        # tampered file: same verdict as the reference
        if c["tamper_byte"] is not None:
            bad = bytearray(data)
            bad[c["tamper_byte"]] ^= 1
            ch = c["chal"]
            chal = Challenge(ch["chunks"], int(ch["v_max"], 16), bytes.fromhex(ch["key"]))
            proof = beat.prove(io.BytesIO(bytes(bad)), chal, tag)
            assert beat.verify(proof, chal, State.fromdict(c["state"])) == c["tamper_verifies"]


def test_encode_with_reference_keys_end_to_end(golden_encode, pys, monkeypatch):
    """PySwizzle.encode drawing the reference's keys reproduces tag AND state."""
    from heartbeat_amd.PySwizzle import PySwizzle
    for c in golden_encode["cases"][::9]:
        queue = [bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]), bytes.fromhex(c["state_iv"])]
        monkeypatch.setattr(pys, "_random_bytes", lambda n: queue.pop(0))
        beat = PySwizzle(c["sectors"], bytes.fromhex(c["state_key"]), int(c["prime"], 16))
        f = io.BytesIO(bytes.fromhex(c["data"]))
        tag, state = beat.encode(f)
        assert f.tell() == c["len"]
        assert tag.todict() == {"sigma": [int(t, 16) for t in c["tags"]]}
        assert state.todict() == c["state"]


def test_reference_files(golden_files, pys):
    from heartbeat_amd.PySwizzle import Challenge, PySwizzle, Tag
    for c in golden_files["cases"]:
        p = int(c["prime"], 16)
        data = fixture_file(c["file"])
        w = (p.bit_length() + 7) // 8
        tag, n = pys.encode_file(p, c["sectors"], bytes.fromhex(c["f_key"]),
                                 bytes.fromhex(c["alpha_key"]), io.BytesIO(data))
        assert n == c["ntags"]
        assert hashlib.sha256(tag.raw(p)).hexdigest() == c["tags_sha256"], c["name"]
        ch = c["chal"]
        beat = PySwizzle(c["sectors"], b"k" * 32, p)
        proof = beat.prove(io.BytesIO(data), Challenge(ch["chunks"], int(ch["v_max"], 16),
                                                       bytes.fromhex(ch["key"])), tag)
        assert proof.sigma == int(c["proof"]["sigma"], 16)
        assert proof.mu == [int(m, 16) for m in c["proof"]["mu"]]


def test_real_file_via_mmap(tmp_path, pys, oracle):
    data = fixture_file("test6.txt")
    fn = tmp_path / "t6.bin"
    fn.write_bytes(data)
    with open(fn, "rb") as f:
        f.read(1000)  # encode starts at the current position, like file.read()
        tag, n = pys.encode_file(P256, 16, b"f" * 32, b"a" * 32, f)
        assert f.tell() == len(data)
    assert tag.sigma == oracle.encode(P256, 16, b"f" * 32, b"a" * 32, data[1000:])


# ------------------------------------------------------------------ reference test flows
def test_generic_correctness():
    """tests/GenericCorrectnessTests.py:5-17 of the reference."""
    from heartbeat_amd.PySwizzle import PySwizzle
    priv = PySwizzle(primebits=256)
    pub = priv.get_public()
    d1, d3 = fixture_file("test.txt"), fixture_file("test3.txt")
    tag, state = priv.encode(io.BytesIO(d1))
    chal = priv.gen_challenge(state)
    assert priv.verify(pub.prove(io.BytesIO(d1), chal, tag), chal, state)
    assert not priv.verify(pub.prove(io.BytesIO(d3), chal, tag), chal, state)


def test_repeated_challenge():
    """GenericCorrectnessTests.py:20-31."""
    from heartbeat_amd.PySwizzle import PySwizzle
    priv = PySwizzle()
    pub = priv.get_public()
    d1 = fixture_file("test.txt")
    tag, state = priv.encode(io.BytesIO(d1))
    chal1 = priv.gen_challenge(state)
    proof1 = pub.prove(io.BytesIO(d1), chal1, tag)
    assert priv.verify(proof1, chal1, state)
    chal2 = priv.gen_challenge(state)
    assert not priv.verify(proof1, chal2, state)


def test_scheme_json_rounds():
    """GenericCorrectnessTests.py:34-116: client/server over JSON, 20 rounds."""
    from heartbeat_amd.PySwizzle import PySwizzle
    hb = PySwizzle
    client = hb()
    server = hb.fromdict(json.loads(json.dumps(client.get_public().todict())))
    data = fixture_file("test.txt")
    tag, state = client.encode(io.BytesIO(data))
    msg = json.loads(json.dumps({"tag": tag.todict(), "state": state.todict()}))
    serv_tag = hb.tag_type().fromdict(msg["tag"])
    serv_state = hb.state_type().fromdict(msg["state"])
    for _ in range(20):
        st = hb.state_type().fromdict(json.loads(json.dumps(serv_state.todict())))
        chal = client.gen_challenge(st)
        msg = json.loads(json.dumps({"challenge": chal.todict(), "state": st.todict()}))
        serv_chal = hb.challenge_type().fromdict(msg["challenge"])
        serv_state = hb.state_type().fromdict(msg["state"])
        proof = server.prove(io.BytesIO(data), serv_chal, serv_tag)
        proof = hb.proof_type().fromdict(json.loads(json.dumps(proof.todict())))
        assert client.verify(proof, chal, st)


def test_sectors_short_file():
    """tests_unit_pyswpriv.py:89-101: a 10-byte file with 10 sectors."""
    from heartbeat_amd.PySwizzle import PySwizzle
    memfile = io.BytesIO(os.urandom(10))
    beat = PySwizzle(10)
    tag, state = beat.encode(memfile)
    chal = beat.gen_challenge(state)
    memfile.seek(0)
    proof = beat.prove(memfile, chal, tag)
    assert beat.verify(proof, chal, state)


def test_keyedprf_consistency():
    from heartbeat_amd.PySwizzle import KeyedPRF
    k = os.urandom(32)
    f1, f2 = KeyedPRF(k, 10000), KeyedPRF(k, 10000)
    assert [f1.eval(i) for i in range(20)] == f2.eval_many(range(20))
    assert all(0 <= v < 10000 for v in f1.eval_many(range(5000)))


# ------------------------------------------------------------------ at scale
@pytest.mark.parametrize("S,prime_name", [(16, "p256"), (1, "p256"), (5, "p255")])
def test_device_resident_64mib_vs_oracle(nat, oracle, S, prime_name):
    primes = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))
    p = int(primes[prime_name], 16)
    w = nat.width_of(p)
    L = 64 << 20
    C = (p.bit_length() // 8) * S
    nb = L // C + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * w)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 12345))
        fk, ak = hashlib.sha256(b"hb-bench-f").digest(), hashlib.sha256(b"hb-bench-alpha").digest()
        tries = dev_encode(nat, p, S, fk, ak, buf.p, L, nb, tb.p)
        data = buf.download()
        assert data[:4096] == splitmix_bytes(12345, 0, 4096)
        got = tb.download()
        want = oracle.encode(p, S, fk, ak, data, nthreads=16)
        assert split_tags(got, w) == want
        # mean tries per F value ~ 2^bitlen/p
        assert nb <= tries < nb * (2.0 ** p.bit_length() / p) * 1.1 + 64
    finally:
        buf.free()
        tb.free()


@pytest.mark.parametrize("prime_name", ["p256", "p256max", "p256lo"])
@pytest.mark.parametrize("S", [4, 6, 17, 20, 36])
def test_mfma_mac_sector_counts_vs_oracle(nat, oracle, S, prime_name, monkeypatch):
    """The first pass's MFMA MAC (hb_mfma_block_acc, dense digit tiles from
    mfma_tables) at the sector counts the 64 MiB test does not reach: S = 4
    (the smallest MFMA case), 6 and 17 (sector-shaped loads, S % 4 != 0),
    20 and 36 (whole-line loads), 17 / 20 / 36 with the A fragments read from
    global memory instead of LDS (S > 16); primes with p just above 2^255
    (p256lo, half the first tries rejected) and just below 2^256 (p256max: the
    digit representatives r - p at the edge of their range).  A ragged 2 MiB
    device-resident file, block_base != 0; every tag == the oracle."""
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")   # the two-pass engine at this size
    primes = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))
    p = int(primes[prime_name], 16)
    L = (2 << 20) + 777
    C = 32 * S
    nb = L // C + 1
    base = 123456789
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 1000 + S))
        fk, ak = hashlib.sha256(b"mf-f%d" % S).digest(), hashlib.sha256(b"mf-a" + prime_name.encode()).digest()
        dev_encode(nat, p, S, fk, ak, buf.p, L, nb, tb.p, block_base=base)
        want = oracle.encode(p, S, fk, ak, buf.download(), block_base=base, nthreads=16)
        assert split_tags(tb.download(), 32) == want
    finally:
        buf.free()
        tb.free()


@pytest.mark.parametrize("switch,S", [("HB_MFMA_LINE32", 20), ("HB_MFMA_LINE32", 36),
                                      ("HB_MFMA_SECTOR_LOADS", 4), ("HB_MFMA_SECTOR_LOADS", 20)])
def test_mfma_selectable_layouts_vs_oracle(nat, oracle, monkeypatch, switch, S):
    """The MAC layouts the shipped build can still select by switch (ADVICE
    r4): HB_MFMA_LINE32 -- the 32x32x32 MFMA with whole-line loads and the
    in-quad DPP transpose (mfma_tables layout 2, S % 4 == 0) -- and
    HB_MFMA_SECTOR_LOADS -- the 32x32x32 MFMA with sector-shaped loads (layout
    1, here at even S, which the default build gives the 16x16x64 MAC).
    Primes just below 2^256 (digit representatives at the edge of their range)
    and p256; a ragged 2 MiB device-resident file; every tag == the oracle."""
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")   # the two-pass engine at this size
    primes = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))
    monkeypatch.setenv(switch, "1")
    L = (2 << 20) + 333
    C = 32 * S
    nb = L // C + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        assert nat.lib().hb_test_switches() != 0, "the test-switch gate is closed (tests/conftest.py)"
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 2000 + S))
        data = buf.download()
        for prime_name in ("p256max", "p256"):
            p = int(primes[prime_name], 16)
            fk, ak = hashlib.sha256(b"lay-f%d" % S).digest(), hashlib.sha256(b"lay-a" + switch.encode()).digest()
            dev_encode(nat, p, S, fk, ak, buf.p, L, nb, tb.p, block_base=77777)
            want = oracle.encode(p, S, fk, ak, data, block_base=77777, nthreads=16)
            assert split_tags(tb.download(), 32) == want, prime_name
    finally:
        buf.free()
        tb.free()


@pytest.mark.parametrize("S,prime_name", [(16, "p256"), (1, "p256"), (5, "p255"), (16, "p256lo"),
                                          (3, "p1024"), (4, "p61")])
def test_two_pass_equals_single_pass(nat, S, prime_name, monkeypatch):
    """The two-pass encode (prefix image first pass + retry list, forced with
    HB_NO_SMALL_ENCODE where the input is small) == the single-pass engine
    (HB_ENCODE_SINGLE_PASS) == the small-input path (placed quad PRF +
    hb_mac_kernel, the default below 65,537 blocks), 16 MiB device-resident;
    p256lo (2^255 < p) rejects half the first tries."""
    primes = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))
    p = int(primes[prime_name], 16)
    w = nat.width_of(p)
    L = (16 << 20) + 1000
    C = (p.bit_length() // 8) * S
    nb = L // C + 1
    buf = DevBuf(nat, L)
    t1 = DevBuf(nat, nb * w)
    t2 = DevBuf(nat, nb * w)
    t3 = DevBuf(nat, nb * w)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 4242))
        fk, ak = hashlib.sha256(b"tp-f").digest(), hashlib.sha256(b"tp-a").digest()
        pb = nat.be(p)
        tries = []
        for flags, tb, two_pass in ((3, t1, True), (3 | nat.HB_ENCODE_SINGLE_PASS, t2, False), (3, t3, False)):
            if two_pass:
                monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
            else:
                monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
            tr = ctypes.c_uint64()
            ctx.check(nat.lib().hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, buf.p, L, nb, tb.p,
                                          flags, ctypes.byref(tr)))
            tries.append(tr.value)
        assert t1.download() == t2.download() == t3.download()
        # same PRF streams: the same number of tries either way
        assert tries[0] == tries[1] == tries[2]
    finally:
        buf.free()
        t1.free()
        t2.free()
        t3.free()


def test_two_pass_retry_list_overflow(nat, monkeypatch):
    """A retry list too small for the rejected first tries: the first pass
    finishes the overflow in place, tags unchanged."""
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")   # the two-pass engine at this size
    p = int(json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))["p256lo"], 16)
    S, L = 4, 4 << 20
    nb = L // (32 * S) + 1
    buf = DevBuf(nat, L)
    t1 = DevBuf(nat, nb * 32)
    t2 = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 77))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, t1.p)
        monkeypatch.setenv("HB_TEST_RETRY_CAP", "1000")
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, t2.p)
        assert t1.download() == t2.download()
    finally:
        buf.free()
        t1.free()
        t2.free()


def test_retry_list_late_entries(nat, oracle, monkeypatch):
    """Retry-list entries without a stored digest (listed after the first try,
    flags 0: the first output word equal to R's top word, ~2^-32 of the
    rejections, forced for all of them by HB_TEST_NO_EARLY_LIST) are hashed by
    the retry pass: tags == the default path (early entries with digests) ==
    the oracle, with a full and an overflowing retry list."""
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")   # the two-pass engine at this size
    p = int(json.load(open(os.path.join(os.path.dirname(__file__), "golden", "primes.json")))["p256"], 16)
    S, L = 16, 6 << 20
    nb = L // (32 * S) + 1
    buf = DevBuf(nat, L)
    tags = [DevBuf(nat, nb * 32) for _ in range(3)]
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 91))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tags[0].p, block_base=987654321)
        monkeypatch.setenv("HB_TEST_NO_EARLY_LIST", "1")
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tags[1].p, block_base=987654321)
        monkeypatch.setenv("HB_TEST_RETRY_CAP", "500")
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tags[2].p, block_base=987654321)
        t0 = tags[0].download()
        assert tags[1].download() == t0
        assert tags[2].download() == t0
        data = buf.download()
        want = oracle.encode(p, S, b"f" * 32, b"a" * 32, data, block_base=987654321, nblocks=600)
        assert split_tags(t0[: 600 * 32], 32) == want
    finally:
        buf.free()
        for t in tags:
            t.free()


def test_shards_concatenate(nat):
    """Block-range shards with awkward boundaries == one whole-file launch."""
    p, S = P256, 16
    w, C = 32, 512
    L = 8 * 1000 * C + 123
    nb = L // C + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * w)
    ts = DevBuf(nat, nb * w)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 7))
        fk, ak = b"F" * 32, b"A" * 32
        dev_encode(nat, p, S, fk, ak, buf.p, L, nb, tb.p)
        cuts = [0, 1, 2999, 5001, nb]
        for a, b in zip(cuts[:-1], cuts[1:]):
            last = b == nb
            dlen = (L - a * C) if last else (b - a) * C
            dev_encode(nat, p, S, fk, ak, buf.p + a * C, dlen, b - a, ts.p + a * w, block_base=a)
        assert tb.download() == ts.download()
    finally:
        buf.free()
        tb.free()
        ts.free()


def test_host_path_chunks_equal_device_path(nat, pys):
    """> 256 MiB from host memory (chunked, double-buffered H2D) == device-resident."""
    p, S = P256, 16
    L = (600 << 20) + 77
    nb = L // 512 + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 99))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tb.p)
        host = buf.download()
        tag, n = pys.encode_file(p, S, b"f" * 32, b"a" * 32, io.BytesIO(host))
        assert n == nb
        assert tag.raw(p) == tb.download()
    finally:
        buf.free()
        tb.free()


def test_host_path_pinned_equals_device_path(nat):
    """Pinned (hb_host_register) host file and tag buffers, S = 1 so that the
    per-chunk tag D2H is as large as the H2D: == device-resident tags."""
    p, S = P256, 1
    L = (300 << 20) + 5
    nb = L // 32 + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    ctx = nat.context()
    lib = nat.lib()
    try:
        ctx.check(lib.hb_fill_random(ctx.h, buf.p, L, 7))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tb.p)
        host = np.frombuffer(buf.download(), dtype=np.uint8).copy()
        tags = np.zeros(nb * 32, dtype=np.uint8)
        ctx.check(lib.hb_host_register(ctx.h, host.ctypes.data, host.nbytes))
        ctx.check(lib.hb_host_register(ctx.h, tags.ctypes.data, tags.nbytes))
        try:
            pb = nat.be(p)
            ctx.check(lib.hb_encode(ctx.h, pb, len(pb), S, b"f" * 32, b"a" * 32, 32, 0,
                                    host.ctypes.data, L, nb, tags.ctypes.data, 0, None))
        finally:
            ctx.check(lib.hb_host_unregister(ctx.h, tags.ctypes.data))
            ctx.check(lib.hb_host_unregister(ctx.h, host.ctypes.data))
        assert tags.tobytes() == tb.download()
    finally:
        buf.free()
        tb.free()


def test_prove_device_resident_vs_oracle(nat, oracle):
    """Config-5 shape at 64 MiB: 10 000-index challenge, device-resident file and tags."""
    p, S = P256, 16
    L = 64 << 20
    nb = L // 512 + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 5))
        fk, ak = b"f" * 32, b"a" * 32
        dev_encode(nat, p, S, fk, ak, buf.p, L, nb, tb.p)
        key = hashlib.sha256(b"hb-bench-chal").digest()
        mu = ctypes.create_string_buffer(32 * S)
        sg = ctypes.create_string_buffer(32)
        pb = nat.be(p)
        ctx.check(nat.lib().hb_prove(ctx.h, pb, 32, S, key, 32, 10000, pb, 32, tb.p, nb, buf.p, L, 3,
                                     mu, sg))
        tags = split_tags(tb.download(), 32)
        data = buf.download()
        omu, osg = oracle.prove(p, S, key, 10000, p, tags, data)
        assert [int.from_bytes(mu.raw[j * 32:(j + 1) * 32], "big") for j in range(S)] == omu
        assert int.from_bytes(sg.raw, "big") == osg
        # verify through the API path (host), and a tampered block is caught
        rhs = ctypes.create_string_buffer(32)
        ctx.check(nat.lib().hb_verify_rhs(ctx.h, pb, 32, S, fk, ak, 32, nb, key, 32, 10000, pb, 32,
                                          mu.raw, rhs))
        assert rhs.raw == sg.raw
    finally:
        buf.free()
        tb.free()


def test_device_resident_4_5gib_sampled_vs_oracle(nat, oracle):
    """PySwizzle mode past 2^32 bytes: a 4.5 GiB + 333-byte device-resident
    file (ragged tail), S = 16, 256-bit prime.  Tags of the first and last
    1,000 blocks (tail included) and 10,000 random blocks == the oracle on the
    same bytes (regenerated on the host from the SplitMix64 stream, with
    block_base); then a 2,000-index prove over the whole file (challenged
    offsets past 4 GiB) == the oracle's prove on the downloaded file."""
    p, S, C, w = P256, 16, 512, 32
    L = (9 << 29) + 333
    nb = L // C + 1
    seed = 2024
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * w)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, seed))
        fk, ak = hashlib.sha256(b"big-f").digest(), hashlib.sha256(b"big-a").digest()
        dev_encode(nat, p, S, fk, ak, buf.p, L, nb, tb.p)
        tags = tb.download()
        rng = np.random.default_rng(7)
        runs = [(0, 1000), (nb - 1000, 1000)] + [(int(b), 1) for b in rng.integers(0, nb, 10000)]
        for b0, n in runs:
            lo, hi = b0 * C, min((b0 + n) * C, L)
            data = splitmix_bytes(seed, lo, hi - lo)
            want = oracle.encode(p, S, fk, ak, data, block_base=b0, nblocks=n)
            assert split_tags(tags[b0 * w:(b0 + n) * w], w) == want, b0
        # prove over the whole file: offsets of challenged blocks past 2^32
        key = hashlib.sha256(b"big-chal").digest()
        chunks = 2000
        mu = ctypes.create_string_buffer(w * S)
        sg = ctypes.create_string_buffer(w)
        pb = nat.be(p)
        ctx.check(nat.lib().hb_prove(ctx.h, pb, 32, S, key, 32, chunks, pb, 32, tb.p, nb, buf.p, L, 3,
                                     mu, sg))
        host = np.empty(L, dtype=np.uint8)
        ctx.check(nat.lib().hb_memcpy(ctx.h, host.ctypes.data, buf.p, L, 2))
        omu = ctypes.create_string_buffer(w * S)
        osg = ctypes.create_string_buffer(w)
        rc = oracle.lib().hbo_prove(pb, len(pb), S, key, 32, chunks, pb, len(pb), nb,
                                    tags, w, host.ctypes.data, L, omu, osg)
        assert rc == 0
        assert (mu.raw, sg.raw) == (omu.raw, osg.raw)
        # at least one challenged block lies past 4 GiB (else the case is vacuous)
        idx = [oracle.prf_eval(key, nb, i) for i in range(chunks)]
        assert max(idx) * C > (1 << 32)
    finally:
        buf.free()
        tb.free()


def test_prove_host_file_multi_batch(nat, oracle, monkeypatch):
    """The host-file prove's batched path (hb_runtime.cpp prove_impl): the
    challenged blocks of a host-resident file gathered by several host
    threads into two pinned buffers, batch k + 1 gathered while batch k is
    copied and summed, partial sums accumulated across batches.  Batches are
    shrunk by the HB_TEST_PROVE_BATCH hook to 2,500 blocks so that a 7,777-index
    challenge runs 4 batches (3 of them gathered on 4 threads); a 255-bit prime
    (31-byte sectors, 10 per block: C = 310) puts each batch's tag region at an
    unaligned offset of its staging buffer.  == the oracle and == the same
    proof with everything device-resident.  (The hook also keeps the 3 MiB
    file from being uploaded whole; the last run, without it, uploads it --
    a small host file is proved device-resident)
    Reference: PySwizzle.py:351-368."""
    from conftest import load_golden
    p = int(load_golden("primes.json")["p255"], 16)
    S, ss = 10, 31
    C, w = S * ss, 32
    L = 3 * (1 << 20) + 123
    nb = L // C + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * w)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 77))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tb.p)
        htags = tb.download()
        hdata = buf.download()
        hd = ctypes.create_string_buffer(hdata, L)
        ht = ctypes.create_string_buffer(htags, len(htags))
        key = hashlib.sha256(b"multi-batch").digest()
        pb = nat.be(p)
        chunks = 7777
        res = []
        monkeypatch.setenv("HB_GATHER_THREADS", "4")
        for tptr, dptr, flags, batch in ((tb.p, buf.p, 3, None), (ht, hd, 0, "2500"), (tb.p, hd, 2, "2500"),
                                         (ht, hd, 0, None)):
            if batch:
                monkeypatch.setenv("HB_TEST_PROVE_BATCH", batch)
            else:
                monkeypatch.delenv("HB_TEST_PROVE_BATCH", raising=False)
            mu = ctypes.create_string_buffer(w * S)
            sg = ctypes.create_string_buffer(w)
            ctx.check(nat.lib().hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), tptr, nb, dptr, L,
                                         flags, mu, sg))
            res.append((mu.raw, sg.raw))
        assert res[0] == res[1] == res[2] == res[3]
        omu, osg = oracle.prove(p, S, key, chunks, p, split_tags(htags, w), hdata)
        assert [int.from_bytes(res[1][0][j * w:(j + 1) * w], "big") for j in range(S)] == omu
        assert int.from_bytes(res[1][1], "big") == osg
    finally:
        buf.free()
        tb.free()


def test_prove_mixed_residency_equals_device(nat, oracle):
    """hb_prove with the file on the device and the tags on the host (the tags
    are uploaded, the file is not copied back), and the other way round, ==
    the all-device prove == the oracle."""
    p, S, L = P256, 16, 16 << 20
    nb = L // 512 + 1
    buf = DevBuf(nat, L)
    tb = DevBuf(nat, nb * 32)
    try:
        ctx = nat.context()
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, L, 123))
        dev_encode(nat, p, S, b"f" * 32, b"a" * 32, buf.p, L, nb, tb.p)
        htags = tb.download()
        hdata = buf.download()
        hd = ctypes.create_string_buffer(hdata, L)
        ht = ctypes.create_string_buffer(htags, len(htags))
        key = hashlib.sha256(b"mixed").digest()
        pb = nat.be(p)
        res = []
        for tptr, dptr, flags in ((tb.p, buf.p, 3), (ht, buf.p, 1), (tb.p, hd, 2), (ht, hd, 0)):
            mu = ctypes.create_string_buffer(32 * S)
            sg = ctypes.create_string_buffer(32)
            ctx.check(nat.lib().hb_prove(ctx.h, pb, 32, S, key, 32, 3000, pb, 32, tptr, nb, dptr, L, flags, mu, sg))
            res.append((mu.raw, sg.raw))
        assert res[0] == res[1] == res[2] == res[3]
        omu, osg = oracle.prove(p, S, key, 3000, p, split_tags(htags, 32), hdata)
        assert [int.from_bytes(res[0][0][j * 32:(j + 1) * 32], "big") for j in range(S)] == omu
        assert int.from_bytes(res[0][1], "big") == osg
    finally:
        buf.free()
        tb.free()


@pytest.mark.parametrize("bits,S,nbytes", [
    (1024, 10, 1 << 20),                    # PySwizzle's defaults on a 1 MiB file
    (256, 16, 65535 * 512),                 # 65,536 blocks: the largest small input (256 CUs)
    (256, 16, 65536 * 512),                 # one block more: the quad engine on a job queue
    (256, 1, 32 << 20),                     # 2^20 + 1 blocks: still the queue (17 x 256 x #CUs)
    (256, 1, 36 << 20),                     # 1,179,649 blocks: the two-pass engine
    (512, 16, 1000 << 20),                  # 1,024,001 blocks of a 512-bit prime: still the queue (16 x 256 x #CUs)
    (256, 16, (600 << 20) + 5),             # host path: three 256 MiB windows, each on the queue
    (1024, 10, (600 << 20) + 5),            # the same at PySwizzle's defaults (209,715-block windows)
    (256, 1, (3 << 20) + 7),                # S = 1, ragged tail
    (384, 3, 200000),                       # 48-byte sectors: byte-wise MAC loads
    (1024, 10, (1 << 20) + 333),            # NL = 32, ragged tail: a short sector, then none
    (1020, 16, 300001),                     # NL = 32, 127-byte sectors
    (2048, 4, 100000),                      # NL = 64: 128-lane workgroups of the split MAC
    (512, 200, 1 << 20),                    # one block per 200-lane workgroup
    (256, 300, 1 << 20),                    # S > 256: one lane per block (hb_mac_kernel)
])
def test_small_encode_equals_two_pass_and_oracle(nat, oracle, monkeypatch, bits, S, nbytes):
    """Small and mid-size inputs (placed quad waves up to 256 x #CUs blocks,
    then the quad engine on a job queue up to 17 x 256 x #CUs) take the
    quad-PRF + MAC-kernel path (the sectors of a
    block over S lanes, hb_mac_split_kernel, for 2 <= S <= 256); the same encode
    forced through the two-pass engine (HB_NO_SMALL_ENCODE) and the oracle
    agree, from device memory and from host memory through the drop-in API.
    Reference: PySwizzle.py:279-314."""
    import random
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(bits * 31 + S)
    while True:
        p = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(p):
            break
    w = nat.width_of(p)
    C = (p.bit_length() // 8) * S
    nb = nbytes // C + 1
    data = np.random.default_rng(bits + S).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"se-f%d" % bits).digest(), hashlib.sha256(b"se-a%d" % bits).digest()
    buf = DevBuf(nat, nbytes)
    res = []
    try:
        buf.upload(data)
        for two_pass in (False, True):
            if two_pass:
                monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
            else:
                monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
            tb = DevBuf(nat, nb * w)
            try:
                dev_encode(nat, p, S, fk, ak, buf.p, nbytes, nb, tb.p)
                res.append(tb.download())
            finally:
                tb.free()
            tag, n = pys.encode_file(p, S, fk, ak, io.BytesIO(data))
            assert n == nb and bytes(tag.raw(p)) == res[-1]
    finally:
        monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
        buf.free()
    assert res[0] == res[1]
    want = oracle.encode(p, S, fk, ak, data, nthreads=8) if nb <= 70000 else None
    if want is not None:
        assert split_tags(res[0], w) == want


@pytest.mark.parametrize("S,nblocks,check", [
    (1, 60000, "oracle"),         # every block against the oracle
    (1, 2 * 1024 * 1024, "mid"),  # 2 M blocks: the two-pass engine against the queued quad engine
])
def test_retry_quad_tail_high_rejection(nat, oracle, monkeypatch, S, nblocks, check):
    """A 256-bit prime just above 2^255 rejects almost half of all tries
    (E[tries] = 2^256/p ~ 2), so the two-pass engine's retry pass ends in
    long chains that each wave hands to quads once its queue is drained
    (hb_engine_tail): its tags == the oracle's, and == the queued quad engine's
    (HB_MID_BLOCKS) on 2 M blocks.  Reference: PySwizzle.py:279-314, util.py:83-96."""
    import random
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(4242)
    while True:
        p = (1 << 255) + (rng.getrandbits(200) | 1)
        if pys._is_probable_prime(p):
            break
    w = nat.width_of(p)
    C = (p.bit_length() // 8) * S
    nbytes = (nblocks - 1) * C + 7
    data = np.random.default_rng(nblocks).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"rt-f").digest(), hashlib.sha256(b"rt-a").digest()
    buf = DevBuf(nat, nbytes)
    res = []
    try:
        buf.upload(data)
        for mode in ("two_pass", check):
            if mode == "two_pass":
                monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
            else:
                monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
                monkeypatch.setenv("HB_MID_BLOCKS", "100000000")
            if mode == "oracle":
                break
            tb = DevBuf(nat, nblocks * w)
            try:
                tries = dev_encode(nat, p, S, fk, ak, buf.p, nbytes, nblocks, tb.p)
                assert tries > 1.8 * nblocks, tries   # the retry pass had long chains to run
                res.append(tb.download())
            finally:
                tb.free()
    finally:
        monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
        monkeypatch.delenv("HB_MID_BLOCKS", raising=False)
        buf.free()
    if check == "oracle":
        assert split_tags(res[0], w) == oracle.encode(p, S, fk, ak, data, nthreads=8)
    else:
        assert res[0] == res[1]
