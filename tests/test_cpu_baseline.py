"""The native CPU baseline encoder (baseline/hb_cpu_swizzle.cpp, bench.py's
"cxx Swizzle" cpu_baseline row) computes exactly PySwizzle's tags: pinned to
the reference-generated golden vectors (tests/golden/encode_cases.json,
file_cases.json: heartbeat/PySwizzle/PySwizzle.py:279-314), on one and
several threads, block ranges with a block base (the row times prefixes of
the bench file), and its SplitMix64 fill equals the GPU stream's host copy."""
import hashlib
import subprocess

import pytest

from conftest import ROOT, fixture_file, splitmix_bytes


@pytest.fixture(scope="module")
def cpu():
    subprocess.check_call(["make", "-s", "-C", ROOT + "/baseline"])
    from baseline import cpu as C
    C.lib()
    return C


def test_golden_encode_cases(cpu, golden_encode):
    n = 0
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        tags = cpu.encode(p, c["sectors"], bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]),
                          bytes.fromhex(c["data"]), threads=1 + n % 3)
        assert tags == [int(t, 16) for t in c["tags"]], c["name"]
        n += 1
    assert n == 176


def test_golden_prove_cases(cpu, golden_encode):
    """The native prove (configs[4]'s "cxx Swizzle" CPU row) == the
    reference's proofs for every golden case and both challenges
    (PySwizzle.py:333-370), on 1-3 threads."""
    n = 0
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        data = bytes.fromhex(c["data"])
        tags = [int(t, 16) for t in c["tags"]]
        for chn, prn in (("chal", "proof"), ("chal2", "proof2")):
            ch = c[chn]
            mu, sg = cpu.prove(p, c["sectors"], bytes.fromhex(ch["key"]), ch["chunks"], int(ch["v_max"], 16),
                               tags, data, threads=1 + n % 3)
            assert mu == [int(m, 16) for m in c[prn]["mu"]], c["name"]
            assert sg == int(c[prn]["sigma"], 16), c["name"]
            n += 1
    assert n == 352


def test_prove_many_threads_vs_oracle(cpu, oracle):
    """A 10,000-index challenge over a 3 MiB file on 16 threads (the bench's
    configs[4] row shape) == the oracle's prove."""
    p = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
    data = splitmix_bytes(0x5EED0005, 0, (3 << 20) + 99)
    fk, ak = hashlib.sha256(b"hb-bench-f").digest(), hashlib.sha256(b"hb-bench-alpha").digest()
    tags = cpu.encode(p, 16, fk, ak, data, threads=8)
    key = hashlib.sha256(b"hb-bench-challenge").digest()
    got = cpu.prove(p, 16, key, 10000, p, tags, data, threads=16)
    assert got == oracle.prove(p, 16, key, 10000, p, tags, data)


def test_golden_file_cases(cpu, golden_files):
    for c in golden_files["cases"]:
        p = int(c["prime"], 16)
        data = fixture_file(c["file"])
        tags = cpu.encode(p, c["sectors"], bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]), data,
                          threads=4)
        w = (p.bit_length() + 7) // 8
        assert len(tags) == c["ntags"]
        h = hashlib.sha256(b"".join(t.to_bytes(w, "big") for t in tags)).hexdigest()
        assert h == c["tags_sha256"], c["name"]


def test_block_ranges_concatenate(cpu, oracle):
    """A prefix encoded as block ranges with block_base == the whole, == the
    oracle (the cpu_baseline row times ranges of the bench file)."""
    p = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
    data = splitmix_bytes(0x5EED0003, 0, 512 * 300 + 77)
    fk, ak = hashlib.sha256(b"hb-bench-f").digest(), hashlib.sha256(b"hb-bench-alpha").digest()
    whole = cpu.encode(p, 16, fk, ak, data, threads=8)
    assert whole == oracle.encode(p, 16, fk, ak, data)
    parts = []
    for b0, b1 in ((0, 100), (100, 101), (101, 301)):
        parts += cpu.encode(p, 16, fk, ak, data[b0 * 512:], block_base=b0, nblocks=b1 - b0, threads=3)
    assert parts == whole


def test_fill_matches_gpu_stream(cpu):
    import ctypes
    for start, n in ((0, 4096), (13, 1000), (1 << 20, 333)):
        buf = ctypes.create_string_buffer(n)
        cpu.lib().hbcpu_fill(ctypes.addressof(buf), start, n, 0x5EED0003, 4)
        assert buf.raw == splitmix_bytes(0x5EED0003, start, n)
