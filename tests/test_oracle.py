"""The CPU oracle (oracle/swizzle_oracle.c) against golden vectors produced by
the reference PySwizzle (tests/golden/make_golden.py).  Pins the oracle."""
import hashlib
import os

from conftest import fixture_file


def test_prf_kats(oracle, golden_prf):
    n = 0
    for c in golden_prf["cases"]:
        key = bytes.fromhex(c["key"])
        rng = int(c["range"])
        for x, o in zip(c["xs"], c["outs"]):
            assert oracle.prf_eval(key, rng, int(x)) == int(o), (c["range"], x)
            n += 1
    assert n > 1000


def test_encode_prove_verify(oracle, golden_encode):
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        S = c["sectors"]
        data = bytes.fromhex(c["data"])
        fk, ak = bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"])
        tags = oracle.encode(p, S, fk, ak, data)
        assert tags == [int(t, 16) for t in c["tags"]], c["name"]
        for chn, prn in (("chal", "proof"), ("chal2", "proof2")):
            ch = c[chn]
            mu, sg = oracle.prove(p, S, bytes.fromhex(ch["key"]), ch["chunks"],
                                  int(ch["v_max"], 16), tags, data)
            assert mu == [int(m, 16) for m in c[prn]["mu"]], c["name"]
            assert sg == int(c[prn]["sigma"], 16), c["name"]
            assert oracle.verify(p, S, fk, ak, len(tags), bytes.fromhex(ch["key"]), ch["chunks"],
                                 int(ch["v_max"], 16), mu, sg)


def test_multithreaded_encode_matches(oracle, golden_files):
    for c in golden_files["cases"]:
        data = fixture_file(c["file"])
        p = int(c["prime"], 16)
        w = (p.bit_length() + 7) // 8
        tags = oracle.encode(p, c["sectors"], bytes.fromhex(c["f_key"]),
                             bytes.fromhex(c["alpha_key"]), data, nthreads=4)
        assert len(tags) == c["ntags"]
        h = hashlib.sha256(b"".join(t.to_bytes(w, "big") for t in tags)).hexdigest()
        assert h == c["tags_sha256"], c["name"]
        ch = c["chal"]
        mu, sg = oracle.prove(p, c["sectors"], bytes.fromhex(ch["key"]), ch["chunks"],
                              int(ch["v_max"], 16), tags, data)
        assert sg == int(c["proof"]["sigma"], 16)
        assert mu == [int(m, 16) for m in c["proof"]["mu"]]


def test_block_range_encode_is_a_slice(oracle):
    """Tags of a block range with block_base == the same blocks of a whole-file run."""
    p = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
    S = 3
    C = 32 * S
    data = bytes(range(256)) * 7 + b"xyz"
    fk, ak = b"f" * 32, b"a" * 32
    full = oracle.encode(p, S, fk, ak, data)
    b0, b1 = 5, 13
    part = oracle.encode(p, S, fk, ak, data[b0 * C:b1 * C], block_base=b0, nblocks=b1 - b0)
    assert part == full[b0:b1]


def test_test6_regenerates():
    assert hashlib.sha256(fixture_file("test6.txt")).hexdigest() == \
        "f07be2d96f37df76af247ea305452706f6558d17a01f04e6550dbfc89c8d7cdd"


def test_cxx_prove_verifies_against_cxx_encode():
    """The oracle's cxx prove / encode restatements agree with the cxx verify
    equation (shacham_waters_private.cxx:791-842): sigma == sum v_i f(idx_i) +
    sum alpha(j) mu_j mod p, sampled and check_all.  Parity unpinned."""
    import hashlib
    from oracle import oracle as O
    p = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
    S = 4
    data = b"".join(hashlib.sha256(b"o%d" % i).digest() for i in range(50)) + b"xyz"
    fk, ak, ck = b"f" * 32, b"a" * 32, b"c" * 32
    tags = O.cxx_encode(p, S, fk, ak, data)
    n = len(tags)
    for chunks in (5, n, n + 3):
        mu, sigma = O.cxx_prove(p, S, ck, chunks, p, n, lambda k: tags[k],
                                lambda off, m: data[off:off + m])
        rhs = 0
        for i in range(min(chunks, n) if chunks >= n else chunks):
            idx = i if chunks >= n else O.cxx_prf_eval(ck, n, i)[0]
            rhs += O.cxx_prf_eval(ck, p, i)[0] * O.cxx_prf_eval(fk, p, idx)[0]
        rhs += sum(O.cxx_prf_eval(ak, p, j)[0] * mu[j] for j in range(S))
        assert sigma == rhs % p, chunks


def test_position_cases(oracle):
    """Reference semantics of the file position (encode reads from tell(),
    prove seeks absolute offsets), 8-bit and 2048-bit primes."""
    from conftest import load_golden
    g = load_golden("position_cases.json")
    for c in g["cases"]:
        p = int(c["prime"], 16)
        S = c["sectors"]
        data = bytes.fromhex(c["data"])
        fk, ak = bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"])
        tags = oracle.encode(p, S, fk, ak, data[c["encode_start"]:])
        assert tags == [int(t, 16) for t in c["tags"]], c["name"]
        for chn, prn, okn in (("chal", "proof", "verifies"), ("chal2", "proof2", "verifies2")):
            ch = c[chn]
            mu, sg = oracle.prove(p, S, bytes.fromhex(ch["key"]), ch["chunks"],
                                  int(ch["v_max"], 16), tags, data)
            assert mu == [int(m, 16) for m in c[prn]["mu"]], c["name"]
            assert sg == int(c[prn]["sigma"], 16), c["name"]
            assert oracle.verify(p, S, fk, ak, len(tags), bytes.fromhex(ch["key"]), ch["chunks"],
                                 int(ch["v_max"], 16), mu, sg) == c[okn], c["name"]


def test_prf_wide_inputs(oracle):
    """KeyedPRF of negative and > 64-bit ints (the reference hashes str(x))."""
    from conftest import load_golden
    for c in load_golden("position_cases.json")["prf_wide_x"]:
        key = bytes.fromhex(c["key"])
        for x, o in zip(c["xs"], c["outs"]):
            assert oracle.prf_eval(key, int(c["range"]), int(x)) == int(o), x


def test_pure_python_port_matches_golden(golden_encode):
    """oracle/pyswizzle_port.py (the single-core "PySwizzle" CPU baseline)."""
    import io
    from oracle import pyswizzle_port as PP
    n = 0
    for c in golden_encode["cases"]:
        if c["len"] > 2000:
            continue
        p = int(c["prime"], 16)
        tags = PP.encode(p, c["sectors"], bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]),
                         io.BytesIO(bytes.fromhex(c["data"])))
        assert tags == [int(t, 16) for t in c["tags"]], c["name"]
        n += 1
    assert n > 100


def test_pure_python_port_prove_verify_match_golden(golden_encode):
    """pyswizzle_port.prove / verify (the "PySwizzle" prove row) == the
    reference's proofs and verdicts."""
    import io
    from oracle import pyswizzle_port as PP
    n = 0
    for c in golden_encode["cases"]:
        if c["len"] > 2000:
            continue
        p = int(c["prime"], 16)
        tags = [int(t, 16) for t in c["tags"]]
        f = io.BytesIO(bytes.fromhex(c["data"]))
        ch, pr = c["chal"], c["proof"]
        mu, sg = PP.prove(p, c["sectors"], f, bytes.fromhex(ch["key"]), ch["chunks"], int(ch["v_max"], 16), tags)
        assert mu == [int(m, 16) for m in pr["mu"]] and sg == int(pr["sigma"], 16), c["name"]
        assert PP.verify(p, c["sectors"], bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"]), len(tags),
                         bytes.fromhex(ch["key"]), ch["chunks"], int(ch["v_max"], 16), mu, sg)
        n += 1
    assert n > 100


def _merkle_file(name):
    import hashlib
    from conftest import fixture_file
    if name in ("test.txt", "test3.txt"):
        return fixture_file(name)
    tag, n = {"rand100k": ("merkle-file", 100003), "tiny5": ("merkle-tiny", 5)}[name]
    out, i = b"", 0
    while len(out) < n:
        out += hashlib.sha256(("%s/%d" % (tag, i)).encode()).digest()
        i += 1
    return out[:n]


def test_oracle_merkle_chunk_hash_vs_reference(oracle):
    """oracle.merkle_chunk_hash == the reference MerkleHelper.get_chunk_hash
    (tests/golden/merkle_cases.json, make_golden_merkle.py)."""
    import json
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_cases.json")))
    from heartbeat_amd.Merkle import MerkleHelper
    ch = g["chain"]
    assert [x.hex() for x in MerkleHelper.seed_chain(bytes.fromhex(ch["key"]), bytes.fromhex(ch["seed"]),
                                                     len(ch["seeds"]))] == ch["seeds"]
    for c in g["cases"]:
        data = _merkle_file(c["file"])
        assert hashlib.sha256(data).hexdigest() == g["files"][c["file"]]["sha256"]
        for sd, leaf in zip(c["seeds"], c["leaves"]):
            assert oracle.merkle_chunk_hash(data, bytes.fromhex(sd), None, c["chunksz"]).hex() == leaf
