#!/usr/bin/env python3
"""Generate golden vectors for the Swizzle hot path from the REFERENCE PySwizzle.

Runs only in the build container (it reads ``/root/reference``, which does not
exist on the GPU box).  It imports the unmodified reference modules

    /root/reference/heartbeat/exc.py
    /root/reference/heartbeat/util.py            (KeyedPRF, util.py:44-96)
    /root/reference/heartbeat/PySwizzle/PySwizzle.py  (encode :279, prove :333,
                                                       verify :372, State :94)

under a synthetic ``heartbeat`` package (the package ``__init__`` would import
the unbuilt C++ extension, ``heartbeat/__init__.py:30``), with the offline
PyCrypto-API shim in ``tests/golden/shim`` standing in for PyCrypto 2.6.1.
The shim's ``Random`` is fed the exact key bytes each case needs, so the
reference's internally drawn ``f_key``/``alpha_key``/IV/challenge keys are
known and recorded.

Output: JSON fixtures next to this script (data only: inputs and the
reference's outputs).  Re-run with ``python tests/golden/make_golden.py``.
"""
import hashlib
import importlib.util
import io
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "shim"))

from Crypto import Random as ShimRandom  # noqa: E402  (shim)
from Crypto.Cipher import AES as ShimAES  # noqa: E402


def load_reference():
    pkg = types.ModuleType("heartbeat")
    pkg.__path__ = [os.path.join(REF, "heartbeat")]
    sys.modules["heartbeat"] = pkg

    def load(name, path, is_pkg=False):
        kw = {"submodule_search_locations": [os.path.dirname(path)]} if is_pkg else {}
        spec = importlib.util.spec_from_file_location(name, path, **kw)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    load("heartbeat.exc", os.path.join(REF, "heartbeat/exc.py"))
    load("heartbeat.util", os.path.join(REF, "heartbeat/util.py"))
    sw = load("heartbeat.PySwizzle", os.path.join(REF, "heartbeat/PySwizzle/__init__.py"), True)
    return sw


# ---------------------------------------------------------------- shim KATs
def check_shim():
    # FIPS-197 Appendix C.3 (AES-256 single block)
    k = bytes(range(32))
    c = ShimAES.new(k, ShimAES.MODE_ECB).encrypt(bytes.fromhex("00112233445566778899aabbccddeeff"))
    assert c.hex() == "8ea2b7ca516745bfeafc49904b496089", c.hex()
    # NIST SP 800-38A F.3.5 CFB8-AES256.Encrypt
    k = bytes.fromhex("603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4")
    iv = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
    pt = bytes.fromhex("6bc1bee22e409f96e93d7e117393172aae2d")
    ct = ShimAES.new(k, ShimAES.MODE_CFB, iv).encrypt(pt)
    assert ct.hex() == "dc1f1a8520a64db55fcc8ac554844e889700", ct.hex()
    # stream continues across encrypt() calls (PyCrypto semantics relied on by KeyedPRF.eval)
    a = ShimAES.new(k, ShimAES.MODE_CFB, iv)
    ct2 = a.encrypt(pt[:5]) + a.encrypt(pt[5:])
    assert ct2 == ct


# ---------------------------------------------------------------- inputs
def det_bytes(tag, n):
    out = b""
    i = 0
    while len(out) < n:
        out += hashlib.sha256(("%s/%d" % (tag, i)).encode()).digest()
        i += 1
    return out[:n]


def test6_bytes():
    line = b"abcdefghijklmnopqrstuvwxyz1234567890\n"
    return (line * (999999 // len(line) + 1))[:999999]


def is_probable_prime(n):
    if n < 2:
        return False
    for q in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % q == 0:
            return n == q
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def seeded_prime(tag, bits):
    x = int.from_bytes(det_bytes(tag, (bits + 7) // 8), "big")
    x &= (1 << bits) - 1
    x |= (1 << (bits - 1)) | 1
    while not is_probable_prime(x):
        x += 2
    assert x.bit_length() == bits
    return x


PRIMES = {
    # the bench prime: seeded search, recorded in DESIGN.md
    "p256": seeded_prime("hb-bench-prime-256", 256),
    "p256max": (1 << 256) - 189,          # largest 256-bit prime: E[tries] ~ 1
    "p255": seeded_prime("hb-golden-prime-255", 255),   # sectorsize 31
    "p1024": seeded_prime("hb-golden-prime-1024", 1024),
    "p61": (1 << 61) - 1,                 # sectorsize 7, nb 8
    "p20": seeded_prime("hb-golden-prime-20", 20),      # sectorsize 2, nb 3
}


def next_prime(x):
    """The smallest prime > x."""
    x = x + 1 if x % 2 == 0 else x + 2
    while not is_probable_prime(x):
        x += 2
    return x


# Primes that only the repo's own tests use (no reference output is recorded
# for them), kept in primes.json next to the reference-case primes:
EXTRA_PRIMES = {
    # the smallest 256-bit prime: the PRF's worst case, E[tries] = 2^256/p ~ 2
    # (two-pass encode and retry-list-overflow tests, tests/test_gpu_parity.py)
    "p256lo": next_prime(1 << 255),
}


def tags_digest(tags, width):
    h = hashlib.sha256()
    for t in tags:
        h.update(int(t).to_bytes(width, "big"))
    return h.hexdigest()


def main():
    check_shim()
    sw = load_reference()
    assert is_probable_prime(PRIMES["p256max"])
    out_dir = HERE

    # ------------------------------------------------------------ PRF KATs
    keys = {
        "k32a": det_bytes("prf-key-32a", 32),
        "k32b": det_bytes("prf-key-32b", 32),
        "k16": det_bytes("prf-key-16", 16),
        "k24": det_bytes("prf-key-24", 24),
    }
    ranges = [1, 2, 255, 256, 257, 10000, 1 << 20, (1 << 27) + 1, 33554433,
              (1 << 255) + 1, PRIMES["p256"], PRIMES["p256max"], PRIMES["p255"],
              PRIMES["p1024"], PRIMES["p61"], PRIMES["p20"], (1 << 300) - 1]
    xs = list(range(0, 40)) + [99, 100, 101, 999, 1000, 12345, 99999999, 100000000,
                                (1 << 32) - 1, 1 << 32, (1 << 40) + 7, 10 ** 19,
                                (1 << 64) - 1]
    prf_cases = []
    for kn, k in keys.items():
        for r in ranges:
            if kn != "k32a" and r not in (10000, PRIMES["p256"], PRIMES["p1024"], 1):
                continue
            f = sw.KeyedPRF(k, r)
            prf_cases.append({"key": k.hex(), "range": str(r),
                              "xs": [str(x) for x in xs],
                              "outs": [str(f.eval(x)) for x in xs]})
    with open(os.path.join(out_dir, "prf_kat.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "heartbeat/util.py:44-96 (KeyedPRF)",
                   "cases": prf_cases}, fh, indent=0)
    print("prf cases", len(prf_cases))

    # ------------------------------------------------------------ encode/prove/verify
    enc_cases = []
    beat_key = det_bytes("pyswizzle-state-key", 32)
    for pname, p in PRIMES.items():
        ss = p.bit_length() // 8
        sector_list = (1, 3, 10, 16) if pname not in ("p1024",) else (1, 10)
        for S in sector_list:
            C = S * ss
            lengths = sorted(set([0, 1, ss - 1, ss, ss + 1, C - 1, C, C + 1, 3 * C + 17]))
            for L in lengths:
                if L < 0:
                    continue
                tag_ = "%s/S%d/L%d" % (pname, S, L)
                data = det_bytes("file/" + tag_, L)
                f_key = det_bytes("f/" + tag_, 32)
                a_key = det_bytes("a/" + tag_, 32)
                iv = det_bytes("iv/" + tag_, 16)
                chal_key = det_bytes("chal/" + tag_, 32)
                beat = sw.PySwizzle(S, beat_key, p)
                ShimRandom.reseed(tag_.encode())
                ShimRandom.push(f_key, a_key, iv)
                tag, state = beat.encode(io.BytesIO(data))
                st = state.todict()
                ntags = len(tag.sigma)
                # prove with the default challenge (chunks = #tags) and a custom one
                ShimRandom.push(chal_key)
                chal = beat.gen_challenge(state)
                proof = beat.get_public().prove(io.BytesIO(data), chal, tag)
                ok = beat.verify(proof, chal, state)
                assert ok
                chal2 = sw.Challenge(7, p, det_bytes("chal2/" + tag_, 32))
                proof2 = beat.prove(io.BytesIO(data), chal2, tag)
                ok2 = beat.verify(proof2, chal2, state)
                assert ok2
                # a tampered file must not verify (unless the file is empty)
                bad = bytearray(data)
                if L:
                    bad[L // 2] ^= 0x01
                proof3 = beat.prove(io.BytesIO(bytes(bad)), chal, tag)
                ok3 = beat.verify(proof3, chal, state)
                enc_cases.append({
                    "name": tag_, "prime": hex(p), "sectors": S, "len": L,
                    "data": data.hex(), "f_key": f_key.hex(), "alpha_key": a_key.hex(),
                    "tags": [hex(t) for t in tag.sigma],
                    "state_key": beat_key.hex(), "state_iv": iv.hex(), "state": st,
                    "chal": {"chunks": chal.chunks, "v_max": hex(chal.v_max), "key": chal_key.hex()},
                    "proof": {"mu": [hex(m) for m in proof.mu], "sigma": hex(proof.sigma)},
                    "chal2": {"chunks": 7, "v_max": hex(p), "key": chal2.key.hex()},
                    "proof2": {"mu": [hex(m) for m in proof2.mu], "sigma": hex(proof2.sigma)},
                    "tamper_byte": L // 2 if L else None, "tamper_verifies": bool(ok3),
                    "ntags": ntags,
                })
    with open(os.path.join(out_dir, "encode_cases.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "heartbeat/PySwizzle/PySwizzle.py:279-395",
                   "cases": enc_cases}, fh, indent=0)
    print("encode cases", len(enc_cases))

    # ------------------------------------------------------------ fixture files
    big = []
    t6 = test6_bytes()
    assert hashlib.sha256(t6).hexdigest() == \
        "f07be2d96f37df76af247ea305452706f6558d17a01f04e6550dbfc89c8d7cdd"
    files = {"test.txt": open(os.path.join(REF, "tests/files/test.txt"), "rb").read(),
             "test3.txt": open(os.path.join(REF, "tests/files/test3.txt"), "rb").read(),
             "test6.txt": t6}
    for fname, pname, S in (("test.txt", "p1024", 10), ("test.txt", "p256", 16),
                            ("test3.txt", "p256", 1), ("test6.txt", "p1024", 10),
                            ("test6.txt", "p256", 16), ("test6.txt", "p256", 1)):
        p = PRIMES[pname]
        tag_ = "%s/%s/S%d" % (fname, pname, S)
        f_key = det_bytes("f/" + tag_, 32)
        a_key = det_bytes("a/" + tag_, 32)
        iv = det_bytes("iv/" + tag_, 16)
        beat = sw.PySwizzle(S, beat_key, p)
        ShimRandom.reseed(tag_.encode())
        ShimRandom.push(f_key, a_key, iv)
        tag, state = beat.encode(io.BytesIO(files[fname]))
        width = (p.bit_length() + 7) // 8
        chal_key = det_bytes("chal/" + tag_, 32)
        chal = sw.Challenge(min(len(tag.sigma), 300), p, chal_key)
        proof = beat.prove(io.BytesIO(files[fname]), chal, tag)
        assert beat.verify(proof, chal, state)
        big.append({"name": tag_, "file": fname, "prime": hex(p), "sectors": S,
                    "f_key": f_key.hex(), "alpha_key": a_key.hex(),
                    "ntags": len(tag.sigma), "tags_sha256": tags_digest(tag.sigma, width),
                    "tags_head": [hex(t) for t in tag.sigma[:4]],
                    "tags_tail": [hex(t) for t in tag.sigma[-4:]],
                    "chal": {"chunks": chal.chunks, "v_max": hex(p), "key": chal_key.hex()},
                    "proof": {"mu": [hex(m) for m in proof.mu], "sigma": hex(proof.sigma)}})
        print(tag_, len(tag.sigma))
    with open(os.path.join(out_dir, "file_cases.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "heartbeat/PySwizzle/PySwizzle.py:279-395",
                   "test6_sha256": hashlib.sha256(t6).hexdigest(),
                   "cases": big}, fh, indent=0)
    with open(os.path.join(out_dir, "primes.json"), "w") as fh:
        json.dump({k: hex(v) for k, v in {**PRIMES, **EXTRA_PRIMES}.items()}, fh, indent=1)


def position_cases(sw):
    """File-position semantics and prime sizes outside the main sweep.

    * encode reads from the file's CURRENT position (PySwizzle.py:299) while
      prove seeks ABSOLUTE offsets (PySwizzle.py:353-355): a BytesIO that
      encode left at EOF, a file encoded from a mid position, a file proved
      from a mid position;
    * an 8-bit prime (sector size 1) and a 2048-bit prime (above the 1024-bit
      default, PySwizzle.py:233,251);
    * KeyedPRF inputs outside [0, 2^64): the reference hashes str(x) of any int
      (util.py:91), negative numbers included.
    """
    beat_key = det_bytes("pyswizzle-state-key", 32)
    cases = []

    def flow(name, p, S, data, start, prove_pos, chunks2=7):
        """encode from `start`, then prove on the SAME object positioned at
        `prove_pos` (None: wherever encode left it, i.e. EOF)."""
        f_key = det_bytes("f/" + name, 32)
        a_key = det_bytes("a/" + name, 32)
        iv = det_bytes("iv/" + name, 16)
        chal_key = det_bytes("chal/" + name, 32)
        beat = sw.PySwizzle(S, beat_key, p)
        ShimRandom.reseed(name.encode())
        ShimRandom.push(f_key, a_key, iv)
        fh = io.BytesIO(data)
        fh.seek(start)
        tag, state = beat.encode(fh)
        st = state.todict()                  # encrypted, as encode returns it
        after_encode = fh.tell()
        ShimRandom.push(chal_key)
        chal = beat.gen_challenge(state)
        if prove_pos is not None:
            fh.seek(prove_pos)
        proof = beat.prove(fh, chal, tag)
        ok = beat.verify(proof, chal, state)
        chal2 = sw.Challenge(chunks2, p, det_bytes("chal2/" + name, 32))
        if prove_pos is not None:
            fh.seek(prove_pos)
        proof2 = beat.prove(fh, chal2, tag)
        ok2 = beat.verify(proof2, chal2, state)
        cases.append({
            "name": name, "prime": hex(p), "sectors": S, "data": data.hex(),
            "encode_start": start, "pos_after_encode": after_encode,
            "prove_pos": prove_pos,
            "f_key": f_key.hex(), "alpha_key": a_key.hex(), "state_key": beat_key.hex(),
            "state": st, "tags": [hex(t) for t in tag.sigma],
            "chal": {"chunks": chal.chunks, "v_max": hex(chal.v_max), "key": chal_key.hex()},
            "proof": {"mu": [hex(m) for m in proof.mu], "sigma": hex(proof.sigma)}, "verifies": bool(ok),
            "chal2": {"chunks": chunks2, "v_max": hex(p), "key": chal2.key.hex()},
            "proof2": {"mu": [hex(m) for m in proof2.mu], "sigma": hex(proof2.sigma)},
            "verifies2": bool(ok2),
        })

    p = PRIMES["p256"]
    C = 3 * 32
    d = det_bytes("pos/data", 5 * C + 7)
    flow("pos/p256/eof", p, 3, d, 0, None)
    flow("pos/p256/prove_mid", p, 3, d, 0, 37)
    flow("pos/p256/encode_mid", p, 3, d, 100, None)
    flow("pos/p256/encode_mid_prove0", p, 3, d, 100, 0)
    flow("pos/p255/eof", PRIMES["p255"], 4, det_bytes("pos/data255", 9 * 31 * 4 + 30), 0, None, 40)
    p8 = 251
    for S in (1, 3):
        for L in (0, 1, 2, 3, 5, 17):
            flow("p8/S%d/L%d" % (S, L), p8, S, det_bytes("p8/%d/%d" % (S, L), L), 0, 0)
    p2048 = seeded_prime("hb-golden-prime-2048", 2048)
    for S in (1, 2):
        for L in (0, 1, 255, 256, 257, 3 * 256 * S + 9):
            flow("p2048/S%d/L%d" % (S, L), p2048, S, det_bytes("p2048/%d/%d" % (S, L), L), 0, 0)

    prf = []
    xs = [-1, -2, -10, -(1 << 64), -(10 ** 30), 1 << 64, (1 << 64) + 1, 1 << 100, 10 ** 30,
          (1 << 128) - 1]
    for r in (10000, PRIMES["p256"], p2048):
        k = det_bytes("prf-key-32a", 32)
        f = sw.KeyedPRF(k, r)
        prf.append({"key": k.hex(), "range": str(r), "xs": [str(x) for x in xs],
                    "outs": [str(f.eval(x)) for x in xs]})
    with open(os.path.join(HERE, "position_cases.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py --only position",
                   "reference": "heartbeat/PySwizzle/PySwizzle.py:279-395, heartbeat/util.py:83-96",
                   "p2048": hex(p2048), "cases": cases, "prf_wide_x": prf}, fh, indent=0)
    print("position cases", len(cases))


if __name__ == "__main__":
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "position":
        check_shim()
        position_cases(load_reference())
    else:
        main()
        position_cases(load_reference())
