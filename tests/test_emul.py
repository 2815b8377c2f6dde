"""CPU emulation of one GPU lane (tests/emul/emul.cpp compiles the kernels'
per-lane code, heartbeat_amd/csrc/hb_lane.hpp, as plain C++) against the
golden vectors: checks the T-table AES-CFB8 (LDS image layout included),
SHA-256 message builder and Montgomery arithmetic without a GPU."""
import ctypes
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "emul", "libhbemul.so")


@pytest.fixture(scope="module")
def emul():
    src = os.path.join(HERE, "emul", "emul.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", SO, src])
    L = ctypes.CDLL(SO)
    c = ctypes
    L.emul_prf.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t, c.c_uint64,
                           c.c_char_p, c.c_int, c.c_int]
    L.emul_encode.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p, c.c_char_p,
                              c.c_size_t, c.c_uint64, c.c_char_p, c.c_uint64, c.c_uint64,
                              c.c_char_p, c.c_int, c.c_int, c.c_int]
    L.emul_prefix_check.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_int]
    L.emul_early.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t, c.c_uint64, c.c_uint64,
                             c.POINTER(c.c_uint64)]
    return L


def _be(n):
    return n.to_bytes((n.bit_length() + 7) // 8, "big")


@pytest.mark.parametrize("use_prefix", [0, 1])
def test_prf_lane_matches_reference(emul, golden_prf, use_prefix):
    lane = 0
    for c in golden_prf["cases"]:
        k = bytes.fromhex(c["key"])
        r = int(c["range"])
        nb = (r.bit_length() + 7) // 8
        for x, o in zip(c["xs"], c["outs"]):
            out = ctypes.create_string_buffer(nb)
            tries = emul.emul_prf(k, len(k), _be(r), len(_be(r)), int(x), out, lane % 64, use_prefix)
            lane += 7
            assert tries >= 1
            assert int.from_bytes(out.raw, "big") == int(o), (c["range"], x)


@pytest.mark.parametrize("align,use_prefix", [(1, 0), (16, 0), (1, 1), (16, 1)])
def test_encode_lane_matches_reference(emul, golden_encode, align, use_prefix):
    for c in golden_encode["cases"]:
        p = int(c["prime"], 16)
        bits = p.bit_length()
        nl = 8 if bits <= 256 else 16 if bits <= 512 else 32
        if align == 16 and bits // 8 != 4 * nl:
            continue
        w = (p.bit_length() + 7) // 8
        data = bytes.fromhex(c["data"])
        nt = c["ntags"]
        out = ctypes.create_string_buffer(w * nt)
        rc = emul.emul_encode(_be(p), len(_be(p)), c["sectors"], bytes.fromhex(c["f_key"]),
                              bytes.fromhex(c["alpha_key"]), 32, 0, data, len(data), nt, out,
                              (nt * 13) % 64, align, use_prefix)
        assert rc == 0
        got = [int.from_bytes(out.raw[i * w:(i + 1) * w], "big") for i in range(nt)]
        assert got == [int(t, 16) for t in c["tags"]], c["name"]


@pytest.mark.parametrize("keylen", [16, 24, 32])
def test_prefix_image_entries(emul, keylen):
    """hb_prefix_kernel's entries (lane AES of hb_pfx_s3(i)) == host AES of the
    register bytes each entry stands for: all of P1, P2 and 4096 P3 entries."""
    key = bytes(range(7, 7 + keylen))
    assert emul.emul_prefix_check(key, keylen, 4096, 37) == 0


CXX_LIMITS = [
    int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16),  # bench prime
    (1 << 255) + 95,          # E[tries] ~ 2: exercises retries
    (1 << 127) + 45,          # 16-byte limit (one CFB block, truncated digest)
    (1 << 384) - 317,         # 48 bytes: zero plaintext beyond the digest
    (1 << 1023) + 1155,       # cxx API default width (1024-bit)
    (17 << 1016) + 1,         # top byte 0x11: clz-derived mask 0x1f, many retries
    # ByteCount not a multiple of 16 (hb_cxx_try_bytes; the cxx prove's
    # indexer has limit = #tags): the CFB-128 stream continues mid-block
    2, 255, 10000, (1 << 27) + 1, 9437185, (1 << 200) + 1, (17 << 120) + 3,
]


def test_cxx_prf_lane_matches_oracle(emul):
    """hb_cxx_try / hb_cxx_try_bytes (full-output T-table AES, CFB-128, SHA256(LE32 i)) == the
    oracle's OpenSSL restatement of cxx/prf.hxx (parity unpinned: no Crypto++)."""
    import oracle.oracle as O
    c = ctypes
    emul.emul_cxx_prf.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t, c.c_uint32,
                                  c.c_char_p, c.c_int]
    lane = 0
    for keylen in (16, 24, 32):
        key = bytes(range(3, 3 + keylen))
        for lim in CXX_LIMITS:
            nb = (lim.bit_length() + 7) // 8
            for x in [0, 1, 2, 255, 256, 65537, 2 ** 31, 2 ** 32 - 1] + list(range(1000, 1040)):
                out = ctypes.create_string_buffer(nb)
                tries = emul.emul_cxx_prf(key, keylen, _be(lim), len(_be(lim)), x, out, lane % 64)
                lane += 5
                v, t = O.cxx_prf_eval(key, lim, x)
                assert (int.from_bytes(out.raw, "big"), tries) == (v, t), (keylen, hex(lim), x)


def test_merkle_lane_matches_reference(emul):
    """The Merkle kernels' lane code (in-lane AES key expansion, KeyedPRF
    eval(0) with per-lane round keys, HMAC-SHA256 with unaligned whole-block
    loads) == the reference MerkleHelper.get_chunk_hash (golden)."""
    import json
    from test_oracle import _merkle_file
    c_ = ctypes
    emul.emul_merkle.argtypes = [c_.c_char_p, c_.c_size_t, c_.c_char_p, c_.c_uint64, c_.c_uint64,
                                 c_.c_uint64, c_.c_int, c_.POINTER(c_.c_uint64), c_.c_char_p]
    g = json.load(open(os.path.join(HERE, "golden", "merkle_cases.json")))
    lane = 0
    for c in g["cases"]:
        data = _merkle_file(c["file"])
        for sd, leaf in zip(c["seeds"], c["leaves"]):
            seed = bytes.fromhex(sd)
            off = ctypes.c_uint64()
            dg = ctypes.create_string_buffer(32)
            tries = emul.emul_merkle(seed, len(seed), data, len(data), len(data), c["chunksz"], lane % 64,
                                     ctypes.byref(off), dg)
            lane += 3
            assert tries >= 1
            assert dg.raw.hex() == leaf, (c["file"], c["chunksz"], sd)


@pytest.mark.parametrize("bits,x0", [(256, 0), (256, 123456789), (255, 10**12), (250, 77), (61, 5), (512, 1000)])
def test_early_retry_listing_premise(emul, bits, x0):
    """The first pass lists an eval for the retry pass before its first try
    when the try's first output word (from the prefix image) exceeds R's top
    32 bits (hb_range_top, HB_RETRY_DIGEST): such a try must always be
    rejected, and the rule must catch nearly every rejection."""
    import random
    rng = random.Random(bits * 1000003 + x0)
    key = bytes(rng.randrange(256) for _ in range(32))
    # a range whose top byte leaves room for rejections (like the bench prime)
    r = rng.randrange(1 << (bits - 1), (1 << bits) - (1 << (bits - 3)))
    counts = (ctypes.c_uint64 * 3)()
    n = 20000
    assert emul.emul_early(key, len(key), _be(r), len(_be(r)), x0, n, counts) == 0
    rejected, early, wrong = counts[0], counts[1], counts[2]
    assert wrong == 0
    assert early <= rejected
    assert rejected > n // 50
    assert early >= rejected - 2, (rejected, early)
