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
