"""GPU parity of the split wide-prime encode (primes above 256 bits): F-only
PRF passes, a device-built int8 digit table and the MFMA MAC
(hb_wide.hpp, hb_runtime.cpp wide_plan).  Its tags == the in-kernel VALU
MAC's ($HB_NO_WIDE) == the CPU oracle, for

* PySwizzle's default shape (1024-bit, S = 10: C = 1280, F in the tag slots),
* 512-bit S = 16 and 2048-bit S = 4 (16 / 64 limbs; two MFMA passes at 64),
* 127- and 125-byte sectors (1020 / 1000-bit primes: tags narrower than the
  limbs, F in a buffer of its own; D = 125 digits, partial last tile),
* ragged files (a short last block, and one past EOF) and a tiny file,
* the host path in 256 MiB chunks,
* a full-size 4 GiB device-resident file at PySwizzle's defaults (sampled).

Sizes below the mid-size threshold take the quad-PRF + MAC-kernel path, so
HB_NO_SMALL_ENCODE forces the two-pass engine where the test needs it.
Reference: PySwizzle.py:279-314 (encode), util.py:83-96 (KeyedPRF)."""
import hashlib
import importlib
import io
import random

import numpy as np
import pytest

from test_gpu_parity import DevBuf, dev_encode, split_tags

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    from heartbeat_amd import _native
    _native.context()
    return _native


def _prime(bits, seed):
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(seed)
    while True:
        p = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(p):
            return p


def _encode_both(nat, monkeypatch, p, S, data, nbytes, nb, fk, ak):
    """(split tags, in-kernel-MAC tags) of a device-resident encode."""
    w = nat.width_of(p)
    buf = DevBuf(nat, max(nbytes, 16))
    res = []
    try:
        buf.upload(data)
        for no_wide in (False, True):
            if no_wide:
                monkeypatch.setenv("HB_NO_WIDE", "1")
            else:
                monkeypatch.delenv("HB_NO_WIDE", raising=False)
            tb = DevBuf(nat, nb * w)
            try:
                dev_encode(nat, p, S, fk, ak, buf.p, nbytes, nb, tb.p)
                res.append(tb.download())
            finally:
                tb.free()
    finally:
        monkeypatch.delenv("HB_NO_WIDE", raising=False)
        buf.free()
    return res


@pytest.mark.parametrize("bits,S,nbytes", [
    (1024, 10, 8 << 20),                 # PySwizzle's defaults: F in the tag slots
    (1024, 10, (8 << 20) + 333),         # a short last block
    (1024, 10, 1280 * 5000),             # whole blocks + one block past EOF
    (1024, 10, 100),                     # one short block
    (512, 16, 8 << 20),                  # 16 limbs, 4 tiles
    (2048, 4, 8 << 20),                  # 64 limbs: two MFMA passes of 8 tiles
    (1020, 16, 6 << 20),                 # 127-byte sectors, tw 128 = 4 NL
    (1000, 32, 6 << 20),                 # 125-byte sectors, tw 125: F in c->vals; D = 125
    (384, 4, 4 << 20),                   # 48-byte sectors, 16 limbs, tw 48
])
def test_split_equals_inkernel_mac_and_oracle(nat, oracle, monkeypatch, bits, S, nbytes):
    p = _prime(bits, bits * 13 + S)
    C = (p.bit_length() // 8) * S
    nb = nbytes // C + 1
    data = np.random.default_rng(bits + S + nbytes).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"wd-f%d" % bits).digest(), hashlib.sha256(b"wd-a%d" % bits).digest()
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
    try:
        split, inkernel = _encode_both(nat, monkeypatch, p, S, data, nbytes, nb, fk, ak)
    finally:
        monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
    assert split == inkernel
    w = nat.width_of(p)
    got = split_tags(split, w)
    if nb <= 7000:
        assert got == oracle.encode(p, S, fk, ak, data, nthreads=8)
    else:
        rng = np.random.default_rng(nb)
        for b in sorted(set(rng.integers(0, nb, 300).tolist()) | {0, nb - 2, nb - 1}):
            blk = data[b * C:(b + 1) * C]
            assert got[b] == oracle.encode(p, S, fk, ak, blk, block_base=b, nblocks=1)[0], b


def test_split_host_path_chunks(nat, oracle, monkeypatch):
    """The host path at PySwizzle's defaults through encode_file, two-pass in
    256 MiB chunks (209,715 blocks each, three chunks), == the device path."""
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    p = _prime(1024, 4242)
    S = 10
    C = 1280
    nbytes = (600 << 20) + 77
    nb = nbytes // C + 1
    data = np.random.default_rng(600).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"hp-f").digest(), hashlib.sha256(b"hp-a").digest()
    monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
    try:
        tag, n = pys.encode_file(p, S, fk, ak, io.BytesIO(data))
        host = bytes(tag.raw(p))
        buf = DevBuf(nat, nbytes)
        tb = DevBuf(nat, nb * 128)
        try:
            buf.upload(data)
            dev_encode(nat, p, S, fk, ak, buf.p, nbytes, nb, tb.p)
            dev = tb.download()
        finally:
            buf.free()
            tb.free()
    finally:
        monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
    assert n == nb and host == dev
    got = split_tags(host, 128)
    for b in (0, 209714, 209715, 419430, 419431, nb - 2, nb - 1):
        assert got[b] == oracle.encode(p, S, fk, ak, data[b * C:(b + 1) * C], block_base=b, nblocks=1)[0], b


def test_split_4gib_defaults_sampled(nat, oracle, monkeypatch):
    """4 GiB device-resident at PySwizzle's defaults (3.36 M blocks, past the
    mid-size threshold: the two-pass split engine without any switch) ==
    the in-kernel MAC, and 2,000 sampled blocks + both ends == the oracle."""
    from conftest import splitmix_bytes
    p = _prime(1024, 1024)
    S = 10
    C = 1280
    n = 4 << 30
    nb = n // C + 1
    w = 128
    fk, ak = hashlib.sha256(b"4g-f").digest(), hashlib.sha256(b"4g-a").digest()
    ctx = nat.context()
    buf = DevBuf(nat, n)
    res = []
    try:
        ctx.check(nat.lib().hb_fill_random(ctx.h, buf.p, n, 4242))
        for no_wide in (False, True):
            if no_wide:
                monkeypatch.setenv("HB_NO_WIDE", "1")
            tb = DevBuf(nat, nb * w)
            try:
                dev_encode(nat, p, S, fk, ak, buf.p, n, nb, tb.p)
                res.append(tb.download())
            finally:
                tb.free()
    finally:
        monkeypatch.delenv("HB_NO_WIDE", raising=False)
        buf.free()
    assert res[0] == res[1]
    got = split_tags(res[0], w)
    rng = np.random.default_rng(7)
    for b in sorted(set(rng.integers(0, nb, 2000).tolist()) | {0, 1, nb - 2, nb - 1}):
        m = min(C, max(0, n - b * C))
        blk = splitmix_bytes(4242, b * C, m)
        assert got[b] == oracle.encode(p, S, fk, ak, blk, block_base=b, nblocks=1)[0], b


@pytest.mark.parametrize("nbytes", [8 << 20, (8 << 20) + 333, 1280 * 5000, 100])
def test_split_cxx_prf_equals_inkernel_mac_and_oracle(nat, oracle, monkeypatch, nbytes):
    """The cxx Swizzle encode (cxx prf, single-pass engine) at its API's
    1024-bit prime, S = 10, through the split MAC == its in-kernel VALU MAC
    ($HB_NO_WIDE) == the oracle's cxx restatement (parity of the cxx mode
    itself is unpinned: no Crypto++).  1280 x 5000 bytes ends on a block
    boundary, so the last block has no sector read and keeps F unreduced
    (shacham_waters_private.cxx:681-690).  Reference: :638-702."""
    p = _prime(1024, 99)
    S, C, w = 10, 1280, 128
    nb = nbytes // C + 1
    data = np.random.default_rng(nbytes).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"cx-f").digest(), hashlib.sha256(b"cx-a").digest()
    ctx = nat.context()
    pb = nat.be(p)
    buf = DevBuf(nat, max(nbytes, 16))
    res = []
    try:
        buf.upload(data)
        for no_wide in (False, True):
            if no_wide:
                monkeypatch.setenv("HB_NO_WIDE", "1")
            tb = DevBuf(nat, nb * w)
            try:
                ctx.check(nat.lib().hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, buf.p, nbytes, nb, tb.p,
                                              3 | nat.HB_PRF_CXX, None))
                res.append(tb.download())
            finally:
                tb.free()
    finally:
        monkeypatch.delenv("HB_NO_WIDE", raising=False)
        buf.free()
    assert res[0] == res[1]
    got = split_tags(res[0], w)
    if nb <= 7000:
        assert got == oracle.cxx_encode(p, S, fk, ak, data, nthreads=8)
    else:
        for b in sorted(set(np.random.default_rng(3).integers(0, nb, 300).tolist()) | {0, nb - 2, nb - 1}):
            assert got[b] == oracle.cxx_encode(p, S, fk, ak, data[b * C:(b + 1) * C], block_base=b, nblocks=1)[0], b


@pytest.mark.parametrize("toff,small", [(16, False), (4, False), (16, True), (4, True)])
def test_split_tag_alignment(nat, oracle, monkeypatch, toff, small):
    """hb_wmac_kernel's coalesced finish (F and tags through LDS in 16-byte
    pieces) runs when the tags are 16-byte aligned, the per-lane finish when
    they are not (toff = 4: F in a buffer of its own, dword tag stores); both
    on the two-pass engine and on the mid-size path (F from the quad-PRF
    launch), with a partial last workgroup (5,001 blocks = 39 x 128 + 9), ==
    the in-kernel MAC == the oracle."""
    p = _prime(1024, 777)
    S, C, w = 10, 1280, 128
    nbytes = C * 5000 + 77
    nb = nbytes // C + 1
    data = np.random.default_rng(toff + 2 * small).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"al-f").digest(), hashlib.sha256(b"al-a").digest()
    buf = DevBuf(nat, nbytes)
    res = []
    try:
        buf.upload(data)
        if not small:
            monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
        for no_wide in (False, True):
            if no_wide:
                monkeypatch.setenv("HB_NO_WIDE", "1")
            tb = DevBuf(nat, nb * w + 32)
            try:
                tb.upload(b"\xa5" * (nb * w + 32))
                dev_encode(nat, p, S, fk, ak, buf.p, nbytes, nb, tb.p + toff)
                raw = tb.download()
                assert raw[:toff] == b"\xa5" * toff and raw[toff + nb * w:] == b"\xa5" * (32 - toff)
                res.append(raw[toff:toff + nb * w])
            finally:
                tb.free()
    finally:
        monkeypatch.delenv("HB_NO_WIDE", raising=False)
        monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
        buf.free()
    assert res[0] == res[1]
    assert split_tags(res[0], w) == oracle.encode(p, S, fk, ak, data, nthreads=8)


@pytest.mark.parametrize("bits,S,nbytes,base", [
    (1024, 64, 8 << 20, 0),          # 8 KiB blocks: 128 K slices
    (1024, 250, 8 << 20, 0),         # C = 32,000: the largest column-sum range the int32 MFMA takes
    (1024, 260, 8 << 20, 0),         # C = 33,280 > 32,768: wide_plan declines, the VALU MAC runs
    (1024, 10, 4 << 20, 12345),      # a shard's block range (block_base != 0)
    (512, 1, 8 << 20, 0),            # one 64-byte sector per block: one slice
    (2048, 1, 4 << 20, 7),           # one 256-byte sector, NL = 64
])
@pytest.mark.parametrize("two_pass", [True, False])
def test_split_shapes_and_block_base(nat, oracle, monkeypatch, bits, S, nbytes, base, two_pass):
    """More split-encode shapes on both engines (two-pass and the mid-size
    quad-PRF path): large and single-slice blocks, the C <= 32 KiB bound of
    the int8 column sums and the fallback past it, and a nonzero block_base
    (the F PRF's input is block_base + k) == the in-kernel MAC == the oracle
    (all blocks up to 7,000, else 300 sampled + both ends)."""
    p = _prime(bits, bits * 7 + S)
    C = (p.bit_length() // 8) * S
    nb = nbytes // C + 1
    w = nat.width_of(p)
    data = np.random.default_rng(bits + S + base).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    fk, ak = hashlib.sha256(b"sb-f%d" % bits).digest(), hashlib.sha256(b"sb-a%d" % bits).digest()
    buf = DevBuf(nat, nbytes)
    res = []
    try:
        buf.upload(data)
        if two_pass:
            monkeypatch.setenv("HB_NO_SMALL_ENCODE", "1")
        for no_wide in (False, True):
            if no_wide:
                monkeypatch.setenv("HB_NO_WIDE", "1")
            tb = DevBuf(nat, nb * w)
            try:
                dev_encode(nat, p, S, fk, ak, buf.p, nbytes, nb, tb.p, block_base=base)
                res.append(tb.download())
            finally:
                tb.free()
    finally:
        monkeypatch.delenv("HB_NO_WIDE", raising=False)
        monkeypatch.delenv("HB_NO_SMALL_ENCODE", raising=False)
        buf.free()
    assert res[0] == res[1]
    got = split_tags(res[0], w)
    if nb <= 7000:
        assert got == oracle.encode(p, S, fk, ak, data, block_base=base, nthreads=8)
    else:
        rng = np.random.default_rng(nb + base)
        for b in sorted(set(rng.integers(0, nb, 300).tolist()) | {0, nb - 2, nb - 1}):
            blk = data[b * C:(b + 1) * C]
            assert got[b] == oracle.encode(p, S, fk, ak, blk, block_base=base + b, nblocks=1)[0], b
