"""ctypes wrapper for the CPU oracle (``oracle/build/libhboracle.so``).

TEST INFRASTRUCTURE ONLY -- importable by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py``; never by the product package.
See ``swizzle_oracle.c`` for what each function restates (reference file:line).
Parity of this oracle is pinned by ``tests/test_oracle.py`` against golden
vectors generated from the reference PySwizzle (``tests/golden/``).
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libhboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c = ctypes
        L.hbo_prf_eval.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t,
                                   c.c_uint64, c.c_char_p, c.c_size_t]
        L.hbo_encode.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p, c.c_char_p,
                                 c.c_size_t, c.c_uint64, c.c_void_p, c.c_uint64, c.c_uint64,
                                 c.c_void_p, c.c_int]
        L.hbo_prf_eval_dec.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t,
                                       c.c_char_p, c.c_char_p, c.c_size_t]
        L.hbo_cxx_prf_eval.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t,
                                       c.c_uint32, c.c_char_p, c.c_size_t]
        L.hbo_cxx_encode.argtypes = L.hbo_encode.argtypes
        L.hbo_prove.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p, c.c_size_t,
                                c.c_uint64, c.c_char_p, c.c_size_t, c.c_uint64, c.c_char_p,
                                c.c_int, c.c_void_p, c.c_uint64, c.c_char_p, c.c_char_p]
        L.hbo_verify.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p, c.c_char_p,
                                 c.c_size_t, c.c_uint64, c.c_char_p, c.c_size_t, c.c_uint64,
                                 c.c_char_p, c.c_size_t, c.c_char_p, c.c_char_p, c.c_int]
        _lib = L
    return _lib


def _be(n):
    n = int(n)
    return n.to_bytes(max(1, (n.bit_length() + 7) // 8), "big")


def _addr(buf):
    """Address of a bytes-like / numpy buffer (read-only use)."""
    try:
        import numpy as np
        if isinstance(buf, np.ndarray):
            return buf.ctypes.data, buf.nbytes
    except ImportError:
        pass
    if isinstance(buf, (bytearray, memoryview)):
        mv = memoryview(buf)
        arr = (ctypes.c_char * mv.nbytes).from_buffer(mv) if not mv.readonly else None
        if arr is not None:
            return ctypes.addressof(arr), mv.nbytes
        buf = bytes(mv)
    b = ctypes.create_string_buffer(bytes(buf), len(buf))
    _addr.keep = b
    return ctypes.addressof(b), len(buf)


def prf_eval(key, rng, x):
    """KeyedPRF(key, rng).eval(x) (heartbeat/util.py:83-96), any int x."""
    nb = (int(rng).bit_length() + 7) // 8
    out = ctypes.create_string_buffer(max(nb, 1))
    rb = _be(rng)
    x = int(x)
    if 0 <= x < (1 << 64):
        rc = lib().hbo_prf_eval(bytes(key), len(key), rb, len(rb), x, out, nb)
    else:
        rc = lib().hbo_prf_eval_dec(bytes(key), len(key), rb, len(rb), str(x).encode(), out, nb)
    if rc <= 0:
        raise ValueError("oracle prf error %d" % rc)
    return int.from_bytes(out.raw[:nb], "big")


def width_of(p):
    return (int(p).bit_length() + 7) // 8


def encode(p, sectors, f_key, alpha_key, data, block_base=0, nblocks=None, nthreads=1,
           _fn="hbo_encode"):
    """Tags (list of ints) of PySwizzle.encode for the given keys."""
    p = int(p)
    ss = p.bit_length() // 8
    C = ss * sectors
    if nblocks is None:
        nblocks = len(data) // C + 1
    w = width_of(p)
    out = ctypes.create_string_buffer(w * max(nblocks, 1))
    addr, n = _addr(data)
    pb = _be(p)
    rc = getattr(lib(), _fn)(pb, len(pb), sectors, bytes(f_key), bytes(alpha_key), len(f_key),
                             block_base, addr, n, nblocks, out, nthreads)
    if rc:
        raise ValueError("oracle encode error %d" % rc)
    raw = out.raw
    return [int.from_bytes(raw[i * w:(i + 1) * w], "big") for i in range(nblocks)]


def encode_raw(p, sectors, f_key, alpha_key, data_addr, data_len, block_base, nblocks,
               out_addr, nthreads, cxx=False):
    """Zero-copy variant for the CPU baseline: raw addresses in and out."""
    pb = _be(p)
    return (lib().hbo_cxx_encode if cxx else lib().hbo_encode)(pb, len(pb), sectors, bytes(f_key), bytes(alpha_key), len(f_key),
                            block_base, data_addr, data_len, nblocks, out_addr, nthreads)


def cxx_prf_eval(key, limit, i):
    """cxx prf::evaluate(i) (cxx/prf.hxx:125-145) -> (value, tries).  Parity unpinned."""
    lb = _be(limit)
    nb = (int(limit).bit_length() + 7) // 8
    out = ctypes.create_string_buffer(nb)
    tries = lib().hbo_cxx_prf_eval(bytes(key), len(key), lb, len(lb), int(i) & 0xffffffff, out, nb)
    if tries <= 0:
        raise ValueError("oracle cxx prf error %d" % tries)
    return int.from_bytes(out.raw, "big"), tries


def cxx_encode(p, sectors, f_key, alpha_key, data, block_base=0, nblocks=None, nthreads=1):
    """cxx shacham_waters_private::encode tags (list of ints).  Parity unpinned."""
    return encode(p, sectors, f_key, alpha_key, data, block_base, nblocks, nthreads, _fn="hbo_cxx_encode")


def cxx_prove(p, sectors, chal_key, chunks, v_max, ntags, tag_at, read_at):
    """(mu list, sigma) of the cxx shacham_waters_private::prove
    (cxx/shacham_waters_private.cxx:731-789) over cxx_prf_eval: every block in
    order when chunks >= #tags (check_all, :754-755, 762), else
    idx_i = prf(key, #tags)(i) (:743-744, 762); v_i = prf(key, v_max)(i)
    (:746-748, 767); sector offset (unsigned int)(index * chunk_size + j * ss) (:738, 763);
    duplicate indices count again.  tag_at(k) -> int, read_at(off, n) -> the
    file bytes [off, off + n) clipped at EOF (a seek past EOF reads nothing).
    Parity unpinned (Crypto++ absent)."""
    p = int(p)
    ss = p.bit_length() // 8
    C = sectors * ss
    check_all = chunks >= ntags
    n = ntags if check_all else chunks
    mu = [0] * sectors
    sigma = 0
    for i in range(n):
        idx = i if check_all else cxx_prf_eval(chal_key, ntags, i)[0]
        v = cxx_prf_eval(chal_key, v_max, i)[0]
        for j in range(sectors):
            # size_t pos = index*chunk_size + j*_sector_size, all unsigned int (:762-763)
            pos = (idx * C + j * ss) & 0xffffffff
            mu[j] = (mu[j] + v * int.from_bytes(read_at(pos, ss), "big")) % p
        sigma = (sigma + v * tag_at(idx)) % p
    return mu, sigma


def prove(p, sectors, chal_key, chunks, v_max, tags, data):
    """(mu list, sigma) of PySwizzle.prove."""
    p = int(p)
    w = width_of(p)
    tb = b"".join(int(t).to_bytes(w, "big") for t in tags)
    mu = ctypes.create_string_buffer(w * sectors)
    sg = ctypes.create_string_buffer(w)
    vb = _be(v_max)
    pb = _be(p)
    addr, n = _addr(data)
    rc = lib().hbo_prove(pb, len(pb), sectors, bytes(chal_key), len(chal_key), chunks, vb,
                         len(vb), len(tags), tb, w, addr, n, mu, sg)
    if rc:
        raise ValueError("oracle prove error %d" % rc)
    m = [int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(sectors)]
    return m, int.from_bytes(sg.raw, "big")


def verify(p, sectors, f_key, alpha_key, state_chunks, chal_key, chunks, v_max, mu, sigma):
    p = int(p)
    w = width_of(p)
    mub = b"".join((int(m) % (1 << (8 * w))).to_bytes(w, "big") for m in mu)
    sb = (int(sigma) % (1 << (8 * w))).to_bytes(w, "big")
    pb = _be(p)
    vb = _be(v_max)
    rc = lib().hbo_verify(pb, len(pb), sectors, bytes(f_key), bytes(alpha_key), len(f_key),
                          state_chunks, bytes(chal_key), len(chal_key), chunks, vb, len(vb),
                          mub, sb, w)
    if rc < 0:
        raise ValueError("oracle verify error %d" % rc)
    return rc == 1


def merkle_chunk(seed, filesz, chunksz):
    """(offset, length) of MerkleHelper.get_chunk_hash's chunk
    (heartbeat/Merkle/Merkle.py:497-504): chunk = min(chunksz, filesz) bytes at
    KeyedPRF(seed, filesz - chunk + 1).eval(0)."""
    if filesz < chunksz:
        chunksz = filesz
    return prf_eval(seed, filesz - chunksz + 1, 0), chunksz


def merkle_chunk_hash(data, seed, filesz=None, chunksz=8192):
    """MerkleHelper.get_chunk_hash (Merkle.py:480-515) over the bytes `data`:
    HMAC-SHA256(seed, data[offset : offset + chunk])."""
    import hashlib
    import hmac
    filesz = len(data) if filesz is None else filesz
    off, n = merkle_chunk(seed, filesz, chunksz)
    return hmac.new(bytes(seed), bytes(data[off:off + n]), hashlib.sha256).digest()
