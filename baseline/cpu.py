"""ctypes binding of baseline/build/libhbcpu.so, the native multi-threaded
CPU encoder timed as bench.py's "cxx Swizzle" cpu_baseline row
(hb_cpu_swizzle.cpp).  Measurement infrastructure: the product package
(heartbeat_amd) never imports it."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "libhbcpu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            raise RuntimeError("baseline/build/libhbcpu.so is not built (make -C baseline)")
        L = ctypes.CDLL(SO)
        c = ctypes
        L.hbcpu_encode.restype = c.c_int
        L.hbcpu_encode.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p, c.c_char_p, c.c_size_t,
                                   c.c_uint64, c.c_void_p, c.c_uint64, c.c_uint64, c.c_void_p, c.c_int,
                                   c.POINTER(c.c_uint64)]
        L.hbcpu_prove.restype = c.c_int
        L.hbcpu_prove.argtypes = [c.c_char_p, c.c_size_t, c.c_uint32, c.c_char_p, c.c_size_t, c.c_uint64,
                                  c.c_char_p, c.c_size_t, c.c_uint64, c.c_void_p, c.c_void_p, c.c_uint64, c.c_int,
                                  c.c_char_p, c.c_char_p]
        L.hbcpu_aesni.restype = c.c_int
        L.hbcpu_fill.restype = None
        L.hbcpu_fill.argtypes = [c.c_void_p, c.c_uint64, c.c_uint64, c.c_uint64, c.c_int]
        _lib = L
    return _lib


def encode_raw(p, sectors, f_key, alpha_key, data_addr, length, block_base, nblocks, tags_addr, threads):
    """Tags of `nblocks` blocks of the host buffer at data_addr (hb_encode's
    contract); returns PRF tries."""
    pb = int(p).to_bytes((int(p).bit_length() + 7) // 8, "big")
    tries = ctypes.c_uint64(0)
    rc = lib().hbcpu_encode(pb, len(pb), sectors, f_key, alpha_key, len(f_key), block_base, data_addr, length,
                            nblocks, tags_addr, threads, ctypes.byref(tries))
    if rc:
        raise RuntimeError("hbcpu_encode error %d" % rc)
    return tries.value


def encode(p, sectors, f_key, alpha_key, data, block_base=0, nblocks=None, threads=1):
    """Tags (ints) of a bytes object."""
    w = (int(p).bit_length() + 7) // 8
    C = (int(p).bit_length() // 8) * sectors
    n = len(data) // C + 1 if nblocks is None else nblocks
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    out = ctypes.create_string_buffer(max(1, n * w))
    encode_raw(p, sectors, f_key, alpha_key, ctypes.addressof(buf) if data else None, len(data), block_base, n,
               ctypes.addressof(out), threads)
    raw = out.raw
    return [int.from_bytes(raw[i * w:(i + 1) * w], "big") for i in range(n)]


def prove_raw(p, sectors, key, chunks, v_max, ntags, tags_addr, data_addr, length, threads):
    """(mu list, sigma) of PySwizzle.prove over host buffers: tags_addr holds
    ntags big-endian tags of ceil(bitlen(p) / 8) bytes, data_addr the file."""
    w = (int(p).bit_length() + 7) // 8
    pb = int(p).to_bytes(w, "big")
    vb = int(v_max).to_bytes(max(1, (int(v_max).bit_length() + 7) // 8), "big")
    mu = ctypes.create_string_buffer(max(1, sectors * w))
    sg = ctypes.create_string_buffer(w)
    rc = lib().hbcpu_prove(pb, len(pb), sectors, key, len(key), chunks, vb, len(vb), ntags, tags_addr, data_addr,
                           length, threads, mu, sg)
    if rc:
        raise RuntimeError("hbcpu_prove error %d" % rc)
    return ([int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(sectors)],
            int.from_bytes(sg.raw, "big"))


def prove(p, sectors, key, chunks, v_max, tags, data, threads=1):
    """prove_raw on a list of int tags and a bytes object."""
    w = (int(p).bit_length() + 7) // 8
    traw = ctypes.create_string_buffer(b"".join(int(t).to_bytes(w, "big") for t in tags), max(1, len(tags) * w))
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    return prove_raw(p, sectors, key, chunks, v_max, len(tags), ctypes.addressof(traw),
                     ctypes.addressof(buf), len(data), threads)
