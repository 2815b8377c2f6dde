"""ctypes binding of libhbswizzle.so (C ABI: include/hbswizzle.h).

The library must have been built (``heartbeat_amd.build.build()`` or
``python __graft_entry__.py``); importing the compute entry points without it,
or calling them without a usable gfx950 GPU, raises HeartbeatError.  There is
no CPU fallback for encode / prove / verify / KeyedPRF.
"""
import ctypes
import os
import threading

from .exc import HeartbeatError

HERE = os.path.dirname(os.path.abspath(__file__))
# HB_LIB_PATH selects an alternative build (A/B experiments); default: in-tree
LIB_PATH = os.environ.get("HB_LIB_PATH") or os.path.join(HERE, "libhbswizzle.so")

HB_DATA_ON_DEVICE = 1
HB_TAGS_ON_DEVICE = 2
HB_ENCODE_SINGLE_PASS = 4
HB_EUNSUPPORTED = -4
HB_PRF_CXX = 8
HB_ASYNC = 16
HB_HOST_REGISTER = 32
HB_BUILD_EXPERIMENT = 1
HB_BUILD_TEST_SWITCHES = 2

_lib = None
_lib_lock = threading.Lock()
_ctx_lock = threading.Lock()
_ctxs = {}

# (name, restype, argtypes) for every symbol of include/hbswizzle.h
_c = ctypes
_P = _c.c_void_p
_B = _c.c_char_p
SIGNATURES = [
    ("hb_abi_version", _c.c_int, []),
    ("hb_build_flags", _c.c_int, []),
    ("hb_build_id", _c.c_char_p, []),
    ("hb_build_flags_string", _c.c_char_p, []),
    ("hb_test_switches", _c.c_uint32, []),
    ("hb_device_count", _c.c_int, [_c.POINTER(_c.c_int)]),
    ("hb_device_pci_bus_id", _c.c_int, [_c.c_int, _P, _c.c_size_t]),
    ("hb_ctx_create", _c.c_int, [_c.c_int, _c.POINTER(_P)]),
    ("hb_ctx_destroy", None, [_P]),
    ("hb_last_error", _c.c_char_p, [_P]),
    ("hb_width", _c.c_size_t, [_B, _c.c_size_t]),
    ("hb_prf_eval", _c.c_int, [_P, _B, _c.c_size_t, _B, _c.c_size_t, _P, _c.c_size_t, _P]),
    ("hb_prf_eval_digests", _c.c_int, [_P, _B, _c.c_size_t, _B, _c.c_size_t, _B, _c.c_size_t, _P]),
    ("hb_encode", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint32, _B, _B, _c.c_size_t, _c.c_uint64,
                             _P, _c.c_uint64, _c.c_uint64, _P, _c.c_uint32,
                             _c.POINTER(_c.c_uint64)]),
    ("hb_block_count", _c.c_uint64, [_B, _c.c_size_t, _c.c_uint32, _c.c_uint64]),
    ("hb_prove", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint32, _B, _c.c_size_t, _c.c_uint64, _B,
                            _c.c_size_t, _P, _c.c_uint64, _P, _c.c_uint64, _c.c_uint32, _P, _P]),
    ("hb_prove_range", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint32, _B, _c.c_size_t, _c.c_uint64,
                                  _c.c_uint64, _c.c_uint64, _B, _c.c_size_t, _P, _c.c_uint64, _P,
                                  _c.c_uint64, _c.c_uint32, _P, _P]),
    ("hb_verify_rhs", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint32, _B, _B, _c.c_size_t,
                                 _c.c_uint64, _B, _c.c_size_t, _c.c_uint64, _B, _c.c_size_t,
                                 _B, _P]),
    ("hb_cxx_verify_rhs", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint32, _B, _B, _c.c_size_t,
                                     _c.c_uint64, _B, _c.c_size_t, _c.c_uint64, _B, _c.c_size_t,
                                     _B, _P]),
    ("hb_aes_cfb8", _c.c_int, [_B, _c.c_size_t, _B, _B, _P, _c.c_size_t, _c.c_int]),
    ("hb_aes_cfb128", _c.c_int, [_B, _c.c_size_t, _B, _B, _P, _c.c_size_t, _c.c_int]),
    ("hb_last_kernel_ms", _c.c_int, [_P, _c.POINTER(_c.c_double), _c.POINTER(_c.c_uint32)]),
    ("hb_device_malloc", _c.c_int, [_P, _c.c_uint64, _c.POINTER(_P)]),
    ("hb_device_free", _c.c_int, [_P, _P]),
    ("hb_memcpy", _c.c_int, [_P, _P, _P, _c.c_uint64, _c.c_int]),
    ("hb_cxx_prf_eval", _c.c_int, [_P, _B, _c.c_size_t, _B, _c.c_size_t, _P, _c.c_size_t, _P]),
    ("hb_host_register", _c.c_int, [_P, _P, _c.c_uint64]),
    ("hb_host_unregister", _c.c_int, [_P, _P]),
    ("hb_fill_random", _c.c_int, [_P, _P, _c.c_uint64, _c.c_uint64]),
    ("hb_stream_read", _c.c_int, [_P, _P, _c.c_uint64, _c.POINTER(_c.c_double)]),
    ("hb_ctx_set_stream", _c.c_int, [_P, _P]),
    ("hb_ctx_wait", _c.c_int, [_P, _c.POINTER(_c.c_uint64)]),
    ("hb_ctx_prepare", _c.c_int, [_P, _c.c_uint32]),
    ("hb_ctx_num_cus", _c.c_int, [_P, _c.POINTER(_c.c_int)]),
    ("hb_last_kernel_phases", _c.c_int, [_P, _c.POINTER(_c.c_double), _c.c_uint32]),
    ("hb_merkle_offsets", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint64, _c.c_uint64, _c.c_uint64, _P]),
    ("hb_merkle_chunk_hmacs", _c.c_int, [_P, _B, _c.c_size_t, _c.c_uint64, _P, _c.c_uint64, _P,
                                         _c.c_uint64, _P]),
]


_PROVENANCE = ("hb_build_id", "hb_build_flags_string", "hb_test_switches")


def lib():
    """The loaded library (raises HeartbeatError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HeartbeatError(
                    "libhbswizzle.so is not built (%s); run heartbeat_amd.build.build()" % LIB_PATH)
            L = ctypes.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                if not hasattr(L, name) and (os.environ.get("HB_LIB_PATH") or name in _PROVENANCE):
                    continue   # an A/B experiment build from before this entry point, or a
                               # library without provenance (refused by check_build_id)
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            flags = L.hb_build_flags() if hasattr(L, "hb_build_flags") else 0
            if not os.environ.get("HB_LIB_PATH"):
                if flags & HB_BUILD_EXPERIMENT:
                    raise HeartbeatError("%s is an experiment build (HB_EXP_* switches may emit wrong "
                                         "tags); rebuild the product library" % LIB_PATH)
                check_build_id(L)
            _lib = L
    return _lib


def check_build_id(L, root=None):
    """Refuse a library that was not built from the sources of the tree at
    `root` (default: the tree this package sits in): its hb_build_id() must
    equal build_id.library_id(SHA-256 of the tree's csrc/ + include/hbswizzle.h,
    the library's compiler flags).  Content hashes, so a touched but unchanged
    tree still matches, and a stale or hand-restored binary does not.  Returns
    the id."""
    from . import build_id as B
    if not hasattr(L, "hb_build_id"):
        raise HeartbeatError("%s has no build id (built before provenance stamping); rebuild it" % LIB_PATH)
    got = L.hb_build_id().decode("ascii", "replace")
    want = B.library_id(B.sources_digest(root), L.hb_build_flags_string().decode("ascii", "replace"))
    if got != want:
        raise HeartbeatError("%s was built from other sources than the tree at %s (library id %s, tree %s); "
                             "rebuild it (heartbeat_amd.build.build())" % (
                                 LIB_PATH, root or os.path.dirname(HERE), got[:16], want[:16]))
    return got


def build_info():
    """Provenance of the loaded library, for bench lines and smoke()."""
    L = lib()
    return {"build_id": L.hb_build_id().decode("ascii", "replace") if hasattr(L, "hb_build_id") else None,
            "build_flags": int(L.hb_build_flags()),
            "test_switches": int(L.hb_test_switches()) if hasattr(L, "hb_test_switches") else None}


def pci_bus_id(device):
    """PCI bus id of a device (None if it cannot be queried)."""
    buf = ctypes.create_string_buffer(64)
    if lib().hb_device_pci_bus_id(int(device), buf, 64) != 0:
        return None
    return buf.value.decode("ascii", "replace")


def default_device():
    for var in ("HB_DEVICE", "LOCAL_RANK"):
        if os.environ.get(var, "").strip():
            return int(os.environ[var])
    return 0


class Context(object):
    """One libhbswizzle context (stream + scratch) on one GPU."""

    def __init__(self, device):
        L = lib()
        h = ctypes.c_void_p()
        rc = L.hb_ctx_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise HeartbeatError("cannot open GPU %d: %s" % (
                device, L.hb_last_error(None).decode("utf-8", "replace")))
        self.h = h
        self.device = int(device)
        self.lock = threading.Lock()

    def check(self, rc):
        if rc != 0:
            raise HeartbeatError(lib().hb_last_error(self.h).decode("utf-8", "replace"))

    def prepare(self, prime_bits):
        """Load the GPU code that encodes / proves with a prime of this size
        launch (hb_ctx_prepare), so that the first such call does not pay it.
        A no-op for an experiment build from before this entry point."""
        L = lib()
        if not hasattr(L, "hb_ctx_prepare"):
            return
        with self.lock:
            self.check(L.hb_ctx_prepare(self.h, int(prime_bits)))

    def last_kernel_phases(self):
        """[set-up, first pass, retry pass, wide MAC] ms of the last
        device-resident two-pass encode (hb_last_kernel_phases), or []."""
        ms = (ctypes.c_double * 4)()
        with self.lock:
            n = lib().hb_last_kernel_phases(self.h, ms, 4)
        if n < 0:
            self.check(n)
        return [round(ms[k], 4) for k in range(n)]

    def num_cus(self):
        """Compute units of the context's GPU (hb_ctx_num_cus)."""
        n = ctypes.c_int()
        self.check(lib().hb_ctx_num_cus(self.h, ctypes.byref(n)))
        return n.value

    def last_kernel_ms(self):
        ms = ctypes.c_double()
        n = ctypes.c_uint32()
        with self.lock:   # it may settle a pending async encode (hb_last_kernel_ms)
            lib().hb_last_kernel_ms(self.h, ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def close(self):
        if self.h:
            lib().hb_ctx_destroy(self.h)
            self.h = None


def context(device=None, instance=0):
    """The process-wide context for `device` (default: $HB_DEVICE, $LOCAL_RANK
    or 0); `instance` > 0 opens further independent contexts on the same
    device (multi.py uses them for repeated device entries)."""
    d = default_device() if device is None else int(device)
    key = (d, int(instance))
    c = _ctxs.get(key)
    if c is None:
        lib()
        with _ctx_lock:
            c = _ctxs.get(key)
            if c is None:
                c = Context(d)
                _ctxs[key] = c
    return c


def be(n, width=None):
    n = int(n)
    if width is None:
        width = max(1, (n.bit_length() + 7) // 8)
    return n.to_bytes(width, "big")


def width_of(p):
    return (int(p).bit_length() + 7) // 8


def aes_cfb128(key, iv, data, encrypt):
    """Host AES-CFB128 (cxx State encrypt-and-sign, shacham_waters_private.cxx:169-306)."""
    key = bytes(key)
    iv = bytes(iv)
    data = bytes(data)
    out = ctypes.create_string_buffer(max(1, len(data)))
    rc = lib().hb_aes_cfb128(key, len(key), iv, data, out, len(data), 1 if encrypt else 0)
    if rc != 0:
        raise HeartbeatError("AES key must be either 16, 24, or 32 bytes long")
    return out.raw[:len(data)]


def aes_cfb8(key, iv, data, encrypt):
    """Host AES-CFB8 (State encryption, PySwizzle.py:162-195)."""
    key = bytes(key)
    iv = bytes(iv)
    data = bytes(data)
    if len(iv) != 16:
        raise HeartbeatError("IV must be 16 bytes long")
    out = ctypes.create_string_buffer(max(1, len(data)))
    rc = lib().hb_aes_cfb8(key, len(key), iv, data, out, len(data), 1 if encrypt else 0)
    if rc != 0:
        raise HeartbeatError("AES key must be either 16, 24, or 32 bytes long")
    return out.raw[:len(data)]
