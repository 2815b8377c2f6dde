"""Pure-Python restatement of the reference PySwizzle encode loop -- the
"PySwizzle" CPU-baseline row of BASELINE.md section 3 / SURVEY.md 8(d).

TEST / MEASUREMENT INFRASTRUCTURE ONLY: imported by tests/ and the
cpu_baseline leg of bench.py, never by the product package.

It keeps the reference's algorithmic cost, so its rate stands in for the
reference PySwizzle on the box's host cores (the reference itself never
travels to the GPU box, and PyCrypto is not installed anywhere):

* KeyedPRF.eval (heartbeat/util.py:83-96): a NEW AES cipher (key schedule)
  per eval, CFB with 8-bit segments and IV 0^16 over pad(SHA256(str(x)), nb),
  masked, rejection sampled with the stream continuing across tries;
* PySwizzle.encode (heartbeat/PySwizzle/PySwizzle.py:279-314): one
  f.eval(chunk_id) per block, alpha.eval(j) recomputed for EVERY sector,
  Python int multiply-accumulate, file.read(sectorsize) per sector, break at
  the first short read, sigma %= p.

AES-CFB8 comes from OpenSSL's libcrypto via ctypes (the survey's calibration of
the reference used the same backend, so PyCrypto 2.6.1 itself would be no
faster).  Pinned against the golden vectors in tests/test_oracle.py.
"""
import ctypes
import ctypes.util
import hashlib

_lib = None


def _crypto():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(name)
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_char_p, ctypes.c_char_p]
        L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                        ctypes.c_char_p, ctypes.c_int]
        for n in ("EVP_aes_128_cfb8", "EVP_aes_192_cfb8", "EVP_aes_256_cfb8"):
            getattr(L, n).restype = ctypes.c_void_p
        _lib = L
    return _lib


class _CFB8(object):
    """AES-CFB8 encryptor with IV 0^16 (PyCrypto AES.new(key, MODE_CFB, '\\0'*16))."""

    def __init__(self, key):
        L = _crypto()
        ev = getattr(L, "EVP_aes_%d_cfb8" % (8 * len(key)))()
        self._ctx = L.EVP_CIPHER_CTX_new()
        L.EVP_EncryptInit_ex(self._ctx, ev, None, key, b"\0" * 16)

    def encrypt(self, data):
        out = ctypes.create_string_buffer(len(data) + 16)
        n = ctypes.c_int(0)
        _crypto().EVP_EncryptUpdate(self._ctx, out, ctypes.byref(n), data, len(data))
        return out.raw[:n.value]

    def __del__(self):
        try:
            _crypto().EVP_CIPHER_CTX_free(self._ctx)
        except Exception:
            pass


class KeyedPRF(object):
    """util.py:44-96."""

    @staticmethod
    def pad(data, length):
        if len(data) > length:
            return data[0:length]
        return data + b"\0" * (length - len(data))

    def __init__(self, key, range):
        self.key = key
        self.range = range
        self.bits = int(range).bit_length()
        self.mask = (1 << self.bits) - 1
        self.nb = (self.bits + 7) // 8

    def eval(self, x):
        aes = _CFB8(self.key)                                    # util.py:88, per eval
        data = self.pad(hashlib.sha256(str(x).encode()).digest(), self.nb)
        while True:
            num = self.mask & int.from_bytes(aes.encrypt(data), "big")
            if num < self.range:
                return num


def encode(p, sectors, f_key, alpha_key, file):
    """PySwizzle.encode's loop (PySwizzle.py:290-311): the tags of `file` from
    its current position, as a list of ints."""
    sectorsize = p.bit_length() // 8
    f = KeyedPRF(f_key, p)
    alpha = KeyedPRF(alpha_key, p)
    sigmas = []
    done = False
    chunk_id = 0
    while not done:
        sigma = f.eval(chunk_id)
        for j in range(0, sectors):
            buffer = file.read(sectorsize)
            if len(buffer) > 0:
                sigma += alpha.eval(j) * int.from_bytes(buffer, "big")
            if len(buffer) != sectorsize:
                done = True
                break
        sigma %= p
        sigmas.append(sigma)
        chunk_id += 1
    return sigmas


def prove(p, sectors, file, chal_key, chunks, v_max, tags):
    """PySwizzle.prove's loops (PySwizzle.py:333-370): (mu list, sigma).  Like
    the reference, index.eval(i) and v.eval(i) are recomputed for every sector
    and again for sigma, and the file is read by seek/read per sector."""
    sectorsize = p.bit_length() // 8
    chunk_size = sectors * sectorsize
    index = KeyedPRF(chal_key, len(tags))
    v = KeyedPRF(chal_key, v_max)
    mu = [0] * sectors
    sigma = 0
    for i in range(0, chunks):
        for j in range(0, sectors):
            pos = index.eval(i) * chunk_size + j * sectorsize
            file.seek(pos)
            buffer = file.read(sectorsize)
            if len(buffer) > 0:
                mu[j] += v.eval(i) * int.from_bytes(buffer, "big")
            if len(buffer) != sectorsize:
                break
    for j in range(0, sectors):
        mu[j] %= p
    for i in range(0, chunks):
        sigma += v.eval(i) * tags[index.eval(i)]
    sigma %= p
    return mu, sigma


def verify(p, sectors, f_key, alpha_key, nchunks, chal_key, chunks, v_max, mu, sigma):
    """PySwizzle.verify's check (PySwizzle.py:372-395)."""
    index = KeyedPRF(chal_key, nchunks)
    v = KeyedPRF(chal_key, v_max)
    f = KeyedPRF(f_key, p)
    alpha = KeyedPRF(alpha_key, p)
    rhs = 0
    for i in range(0, chunks):
        rhs += v.eval(i) * f.eval(index.eval(i))
    for j in range(0, sectors):
        rhs += alpha.eval(j) * mu[j]
    return sigma == rhs % p
