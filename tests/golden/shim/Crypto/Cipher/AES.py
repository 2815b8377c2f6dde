"""PyCrypto-compatible ``Crypto.Cipher.AES`` backed by OpenSSL EVP (ctypes)."""
import ctypes

MODE_ECB = 1
MODE_CBC = 2
MODE_CFB = 3
block_size = 16
key_size = (16, 24, 32)

_lib = ctypes.CDLL("libcrypto.so.3")
_lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
_lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_char_p, ctypes.c_char_p]
_lib.EVP_DecryptInit_ex.argtypes = _lib.EVP_EncryptInit_ex.argtypes
_lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                   ctypes.c_char_p, ctypes.c_int]
_lib.EVP_DecryptUpdate.argtypes = _lib.EVP_EncryptUpdate.argtypes
_lib.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
for _n in ("EVP_aes_128_cfb8", "EVP_aes_192_cfb8", "EVP_aes_256_cfb8",
           "EVP_aes_128_cfb128", "EVP_aes_192_cfb128", "EVP_aes_256_cfb128",
           "EVP_aes_128_ecb", "EVP_aes_192_ecb", "EVP_aes_256_ecb"):
    getattr(_lib, _n).restype = ctypes.c_void_p


def _as_bytes(x):
    if isinstance(x, str):
        return x.encode("latin-1")
    return bytes(x)


class _Cipher(object):
    def __init__(self, key, mode, iv, segment_size):
        key = _as_bytes(key)
        if len(key) not in key_size:
            raise ValueError("AES key must be either 16, 24, or 32 bytes long")
        bits = len(key) * 8
        if mode == MODE_CFB:
            if segment_size == 8:
                ev = getattr(_lib, "EVP_aes_%d_cfb8" % bits)()
            elif segment_size == 128:
                ev = getattr(_lib, "EVP_aes_%d_cfb128" % bits)()
            else:
                raise ValueError("unsupported segment size")
            iv = _as_bytes(iv) if iv is not None else b"\0" * 16
            if len(iv) != 16:
                raise ValueError("IV must be 16 bytes long")
        elif mode == MODE_ECB:
            ev = getattr(_lib, "EVP_aes_%d_ecb" % bits)()
            iv = None
        else:
            raise ValueError("unsupported mode")
        self._enc = _lib.EVP_CIPHER_CTX_new()
        self._dec = _lib.EVP_CIPHER_CTX_new()
        assert _lib.EVP_EncryptInit_ex(self._enc, ev, None, key, iv) == 1
        assert _lib.EVP_DecryptInit_ex(self._dec, ev, None, key, iv) == 1
        _lib.EVP_CIPHER_CTX_set_padding(self._enc, 0)
        _lib.EVP_CIPHER_CTX_set_padding(self._dec, 0)
        self.block_size = block_size
        self.IV = iv

    def _run(self, fn, ctx, data):
        data = _as_bytes(data)
        out = ctypes.create_string_buffer(len(data) + 32)
        n = ctypes.c_int(0)
        assert fn(ctx, out, ctypes.byref(n), data, len(data)) == 1
        return out.raw[:n.value]

    def encrypt(self, data):
        return self._run(_lib.EVP_EncryptUpdate, self._enc, data)

    def decrypt(self, data):
        return self._run(_lib.EVP_DecryptUpdate, self._dec, data)

    def __del__(self):
        try:
            _lib.EVP_CIPHER_CTX_free(self._enc)
            _lib.EVP_CIPHER_CTX_free(self._dec)
        except Exception:
            pass


def new(key, mode=MODE_ECB, IV=None, **kw):
    # PyCrypto 2.6.1: CFB segment_size defaults to 8 bits
    if "iv" in kw:
        IV = kw.pop("iv")
    return _Cipher(key, mode, IV, kw.get("segment_size", 8))
