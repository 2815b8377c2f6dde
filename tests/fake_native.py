"""A CPU stand-in for libhbswizzle.so, for testing bench.py's Python plumbing
without a GPU (TEST INFRASTRUCTURE ONLY; never importable by the product).

"Device" memory is host memory; hb_encode / hb_prove delegate to the CPU
oracle (oracle/swizzle_oracle.c), so tags and proofs are the real ones and the
bench's own cross-checks (parity sample, CPU baseline, host-path equality,
device-vs-API proof) are exercised for real.  Only the entry points bench.py
and heartbeat_amd's Python layer call are provided."""
import ctypes

import numpy as np

from conftest import splitmix_bytes


def _v(x):
    """Address / integer out of a ctypes object, a ctypes buffer or an int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "value") and not isinstance(x, (bytes, bytearray)) and not hasattr(x, "raw"):
        return x.value
    return ctypes.addressof(x)


def _set(ref, value):
    if ref is not None:
        ref._obj.value = value


class FakeLib(object):
    def __init__(self):
        self.bufs = {}
        self.encodes = []          # (flags, nblocks) of every hb_encode
        self.registered = set()

    # --- context / build
    def hb_ctx_create(self, device, ref):
        _set(ref, 1 + device)
        return 0

    def hb_ctx_destroy(self, h):
        pass

    def hb_ctx_prepare(self, h, bits):
        return 0

    def hb_last_error(self, h):
        return b"fake"

    def hb_device_count(self, ref):
        _set(ref, 1)
        return 0

    def hb_device_pci_bus_id(self, device, buf, n):
        ctypes.memmove(buf, b"0000:00:00.0\0", 13)
        return 0

    def hb_build_id(self):
        return b"0" * 64

    def hb_build_flags(self):
        return 0

    def hb_test_switches(self):
        return 0

    def hb_last_kernel_ms(self, h, ms, n):
        _set(ms, 1.0)
        _set(n, 3)
        return 0

    def hb_last_kernel_phases(self, h, ms, n):
        for k in range(min(int(n), 4)):
            ms[k] = 0.25
        return min(int(n), 4)

    def hb_ctx_num_cus(self, h, ref):
        _set(ref, 256)
        return 0

    # --- memory
    def hb_device_malloc(self, h, nbytes, ref):
        a = np.zeros(max(int(nbytes), 16), dtype=np.uint8)
        addr = a.ctypes.data
        self.bufs[addr] = a
        _set(ref, addr)
        return 0

    def hb_device_free(self, h, p):
        self.bufs.pop(_v(p), None)
        return 0

    def hb_memcpy(self, h, dst, src, n, kind):
        ctypes.memmove(_v(dst), _v(src), int(n))
        return 0

    def hb_fill_random(self, h, p, n, seed):
        b = splitmix_bytes(int(seed), 0, int(n))
        ctypes.memmove(_v(p), b, len(b))
        return 0

    def hb_stream_read(self, h, p, n, ms):
        _set(ms, 1.0)
        return 0

    def hb_host_register(self, h, p, n):
        self.registered.add(_v(p))
        return 0

    def hb_host_unregister(self, h, p):
        self.registered.discard(_v(p))
        return 0

    # --- compute (the CPU oracle)
    def hb_encode(self, h, pb, plen, S, fk, ak, klen, block_base, data, length, nblocks, tags, flags, tries):
        from oracle import oracle as O
        p = int.from_bytes(bytes(pb[:plen]), "big")
        rc = O.encode_raw(p, S, bytes(fk[:klen]), bytes(ak[:klen]), _v(data) or 0, int(length), int(block_base),
                          int(nblocks), _v(tags), 4)
        self.encodes.append((int(flags), int(nblocks)))
        _set(tries, int(nblocks))
        return rc

    def hb_prove_range(self, h, pb, plen, S, key, klen, chunks, i0, i1, vb, vlen, tags, ntags, data, length,
                       flags, mu, sg):
        from oracle import oracle as O
        if not (i0 == 0 and i1 >= chunks):
            raise NotImplementedError("the fake proves whole challenges only")
        w = (int.from_bytes(bytes(pb[:plen]), "big").bit_length() + 7) // 8
        return O.lib().hbo_prove(bytes(pb[:plen]), plen, S, bytes(key[:klen]), klen, chunks, bytes(vb[:vlen]), vlen,
                                 ntags, ctypes.cast(_v(tags), ctypes.c_char_p), w, _v(data) or 0, int(length), mu, sg)

    def hb_verify_rhs(self, h, pb, plen, S, fk, ak, klen, nchunks, key, kl2, chunks, vb, vlen, mu, rhs):
        """sum_i v_i F(idx_i) + sum_j alpha_j mu_j mod p (PySwizzle.py:380-395)
        from the oracle's KeyedPRF, memoised per argument set."""
        from oracle import oracle as O
        p = int.from_bytes(bytes(pb[:plen]), "big")
        w = (p.bit_length() + 7) // 8
        arg = (bytes(pb[:plen]), S, bytes(fk[:klen]), bytes(ak[:klen]), nchunks, bytes(key[:kl2]), chunks,
               bytes(vb[:vlen]), bytes(mu[:S * w]))
        memo = self.__dict__.setdefault("_rhs", {})
        if arg not in memo:
            vmax = int.from_bytes(bytes(vb[:vlen]), "big")
            r = 0
            for i in range(chunks):
                ix = O.prf_eval(arg[5], nchunks, i)
                r += O.prf_eval(arg[5], vmax, i) * O.prf_eval(arg[2], p, ix)
            for j in range(S):
                r += O.prf_eval(arg[3], p, j) * int.from_bytes(arg[8][j * w:(j + 1) * w], "big")
            memo[arg] = r % p
        ctypes.memmove(rhs, memo[arg].to_bytes(w, "big"), w)
        return 0

    def hb_prove(self, h, pb, plen, S, key, klen, chunks, vb, vlen, tags, ntags, data, length, flags, mu, sg):
        return self.hb_prove_range(h, pb, plen, S, key, klen, chunks, 0, chunks, vb, vlen, tags, ntags, data,
                                   length, flags, mu, sg)


def install(monkeypatch):
    """Make heartbeat_amd._native use a FakeLib; returns it."""
    from heartbeat_amd import _native
    fake = FakeLib()
    monkeypatch.setattr(_native, "_lib", fake)
    monkeypatch.setattr(_native, "_ctxs", {})
    return fake
