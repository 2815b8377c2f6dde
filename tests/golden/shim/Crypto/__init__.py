"""Offline stand-in for the PyCrypto 2.6.1 API surface that the reference
PySwizzle imports (``heartbeat/PySwizzle/PySwizzle.py:26-30``,
``heartbeat/util.py:25-27``).

Test infrastructure only: used by ``tests/golden/make_golden.py`` to run the
reference PySwizzle in the build container and record golden vectors.  It is
never imported by the product (``heartbeat_amd``) and never used on the GPU box.

Backends: OpenSSL ``libcrypto.so.3`` (AES via EVP, ctypes) and the Python
standard library (hashlib / hmac).  PyCrypto semantics that matter here:
``AES.new(key, MODE_CFB, iv)`` defaults to segment_size=8 (CFB-8), accepts a
``str`` IV, and keeps the cipher stream across ``encrypt`` calls.
"""
