import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The GPU tests that select engine / MAC variants or shrink buffers through
# environment switches (HB_NO_QUAD, HB_MFMA_*, HB_TEST_*) need the gate open
# when their context is created: libhbswizzle reads HB_ENABLE_TEST_SWITCHES
# once per context and ignores every switch without it (hb_runtime.cpp).
# Opened for the test session only; bench.py and smoke() never set it.  The
# CPU test of the gate (test_provenance.py) closes it itself.
os.environ["HB_ENABLE_TEST_SWITCHES"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def golden_prf():
    return load_golden("prf_kat.json")


@pytest.fixture(scope="session")
def golden_encode():
    return load_golden("encode_cases.json")


@pytest.fixture(scope="session")
def golden_files():
    return load_golden("file_cases.json")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


def test6_bytes():
    line = b"abcdefghijklmnopqrstuvwxyz1234567890\n"
    return (line * (999999 // len(line) + 1))[:999999]


def fixture_file(name):
    if name == "test6.txt":
        return test6_bytes()
    with open(os.path.join(GOLDEN, "files", name), "rb") as fh:
        return fh.read()


def splitmix_bytes(seed, start, n):
    """Host copy of the device synthetic stream (hb_fill_random)."""
    import numpy as np
    M = (1 << 64) - 1
    out = bytearray()
    k = start - (start % 16)
    q0 = k // 16
    nq = (start + n - k + 15) // 16
    qs = np.arange(q0, q0 + nq, dtype=np.uint64)
    res = []
    for half in (0, 1):
        x = np.uint64(seed) ^ ((np.uint64(2) * qs + np.uint64(half)) * np.uint64(0xD1B54A32D192ED03))
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        res.append(x)
    words = np.stack(res, axis=1).reshape(-1)   # little-endian u64 pairs
    b = words.astype("<u8").tobytes()
    off = start - k
    return b[off:off + n]
