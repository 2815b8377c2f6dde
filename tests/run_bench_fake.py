"""Run bench.py's main() against tests/fake_native.py (the oracle-backed CPU
stand-in for libhbswizzle.so) -- TEST INFRASTRUCTURE ONLY, started by
tests/test_bench_cpu.py as the ranks of a multi-rank (gloo) run."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import fake_native  # noqa: E402
from heartbeat_amd import _native  # noqa: E402

_native._lib = fake_native.FakeLib()
_native._ctxs.clear()

import bench  # noqa: E402

if __name__ == "__main__":
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
