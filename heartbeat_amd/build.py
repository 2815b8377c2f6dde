"""Build libhbswizzle.so (gfx950) in-tree: heartbeat_amd/libhbswizzle.so."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs=8, verbose=False):
    cmd = ["make", "-C", os.path.join(HERE, "csrc"), "-j%d" % jobs]
    if not verbose:
        cmd.insert(1, "-s")
    subprocess.check_call(cmd)
    return os.path.join(HERE, "libhbswizzle.so")


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
