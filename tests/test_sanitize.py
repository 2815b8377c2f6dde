"""ASan + UBSan over the CPU builds: the lane emulator
(tests/emul/emul.cpp = hb_lane.hpp as plain C++) and the C oracle
(oracle/swizzle_oracle.c) linked into one executable with
-fsanitize=address,undefined and no recovery, run over PRF / cxx-PRF / encode
inputs that also cross-check the two (tests/emul/sanitize_main.cpp)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_emul_and_oracle_under_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    objs = []
    for src, cc, std in [(os.path.join(HERE, "emul", "emul.cpp"), "g++", "-std=c++17"),
                         (os.path.join(HERE, "emul", "sanitize_main.cpp"), "g++", "-std=c++17"),
                         (os.path.join(ROOT, "oracle", "swizzle_oracle.c"), "gcc", "-std=gnu11")]:
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        subprocess.check_call([cc, std, *san, "-c", src, "-o", obj])
        objs.append(obj)
    exe = str(tmp_path / "sanitize")
    subprocess.check_call(["g++", *san, *objs, "-o", exe, "-lcrypto", "-lpthread"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
