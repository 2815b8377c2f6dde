"""Provenance of libhbswizzle.so and the test-switch gate (CPU only).

* The library carries hb_build_id() = SHA-256 of its sources + flags
  (heartbeat_amd/build_id.py); heartbeat_amd._native refuses a library that
  does not match the tree it sits in.  A touched but unchanged tree still
  matches (content hashes); an edited source with the old library does not.
* csrc/Makefile keys every object group on a stamp holding the hash of its
  inputs, so objects left from another state of the tree -- mtimes newer than
  the sources, as after a revert with restored objects -- are rebuilt.
* The A/B and test switches are ignored unless HB_ENABLE_TEST_SWITCHES=1.
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def _copy_tree(dst, with_objects=False):
    """heartbeat_amd/{csrc, build_id.py} and include/ under dst (mtimes kept)."""
    src_csrc = os.path.join(ROOT, "heartbeat_amd", "csrc")
    ignore = None if with_objects else shutil.ignore_patterns("build", "build_*")
    shutil.copytree(src_csrc, os.path.join(dst, "heartbeat_amd", "csrc"), copy_function=shutil.copy2,
                    ignore=ignore)
    shutil.copy2(os.path.join(ROOT, "heartbeat_amd", "build_id.py"), os.path.join(dst, "heartbeat_amd"))
    os.makedirs(os.path.join(dst, "include"))
    shutil.copy2(os.path.join(ROOT, "include", "hbswizzle.h"), os.path.join(dst, "include"))


def test_library_id_matches_tree():
    from heartbeat_amd import _native
    L = _native.lib()
    got = _native.check_build_id(L)
    assert len(got) == 64 and int(got, 16) >= 0
    assert _native.build_info()["build_id"] == got


def test_touched_tree_matches_edited_tree_refused(tmp_path):
    from heartbeat_amd import HeartbeatError, _native
    L = _native.lib()
    _copy_tree(str(tmp_path))
    # touched, unchanged: still the same sources
    for dirpath, _, files in os.walk(str(tmp_path)):
        for f in files:
            os.utime(os.path.join(dirpath, f), None)
    assert _native.check_build_id(L, str(tmp_path)) == _native.check_build_id(L)
    # one source edited (a comment): the library is refused for that tree
    p = os.path.join(str(tmp_path), "heartbeat_amd", "csrc", "hb_runtime.cpp")
    with open(p, "a") as fh:
        fh.write("// edited\n")
    with pytest.raises(HeartbeatError) as ex:
        _native.check_build_id(L, str(tmp_path))
    assert "other sources" in str(ex.value)
    # the header counts too
    os.truncate(p, os.path.getsize(p) - len("// edited\n"))
    assert _native.check_build_id(L, str(tmp_path)) == _native.check_build_id(L)
    with open(os.path.join(str(tmp_path), "include", "hbswizzle.h"), "a") as fh:
        fh.write("\n")
    with pytest.raises(HeartbeatError):
        _native.check_build_id(L, str(tmp_path))


def test_stamp_written_only_on_change(tmp_path):
    tool = os.path.join(ROOT, "heartbeat_amd", "build_id.py")
    st = str(tmp_path / "b" / "x.id")
    subprocess.check_call(["python3", tool, "stamp", st, "abc"])
    os.utime(st, (1000, 1000))
    subprocess.check_call(["python3", tool, "stamp", st, "abc"])
    assert os.stat(st).st_mtime == 1000          # same content: untouched
    subprocess.check_call(["python3", tool, "stamp", st, "abd"])
    assert os.stat(st).st_mtime > 1000 and open(st).read().strip() == "abd"


def test_restored_objects_do_not_satisfy_make(tmp_path):
    """A copy of the built tree: `make -n` has nothing to do.  Then the
    stamps are made to hold another tree state's hashes (objects restored
    from a reverted experiment keep their newer mtimes, but their stamps
    record other inputs): make wants to recompile those objects."""
    csrc = os.path.join(ROOT, "heartbeat_amd", "csrc")
    if not os.path.exists(os.path.join(csrc, "build", "hb_kern_nl8.id")):
        pytest.skip("library not built with provenance stamps")
    _copy_tree(str(tmp_path), with_objects=True)
    shutil.copy2(os.path.join(ROOT, "heartbeat_amd", "libhbswizzle.so"), os.path.join(str(tmp_path), "heartbeat_amd"))
    tcsrc = os.path.join(str(tmp_path), "heartbeat_amd", "csrc")
    r = subprocess.run(["make", "-n", "-C", tcsrc], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "hipcc" not in r.stdout, r.stdout
    for stamp in ("hb_kern_nl8.id", "rt.id"):
        p = os.path.join(tcsrc, "build", stamp)
        with open(p, "w") as fh:
            fh.write("0" * 64 + "\n")
        os.utime(p, (1000, 1000))                   # older than every object
    r = subprocess.run(["make", "-n", "-C", tcsrc], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "hb_runtime.cpp" in r.stdout and "hb_kern_nl8.hip" in r.stdout, r.stdout


def test_switches_ignored_without_gate(monkeypatch):
    from heartbeat_amd import _native
    L = _native.lib()
    monkeypatch.delenv("HB_ENABLE_TEST_SWITCHES", raising=False)
    for name in ("HB_NO_QUAD", "HB_NO_MFMA", "HB_MFMA_LINE32", "HB_TEST_NO_EARLY_LIST", "HB_TEST_PROVE_BATCH",
                 "HB_MFMA_MIN_S", "HB_TRACE_PHASES", "HB_NO_PROVE_FUSE", "HB_NO_VERIFY_FUSE", "HB_NO_SMALL_ENCODE",
                 "HB_MID_BLOCKS", "HB_NO_WIDE", "HB_WMAC_WPE", "HB_WIDE_SYNC_ALPHA", "HB_QCHUNK"):
        monkeypatch.setenv(name, "1")
    assert L.hb_test_switches() == 0
    assert L.hb_build_flags() & _native.HB_BUILD_TEST_SWITCHES == 0
    monkeypatch.setenv("HB_ENABLE_TEST_SWITCHES", "1")
    m = L.hb_test_switches()
    assert m & 1 and m & 2 and m & 8 and m & 32 and m & 128 and m & 16 and m & 256   # HB_SW_* (hbswizzle.h)
    assert m & 8192 and m & 32768 and m & 65536 and m & 262144
    assert m & 524288 and m & 1048576 and m & 2097152 and m & 4194304   # round 6: wide encode, queue refills
    assert L.hb_build_flags() & _native.HB_BUILD_TEST_SWITCHES
    monkeypatch.setenv("HB_ENABLE_TEST_SWITCHES", "yes")   # only "1" opens the gate
    assert L.hb_test_switches() == 0
