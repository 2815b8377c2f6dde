"""bench.py's whole N = 1 encode path on the CPU, through a stand-in for the
native library (tests/fake_native.py: "device" memory is host memory and
hb_encode / hb_prove are the CPU oracle).  Catches plumbing errors in the
legs the driver runs -- timed loop, sustained leg, parity sample, CPU rows,
host-memory rows, JSON line -- before they cost a GPU run.  Numbers are
meaningless here; only the structure and the built-in cross-checks are
asserted."""
import json
import os
import socket
import subprocess
import sys

import pytest

import fake_native
from conftest import ROOT


@pytest.fixture
def fake(monkeypatch):
    return fake_native.install(monkeypatch)


def _run_bench(monkeypatch, capsys, *argv):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"] + list(argv))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    bench.main()
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def test_default_encode_line_with_every_leg(fake, monkeypatch, capsys, tmp_path):
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    monkeypatch.setenv("OMP_NUM_THREADS", "4")
    d = _run_bench(monkeypatch, capsys, "--gib", "0.001", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.3",
                   "--py-seconds", "0.2", "--sustain-seconds", "0.05", "--parity-blocks", "100",
                   "--prove-proofs", "2")
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["unit"] == "GiB/s"
    assert "[--gib 0.001" in d["config"]["workload"]
    assert d["parity_sample"]["ok"] is True
    assert d["cpu_baseline"]["tags_equal_gpu"] is True
    assert d["cpu_baseline"]["oracle_row"]["tags_equal_gpu"] is True
    assert d["sustained"]["steps"] >= 1
    pr = d["prove"]
    assert pr["proof_equal_oracle"] is True and pr["cpu_native_equal_gpu"] is True and pr["proofs"] == 2
    assert pr["workload"].startswith("configs[4]")
    assert pr["verify"]["verified"] is True
    assert d["build"]["build_id"] == "0" * 64
    for row, bits in (("wide", 1024), ("configs1", 256)):
        r = d[row]
        assert r["parity_sample"]["ok"] is True and r["value"] > 0 and r["aes_per_block"] > 0, row
        assert r["workload"].startswith("%d-bit" % bits) and set(r["phases_ms"]) and r["roofline"]["frac"] > 0
    wp = d["wide"]["prove"]
    assert wp["proof_equal_oracle"] is True and wp["verify"]["verified"] is True and wp["ms_per_proof"] > 0
    assert "prove" not in d["configs1"]
    n = d["config"]["file_bytes_per_rank"]
    assert d["wide"]["blocks"] == n // 1280 + 1 and d["configs1"]["blocks"] == n // 32 + 1
    hp = d["host_path"]
    assert hp["raw_tags_equal"] is True and hp["api_tags_equal"] is True
    assert hp["api_prove_file"]["equal_device_resident_proof"] is True
    for k in ("raw_pageable_gib_s", "raw_register_windows_gib_s", "raw_pinned_gib_s", "api_bytesio_gib_s",
              "api_bytesio_register_gib_s", "api_file_mmap_gib_s", "api_file_mmap_register_gib_s",
              "api_bytesio_register_p1024_s10_gib_s"):
        assert hp[k] > 0, k
    assert set(hp["api_file_mmap_register_phases"]) == {"filebuffer_ms", "encode_ms", "close_ms"}
    assert hp["api_default"]["register_kinds"] == ["mmap", "bytesio", "bytes", "read"]
    # the registered rows really asked the library to register
    from heartbeat_amd import _native
    assert any(f & _native.HB_HOST_REGISTER for f, _ in fake.encodes)
    assert not fake.registered          # every caller registration was undone


def test_no_host_path_flag(fake, monkeypatch, capsys):
    d = _run_bench(monkeypatch, capsys, "--gib", "0.001", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
                   "--no-parity-sample", "--no-host-path", "--sustain-seconds", "0")
    assert "host_path" not in d and "sustained" not in d and "cpu_baseline" not in d


def test_prove_line(fake, monkeypatch, capsys):
    d = _run_bench(monkeypatch, capsys, "--config", "c5", "--gib", "0.002", "--steps", "2", "--warmup", "1",
                   "--cpu-seconds", "0.2")
    assert d["unit"] == "ms" and d["higher_is_better"] is False
    assert d["proof_equal_oracle"] is True
    assert d["cpu_baseline"]["proof_equal_gpu"] is True
    assert d["verify"]["verified"] is True


def test_two_rank_encode_line(tmp_path):
    """Two ranks (gloo, one process each) of the c4 plan through the stand-in
    library: every leg that runs at N > 1 -- shard plan, timed loop with
    barriers and max-over-ranks, sustained leg, per-rank parity sample summed
    over ranks -- and exactly one JSON line from rank 0."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TMPDIR=str(tmp_path))
        env.pop("HB_BENCH_SAME_DEVICE", None)
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "run_bench_fake.py"), "--gpus", "2", "--gib", "0.001",
             "--steps", "2", "--warmup", "1", "--sustain-seconds", "0.05", "--parity-blocks", "50"],
            env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["workload"].startswith("configs[3]")
    assert d["parity_sample"]["ok"] is True and d["sustained"]["steps"] >= 1
    assert "host_path" not in d and "cpu_baseline" not in d
