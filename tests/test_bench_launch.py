"""bench.py's launch plumbing on CPU (no HIP calls, --dry-run): `--gpus 2`
starts two ranks by itself (gloo control plane), rank 0 prints exactly one
JSON line with n_gpus = 2 and the max-over-ranks step time; the N = 1 path
prints one line with n_gpus = 1; c4 plans its 256 GiB share in resident
pieces."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(*args, extra_env=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HB_BENCH_SAME_DEVICE"):
        env.pop(k, None)
    env.update(extra_env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"] + list(args),
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_two_ranks_one_line():
    d = _run("--gpus", "2", "--steps", "3", "--warmup", "1")
    assert d["n_gpus"] == 2
    assert d["steps"] == 3
    # rank 1 sleeps 4 ms per step, rank 0 2 ms: the max over ranks is reported
    assert d["ms_per_step"] >= 3.5
    assert d["config"]["blocks_summed"] == d["config"]["blocks_total"]
    assert d["distinct_devices"] == 2 and "same_device_rehearsal" not in d


def test_same_device_rehearsal_is_marked():
    """Two ranks on one GPU (HB_BENCH_SAME_DEVICE) report n_gpus = 2 but
    distinct_devices = 1 and same_device_rehearsal: such a line can never
    pass for a 2-GPU measurement."""
    d = _run("--gpus", "2", "--steps", "1", extra_env={"HB_BENCH_SAME_DEVICE": "1"})
    assert d["n_gpus"] == 2 and d["distinct_devices"] == 1 and d["same_device_rehearsal"] is True


def test_single_rank():
    d = _run("--steps", "2")
    assert d["n_gpus"] == 1 and d["scaling"] == "weak" and d["distinct_devices"] == 1
    assert d["config"]["file_bytes"] == 64 << 30


def test_c4_strong_scaling_plan():
    d = _run("--gpus", "2", "--config", "c4", "--steps", "1")
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["file_bytes"] == 256 << 30
    d1 = _run("--config", "c4", "--steps", "1")
    assert d1["config"]["pieces_rank0"] == 2      # 256 GiB does not fit one GPU's HBM with its tags


def test_multi_gpu_default_is_configs3():
    """`bench.py --gpus N` with N > 1 and no --config measures configs[3] (one
    256 GiB file sharded over the N ranks, strong scaling), the N = 1 default
    stays configs[2] (the driver's 8-GPU run must measure the
    BASELINE config)."""
    d = _run("--gpus", "2", "--steps", "1")
    assert d["scaling"] == "strong" and d["config"]["file_bytes"] == 256 << 30
    assert d["config"]["workload"].startswith("configs[3]")
    assert d["config"]["blocks_summed"] == d["config"]["blocks_total"] == (256 << 30) // 512 + 1
    d1 = _run("--steps", "1")
    assert d1["config"]["workload"].startswith("configs[2]") and d1["scaling"] == "weak"
