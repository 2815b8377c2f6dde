#!/usr/bin/env python3
"""Swizzle encode benchmark (BASELINE.json metric: GiB/s of file bytes tagged,
Swizzle encode, device-resident, at 1/2/4/8 GPUs).

One step = one pass of the encode hot path (hb_encode: alpha PRF + Montgomery
conversion + prefix image + the encode kernels) over every block of this
rank's device-resident synthetic file.  Workloads (BASELINE.json configs):
  c3 (default): configs[2], 64 GiB random file, 256-bit prime, 16 sectors per
                block -- the largest single-GPU configuration; for N > 1 every
                rank encodes its own 64 GiB block-range shard of an N*64 GiB
                file (weak scaling, no collective: blocks are independent).
  c2:           configs[1], 1 GiB, 256-bit prime, 1 sector per block.
  c4:           configs[3], ONE 256 GiB file sharded over the N ranks (strong
                scaling, 256/N GiB per rank).  A rank whose share does not fit
                in HBM next to its tags (N = 1) holds it as consecutive
                resident pieces; only the encode calls are timed.
  c5:           configs[4], prove() on a 64 GiB device-resident file with a
                10,000-index challenge (ms per proof).

Launch: `python bench.py [--gpus N --steps K --warmup W]`.  With N > 1 and no
torch.distributed environment the script starts N ranks itself (one process
per GPU, LOCAL_RANK = GPU ordinal) before touching any GPU; under
`torch.distributed.run` it is one of the launched ranks.  Ranks share nothing
but a gloo barrier and the max-over-ranks time (no data-path collective; the
control plane does not need RCCL).

Besides the contract fields the JSON line carries
  roofline:     the encode kernels' algorithmic file bytes per launch / their
                mean duration (HIP events on the kernel stream) against the HBM
                read peak (vendor 8.0 TB/s; `peak_measured` = hb_stream_read on
                the same buffer), traffic from the committed rocprofv3 PMC pass
                when it matches this workload, and the LDS-lookup and VALU
                resources that actually bind;
  parity_sample: >= 10,000 random blocks plus the first and last 1,000 (the
                tail block included) of every rank's tags, after the timed
                region, against the CPU oracle;
  cpu_baseline: the repo's C oracle (OpenSSL AES-NI + BIGNUM, pthreads) on a
                bounded prefix of the same file, and the pure-Python PySwizzle
                restatement (oracle/pyswizzle_port.py) on 1 MiB and on a
                bounded prefix of 64 MiB, single core (rank 0, N = 1).
"""
import argparse
import ctypes
import hashlib
import json
import os
import platform
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)
GIB = 1 << 30
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E vendor peak (MI355X_MICROARCH.md)
LDS_LOOKUPS_PER_CLK_CU = 32.0  # one wave-wide ds_read_b32 per 2 clocks per CU
CLOCK_GHZ = 2.4
NUM_CUS = 256
MAX_RESIDENT_GIB = 160         # per-rank resident file bytes (HBM 288 GB minus tags / scratch)
METRIC = "GiB/s file bytes tagged (Swizzle encode, device-resident) at 1/2/4/8 GPUs"

CONFIGS = {
    "c3": dict(name="configs[2]: 64 GiB random file, Swizzle encode, 256-bit prime, "
                    "16 sectors/block, 1 MI355X (per rank for N>1: 64 GiB shard)",
               gib_per_rank=64, sectors=16, weak=True),
    "c2": dict(name="configs[1]: 1 GiB random file, Swizzle encode, 256-bit prime, "
                    "1 sector/block (per rank for N>1)",
               gib_per_rank=1, sectors=1, weak=True),
    "c5": dict(name="configs[4]: Swizzle prove() on a 64 GiB device-resident file, 10 000-index "
                    "challenge, 256-bit prime, 16 sectors/block, 1 MI355X",
               gib_per_rank=64, sectors=16, weak=True, prove_chunks=10000),
    "c4": dict(name="configs[3]: 256 GiB random file, Swizzle encode, 256-bit prime, "
                    "16 sectors/block, block ranges sharded over N GPUs (no collective)",
               gib_total=256, sectors=16, weak=False),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: c3 (configs[2]) at --gpus 1, c4 (configs[3], 256 GiB sharded) at --gpus N > 1")
    ap.add_argument("--gib", type=float, default=None, help="override file GiB per rank")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="oracle threads (default: this process's CPU share, $OMP_NUM_THREADS or affinity)")
    ap.add_argument("--py-seconds", type=float, default=15.0,
                    help="budget of the pure-Python PySwizzle row on the 64 MiB input")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity-sample", action="store_true")
    ap.add_argument("--parity-blocks", type=int, default=10000)
    ap.add_argument("--single-pass", action="store_true",
                    help="one-pass PRF engine instead of prefix-image first pass + retry pass")
    ap.add_argument("--prf", default="pyswizzle", choices=["pyswizzle", "cxx"],
                    help="pyswizzle: KeyedPRF, tags bit-exact vs PySwizzle (the headline); cxx: the "
                         "cxx Swizzle extension's PRF (cxx/prf.hxx, CFB-128), parity unpinned")
    ap.add_argument("--sustain-seconds", type=float, default=6.0,
                    help="after the timed region, keep encoding the same file for about this long and report "
                         "the sustained rate (steady-state clock and power; 0 = skip)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-memory path rows (4 GiB prefix, after the CPU rows; on by default "
                         "for the N = 1 configs[2] run)")
    ap.add_argument("--host-path", action="store_true",
                    help="time the host-memory path rows in any configuration")
    ap.add_argument("--no-prove", action="store_true",
                    help="skip the configs[4] prove row of the default N = 1 configs[2] run")
    ap.add_argument("--prove-proofs", type=int, default=200, help="timed proofs of that row")
    ap.add_argument("--no-wide", action="store_true",
                    help="skip the `wide` row (PySwizzle's default 1024-bit prime, S = 10, 8 GiB) of the default "
                         "N = 1 configs[2] run")
    ap.add_argument("--no-configs1", action="store_true",
                    help="skip the `configs1` row (configs[1]: 1 GiB, S = 1) of the default N = 1 configs[2] run")
    ap.add_argument("--dry-run", action="store_true",
                    help="exercise the launch / rank / timing / JSON plumbing without HIP calls (CPU tests)")
    args = ap.parse_args(argv)
    if args.config is None:
        # one GPU: configs[2], the largest single-GPU configuration (the BENCH
        # line and the N = 1 point of the scaling curve); several GPUs:
        # configs[3], the 256 GiB file sharded over them
        args.config = "c3" if args.gpus == 1 else "c4"
    return args


# ---------------------------------------------------------------- ranks
def spawn_ranks(args):
    """Start args.gpus ranks of this script (one process per GPU) and return
    the worst exit code.  Runs before anything touches a GPU."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(args.gpus),
                    "LOCAL_WORLD_SIZE": str(args.gpus), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    return rc


class Ranks(object):
    """This process's place in the job and the gloo control plane."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal of the N-rank path on a one-GPU box: every rank on device 0
        self.device = 0 if os.environ.get("HB_BENCH_SAME_DEVICE") else self.local
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def gather(self, obj):
        """obj of every rank, in rank order (gloo all_gather_object)."""
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def device_report(self, bus_id):
        """How many physically distinct GPUs the ranks ran on: an N-rank line
        from a one-GPU rehearsal (HB_BENCH_SAME_DEVICE) must not read as N
        GPUs."""
        ids = self.gather((self.device, bus_id))
        distinct = len({b if b is not None else "ordinal %d" % d for d, b in ids})
        rep = {"distinct_devices": distinct, "device_pci_bus_ids": [b for _, b in ids]}
        if os.environ.get("HB_BENCH_SAME_DEVICE"):
            rep["same_device_rehearsal"] = True
        return rep

    def reduce(self, x, op):
        """x (float) reduced over ranks with op in {"max", "min", "sum"}."""
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        o = {"max": self.dist.ReduceOp.MAX, "min": self.dist.ReduceOp.MIN,
             "sum": self.dist.ReduceOp.SUM}[op]
        self.dist.all_reduce(t, op=o)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


# ---------------------------------------------------------------- workload
def workload_name(args, cfg):
    """The BASELINE config's name, marked when --gib overrides its size (a
    rehearsal or a test, not that config's measurement)."""
    if args.gib is None:
        return cfg["name"]
    return "%s [--gib %g: %g GiB per rank instead]" % (cfg["name"], args.gib, args.gib)


def plan_for(args, cfg, world, rank):
    from heartbeat_amd.shard import shard_plan
    S = cfg["sectors"]
    C = 32 * S
    if args.gib is not None:
        file_len = int(args.gib * GIB) * world
    elif cfg["weak"]:
        file_len = cfg["gib_per_rank"] * GIB * world
    else:
        file_len = cfg["gib_total"] * GIB
    plan = shard_plan(file_len, C, rank, world)
    # resident pieces of this rank's share (whole blocks)
    max_piece = MAX_RESIDENT_GIB * GIB // C * C
    pieces = []
    off = 0
    while True:
        n = min(max_piece, plan["byte_len"] - off)
        pieces.append((off, n))
        off += n
        if off >= plan["byte_len"]:
            break
    return file_len, plan, pieces


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    R = Ranks()
    try:
        if args.dry_run:
            return dry_run(args, R)
        cfg = CONFIGS[args.config]
        if "prove_chunks" in cfg:
            return bench_prove(args, cfg, R)
        return bench_encode(args, cfg, R)
    finally:
        R.close()


def dry_run(args, R):
    """The launch / barrier / max-over-ranks / JSON path with a sleep for a step."""
    cfg = CONFIGS[args.config]
    file_len, plan, pieces = plan_for(args, cfg, R.world, R.rank)
    for _ in range(args.warmup):
        time.sleep(0.001)
    R.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.002 * (1 + R.rank))
    R.barrier()
    elapsed = R.reduce(time.perf_counter() - t0, "max")
    blocks = R.reduce(plan["nblocks"], "sum")
    rep = R.device_report(None)
    if R.rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": R.world,
                          **rep, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak" if cfg["weak"] else "strong", "dry_run": True,
                          "config": {"workload": workload_name(args, cfg), "file_bytes": file_len,
                                     "blocks_total": plan["total_blocks"], "blocks_summed": int(blocks),
                                     "pieces_rank0": len(pieces)}}), flush=True)


def bench_encode(args, cfg, R):
    from heartbeat_amd import _native
    L = _native.lib()
    ctx = _native.context(R.device)
    S = cfg["sectors"]
    p = P256
    pb = _native.be(p)
    # context setup outside the timed region, as a library handle would be:
    # load the 256-bit kernels' code object (hb_ctx_prepare), which the HIP
    # runtime otherwise loads inside the first encode
    t = time.perf_counter()
    if not args.dry_run:
        ctx.prepare(p.bit_length())
    prepare_ms = (time.perf_counter() - t) * 1e3
    w = 32
    C = 32 * S
    file_len, plan, pieces = plan_for(args, cfg, R.world, R.rank)
    b0 = plan["b0"]
    nblocks = plan["nblocks"]
    length = plan["byte_len"]
    fk = hashlib.sha256(b"hb-bench-f").digest()
    ak = hashlib.sha256(b"hb-bench-alpha").digest()
    seed = 0x5EED0000 + 3 + R.rank

    piece_bytes = max(n for _, n in pieces)
    dptr = ctypes.c_void_p()
    tptr = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, max(piece_bytes, 16), ctypes.byref(dptr)))
    ctx.check(L.hb_device_malloc(ctx.h, nblocks * w, ctypes.byref(tptr)))

    def fill(k):
        # resident piece k of this rank's share, its own seeded stream
        ctx.check(L.hb_fill_random(ctx.h, dptr, pieces[k][1], seed ^ (k << 24)))

    fill(0)
    tries = ctypes.c_uint64()
    cxx = args.prf == "cxx"
    flags = 3 | (_native.HB_ENCODE_SINGLE_PASS if args.single_pass else 0) | (_native.HB_PRF_CXX if cxx else 0)
    tries_total = [0]

    def encode_piece(k):
        off, n = pieces[k]
        pb0 = off // C                                   # first block of the piece in the rank
        last = k == len(pieces) - 1
        nb = (nblocks - pb0) if last else n // C
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, b0 + pb0, dptr, n, nb,
                              tptr.value + pb0 * w, flags, ctypes.byref(tries)))
        tries_total[0] += tries.value
        return ctx.last_kernel_ms()[0]

    def step():
        """Encode this rank's whole share; returns (wall s, kernel ms) of the
        encode calls only (piece refills, when there are several, excluded)."""
        wall, kms = 0.0, 0.0
        for k in range(len(pieces)):
            if len(pieces) > 1:
                fill(k)
            t = time.perf_counter()
            kms += encode_piece(k)
            wall += time.perf_counter() - t
        return wall, kms

    for _ in range(args.warmup):
        step()
    tries_total[0] = 0
    R.barrier()
    t0 = time.perf_counter()
    kms_list = []
    wall_sum = 0.0
    for _ in range(args.steps):
        wall, kms = step()
        wall_sum += wall
        kms_list.append(kms)
    R.barrier()
    elapsed = time.perf_counter() - t0
    if len(pieces) > 1:
        elapsed = wall_sum          # refills of the resident piece are not part of the encode
    elapsed = R.reduce(elapsed, "max")

    total_bytes = file_len * args.steps
    value = total_bytes / GIB / elapsed
    kernel_ms = sum(kms_list) / len(kms_list)
    achieved_gbs = length / (kernel_ms * 1e-3) / 1e9
    tries_step = tries_total[0] / args.steps
    tries_per_block = tries_step / nblocks
    if cxx:
        aes = tries_step * 2                       # CFB-128 over 32 bytes: 2 full AES per try
        lookups = aes * 16 * 14
    else:
        aes = tries_step * 32                      # nb = 32 byte-0 AES per try
        if not args.single_pass:
            # the first 4 of every block's first try come from the prefix image,
            # built once per step (2^24 + 2^16 + 2^8 byte-0 AES) per piece
            aes += len(pieces) * ((1 << 24) + (1 << 16) + (1 << 8)) - 4 * nblocks
        lookups = aes * (16 * 12 + 5)
        if not args.single_pass:
            # a first try's steps 4-7 skip the round-1 lookups of the register's
            # zero words (hb_lane.hpp, hb_aes_round1_z): 12 + 3 * 8 per block
            lookups -= 36 * nblocks
    lds_rate = lookups / (kernel_ms * 1e-3)
    lds_peak = NUM_CUS * CLOCK_GHZ * 1e9 * LDS_LOOKUPS_PER_CLK_CU

    traffic = None
    traffic_source = None
    pmc = None
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            rec = json.load(open(prof)).get(args.config + ("_cxx" if cxx else ""))
            if rec and rec.get("file_bytes") == length and len(pieces) == 1:
                traffic = rec["hbm_bytes_per_launch"]
                # not measured in this run: PMC counters cannot be read without
                # the profiler; the committed pass of the same workload is quoted
                traffic_source = ("profiles/pmc_traffic.json[%s]: rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE pass "
                                  "of this workload (%s), committed; not measured in this run" % (
                                      args.config + ("_cxx" if cxx else ""), rec.get("source_pmc", "?")))
                pmc = {k: rec[k] for k in ("lds_busy", "held_clock_ghz", "valu_wave_instr_per_cu_clk", "source_pmc")
                       if k in rec} or None
        except (ValueError, KeyError):
            traffic = None

    # measured streaming-read peak on the same buffer (outside the timed region)
    peak_measured = None
    ms = ctypes.c_double()
    nread = piece_bytes // 16 * 16
    if nread:
        for _ in range(2):          # the second pass is the measurement
            ctx.check(L.hb_stream_read(ctx.h, dptr, nread, ctypes.byref(ms)))
        peak_measured = round(nread / (ms.value * 1e-3) / 1e9, 1)

    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": R.world,
        **R.device_report(_native.pci_bus_id(R.device)),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak" if cfg["weak"] else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (SplitMix64 random file bytes, seeded keys)",
        "config": {
            "workload": workload_name(args, cfg),
            "file_bytes": file_len,
            "file_bytes_per_rank": length,
            "resident_pieces_per_rank": len(pieces),
            "blocks_total": plan["total_blocks"],
            "sectors": S,
            "prime_bits": 256,
            "prime": hex(p),
            "expected_tries_per_prf": round(2.0 ** 256 / p, 4),
            "prf": "cxx Swizzle prf (cxx/prf.hxx:125-176, CFB-128 over SHA256(LE32 i)); parity unpinned"
                   if cxx else "PySwizzle KeyedPRF (util.py:83-96, CFB-8 over SHA256(str(i))); bit-exact",
            "parallelism": "dp%d block-range shards, no collective (gloo barrier + max time only)" % R.world,
        },
        "roofline": {
            # the roofline the line is priced against (HBM bytes; the encode has
            # no MFMA-bound phase); what actually binds it is `binding`
            "bound": "hbm",
            "binding": "lds" if not cxx else "valu",
            "binding_note": ("the encode is NOT HBM-bound: it is bound by LDS T-table lookups at the clock the "
                             "socket power limit leaves (binding_resource, DESIGN.md 5.1); frac is the fraction "
                             "of the HBM roofline it reaches") if not cxx else
                            "cxx prf: per-block SHA-256 and the VALU MAC (DESIGN.md 5.2)",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "peak_measured": peak_measured,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "frac_of_measured": round(achieved_gbs / peak_measured, 4) if peak_measured else None,
            "traffic": traffic,
            "traffic_source": traffic_source,
            "kernel": "hb_cxx_encode_kernel" if cxx else "hb_encode_kernel" if args.single_pass else
                      "hb_prefix_kernel + hb_encode_first_kernel + hb_encode_retry_kernel",
            "kernel_ms": round(kernel_ms, 3),
            "algorithmic_bytes_per_launch": length,
            "binding_resource": {
                "resource": "LDS ds_read_b32 T-table lookups at the power-limited held clock (DESIGN.md 5.1)",
                "achieved_per_s": lds_rate,
                "peak_per_s": lds_peak,
                "frac": round(lds_rate / lds_peak, 4),
                "frac_at_held_clock": round(lds_rate / (lds_peak / CLOCK_GHZ * pmc["held_clock_ghz"]), 4)
                if pmc and pmc.get("held_clock_ghz") else None,
                "pmc": pmc,
            },
        },
        "context_prepare_ms": round(prepare_ms, 2),   # hb_ctx_prepare, before the timed region
        "build": _native.build_info(),   # provenance of libhbswizzle.so (hb_build_id, checked against the tree)
        "prf_tries_per_block": round(tries_per_block, 4),
        "aes_per_block": round(aes / nblocks, 3),
    }

    if args.sustain_seconds > 0 and len(pieces) == 1:
        line["sustained"] = sustained(args, R, step, elapsed / args.steps, file_len)
    # configs[4] on this very file (64 GiB, S = 16, 256-bit prime, its tags
    # just computed): the prove row of the same run, before the host-path rows
    # reuse the device buffer
    if R.rank == 0 and R.world == 1 and args.config == "c3" and not cxx and not args.no_prove and len(pieces) == 1:
        t = time.perf_counter()
        line["prove"] = prove_row(ctx, L, dptr, tptr, length, nblocks, S, p, C, w, args, fk, ak,
                                  proofs=args.prove_proofs)
        line["prove"]["seconds_spent"] = round(time.perf_counter() - t, 1)
    # the host-memory rows come right after the device-resident ones: after
    # the CPU rows (16 threads streaming 64 GiB through host buffers) the same
    # rows measured 21-25 instead of 31-38 GiB/s for a real file
    # (profiles/r05/f: bench_c3 vs bench_c3_nocpu), a state of the process's
    # host memory, not of the encode
    want_host = args.host_path or (R.world == 1 and args.config == "c3" and not cxx and not args.single_pass)
    if R.rank == 0 and want_host and not args.no_host_path:
        t = time.perf_counter()
        line["host_path"] = host_path(ctx, L, dptr, pieces[0][1], S, pb, fk, ak, C)
        line["host_path"]["seconds_spent"] = round(time.perf_counter() - t, 1)
    # the other encode shapes, on prefixes of this very file with tags of
    # their own: PySwizzle's default prime size (1024-bit, S = 10) and
    # configs[1] (1 GiB, S = 1); rows beside the headline, never `value`.
    # After the host-memory rows: their parity samples copy ~2 GiB of tags to
    # host memory, and the API rows measured 23-36 instead of 30-48 GiB/s
    # behind them (profiles/r06/h)
    if R.rank == 0 and R.world == 1 and args.config == "c3" and not cxx and len(pieces) == 1:
        aes_rate_c3 = aes / (kernel_ms * 1e-3)
        line["aes_g_per_s"] = round(aes_rate_c3 / 1e9, 2)
        if not args.no_wide:
            t = time.perf_counter()
            line["wide"] = extra_encode_row(ctx, L, dptr, min(8 * GIB, length), 1024, 10, fk, ak, args,
                                            steps=5, warmup=2, aes_rate_ref=aes_rate_c3, with_prove=not args.no_prove)
            line["wide"]["seconds_spent"] = round(time.perf_counter() - t, 1)
        if not args.no_configs1:
            t = time.perf_counter()
            line["configs1"] = extra_encode_row(ctx, L, dptr, min(1 * GIB, length), 256, 1, fk, ak, args,
                                                steps=20, warmup=3, aes_rate_ref=aes_rate_c3)
            line["configs1"]["seconds_spent"] = round(time.perf_counter() - t, 1)
    if not args.no_parity_sample:
        ok, n = parity_sample(ctx, L, dptr, tptr, pieces, plan, S, p, fk, ak, C, w, args, cxx, fill)
        n_all = int(R.reduce(n, "sum"))
        ok_all = R.reduce(1.0 if ok else 0.0, "min") == 1.0
        line["parity_sample"] = {"n": n_all, "ok": ok_all,
                                 "what": ">= %d random blocks + first/last 1,000 per rank (tail included) "
                                         "vs oracle/swizzle_oracle.c" % args.parity_blocks}
    if R.rank == 0 and R.world == 1 and not args.no_cpu_baseline:
        if len(pieces) > 1:
            fill(0)
        line["cpu_baseline"] = cpu_baseline(ctx, L, dptr, tptr, pieces[0][1], S, p, fk, ak, C,
                                            args.cpu_seconds, args.cpu_threads, args.py_seconds, cxx)

    if R.rank == 0:
        print(json.dumps(line), flush=True)
    ctx.check(L.hb_device_free(ctx.h, dptr))
    ctx.check(L.hb_device_free(ctx.h, tptr))


def seeded_prime(bits):
    """The benchmark prime of a size: P256 for 256 bits (E[tries] 1.17), else
    the first probable prime of a seeded stream (scripts/encode_rate.py's)."""
    if bits == 256:
        return P256
    import importlib
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(5000 + bits)
    while True:
        x = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(x):
            return x


def extra_encode_row(ctx, L, dptr, length, bits, S, fk, ak, args, steps, warmup, aes_rate_ref, with_prove=False):
    """A device-resident encode of another shape on the first `length` bytes
    of the bench file, tags in a buffer of their own, after the timed region:
    GiB/s over `steps` timed calls, the kernel phases (hb_last_kernel_phases),
    PRF tries and AES per block, the AES rate against the headline kernel's
    (`aes_rate_ref`), the HBM-roofline fraction of the file bytes, and a
    parity sample (first / last 1,000 blocks + --parity-blocks random ones vs
    the oracle).  Never `value`."""
    from heartbeat_amd import _native
    p = seeded_prime(bits)
    pb = _native.be(p)
    w = _native.width_of(p)
    ss = p.bit_length() // 8
    C = ss * S
    nblocks = length // C + 1
    nb_prf = (p.bit_length() + 7) // 8       # keystream bytes (AES) per PRF try
    tptr = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, nblocks * w, ctypes.byref(tptr)))
    tries = ctypes.c_uint64()
    ctx.prepare(p.bit_length())
    try:
        def one():
            ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, len(fk), 0, dptr, length, nblocks, tptr, 3,
                                  ctypes.byref(tries)))
            return ctx.last_kernel_ms()[0], ctx.last_kernel_phases(), tries.value

        for _ in range(warmup):
            one()
        t0 = time.perf_counter()
        runs = [one() for _ in range(steps)]
        el = time.perf_counter() - t0
        kms = sum(r[0] for r in runs) / steps
        ph = [round(sum(r[1][k] for r in runs) / steps, 4) for k in range(len(runs[0][1]))]
        tr = sum(r[2] for r in runs) / steps
        # the first 4 keystream bytes of every first try come from the prefix
        # image, built once per call (2^24 + 2^16 + 2^8 byte-0 AES)
        two_pass = len(ph) == 4
        aes_prf = tr * nb_prf - (4 * nblocks if two_pass else 0)
        aes_all = aes_prf + ((1 << 24) + (1 << 16) + (1 << 8) if two_pass else 0)
        row = {"workload": "%d-bit seeded prime, %d sector%s/block (%d-byte sectors), %.3g GiB device-resident "
                           "prefix of the bench file" % (bits, S, "s" if S > 1 else "", ss, length / GIB),
               "prime": hex(p), "expected_tries_per_prf": round((1 << p.bit_length()) / p, 4),
               "file_bytes": length, "blocks": nblocks,
               "value": round(length * steps / GIB / el, 3), "unit": "GiB/s",
               "ms_per_step": round(el / steps * 1e3, 3), "steps": steps, "warmup": warmup,
               "kernel_ms": round(kms, 3),
               "kernel_gib_s": round(length / GIB / (kms * 1e-3), 3),
               "roofline": {"bound": "hbm", "achieved": round(length / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(length / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
               "prf_tries_per_block": round(tr / nblocks, 4),
               "aes_per_block": round(aes_all / nblocks, 3),
               "aes_g_per_s": round(aes_all / (kms * 1e-3) / 1e9, 2),
               "aes_rate_vs_headline_kernel": round(aes_all / (kms * 1e-3) / aes_rate_ref, 4),
               "note": "after the timed region; never `value`"}
        if two_pass:
            row["phases_ms"] = {"setup (prefix image, MAC tables)": ph[0], "first_pass": ph[1], "retry_pass": ph[2],
                                "wide_mac (hb_wmac_kernel)": ph[3]}
            row["prf_pass_aes_g_per_s"] = round(aes_prf / ((ph[1] + ph[2]) * 1e-3) / 1e9, 2)
        if not args.no_parity_sample:
            row["parity_sample"] = row_parity(ctx, L, dptr, tptr, length, nblocks, S, p, fk, ak, C, w,
                                              args.parity_blocks)
        if with_prove:
            row["prove"] = extra_prove(ctx, L, dptr, tptr, length, nblocks, S, p, C, w, fk, ak,
                                       check=not args.no_parity_sample)
    finally:
        ctx.check(L.hb_device_free(ctx.h, tptr))
    return row


def extra_prove(ctx, L, dptr, tptr, length, nblocks, S, p, C, w, fk, ak, proofs=50, chunks=10000, check=True):
    """PySwizzle.prove (PySwizzle.py:333-370) of a 10,000-index challenge
    (v_max = p) over an extra row's device-resident file and tags, and its
    verify (PySwizzle.py:372-395, hb_verify_rhs), timed back to back; the
    proof checked against oracle/swizzle_oracle.c on the challenged blocks
    and tags copied back."""
    from heartbeat_amd import _native
    pb = _native.be(p)
    ck = hashlib.sha256(b"hb-bench-challenge-wide").digest()
    mu = ctypes.create_string_buffer(w * S)
    sg = ctypes.create_string_buffer(w)

    def one():
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, ck, len(ck), chunks, pb, len(pb), tptr, nblocks, dptr, length,
                             3, mu, sg))

    for _ in range(10):
        one()
    t = time.perf_counter()
    for _ in range(proofs):
        one()
    row = {"challenge": "%d indices, v_max = p" % chunks,
           "ms_per_proof": round((time.perf_counter() - t) / proofs * 1e3, 4), "proofs": proofs,
           "launches_per_proof": ctx.last_kernel_ms()[1]}
    row["verify"] = verify_timing(ctx, L, pb, S, fk, ak, nblocks, ck, chunks, mu, sg, proofs)
    if check:
        import numpy as np
        from oracle import oracle as O
        idx = sorted({O.prf_eval(ck, nblocks, i) for i in range(chunks)})
        host = np.zeros(length, dtype=np.uint8)          # untouched pages stay unallocated
        tags = np.zeros(nblocks * w, dtype=np.uint8)
        for ix in idx:
            a = ix * C
            if a < length:
                ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data + a, dptr.value + a, min(C, length - a), 2))
            ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data + ix * w, tptr.value + ix * w, w, 2))
        ref_mu = ctypes.create_string_buffer(w * S)
        ref_sg = ctypes.create_string_buffer(w)
        rc = O.lib().hbo_prove(pb, len(pb), S, ck, len(ck), chunks, pb, len(pb), nblocks,
                               ctypes.cast(tags.ctypes.data, ctypes.c_char_p), w, host.ctypes.data, length,
                               ref_mu, ref_sg)
        if rc:
            raise RuntimeError("oracle prove error %d" % rc)
        row["proof_equal_oracle"] = ref_mu.raw == mu.raw and ref_sg.raw == sg.raw
    return row


def row_parity(ctx, L, dptr, tptr, length, nblocks, S, p, fk, ak, C, w, nrand):
    """First / last 1,000 blocks (the short tail block included) and `nrand`
    random ones of a one-piece encode vs the oracle."""
    import numpy as np
    from oracle import oracle as O
    rng = random.Random(0xC0FFEE + C)
    picks = set(range(min(1000, nblocks))) | set(range(max(0, nblocks - 1000), nblocks))
    while len(picks) < min(nblocks, nrand + 2000):
        picks.add(rng.randrange(nblocks))
    picks = sorted(picks)
    tags = np.empty(nblocks * w, dtype=np.uint8)
    ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data, tptr.value, nblocks * w, 2))
    ok, i = True, 0
    while i < len(picks):
        j = i
        while j + 1 < len(picks) and picks[j + 1] == picks[j] + 1:
            j += 1
        r0, r1 = picks[i], picks[j] + 1
        lo, hi = r0 * C, min(r1 * C, length)
        data = np.empty(max(hi - lo, 0), dtype=np.uint8)
        if hi > lo:
            ctx.check(L.hb_memcpy(ctx.h, data.ctypes.data, dptr.value + lo, hi - lo, 2))
        want = O.encode(p, S, fk, ak, data, block_base=r0, nblocks=r1 - r0, nthreads=4)
        ok = ok and tags[r0 * w:r1 * w].tobytes() == b"".join(t.to_bytes(w, "big") for t in want)
        i = j + 1
    return {"n": len(picks), "ok": ok, "what": "first/last 1,000 + %d random blocks vs oracle/swizzle_oracle.c" % nrand}


def sustained(args, R, step, sec_per_step, file_len):
    """After the timed region: the same encode step repeated for about
    --sustain-seconds (the same step count on every rank), timed like the
    headline (barriers, max over ranks).  A steady-state check -- held clock,
    socket power at its cap -- of the short timed region, and several seconds
    of GPU activity for an outside utilisation sampler.  Never `value`."""
    steps = max(1, int(round(args.sustain_seconds / max(sec_per_step, 1e-6))))
    R.barrier()
    t0 = time.perf_counter()
    kms = 0.0
    for _ in range(steps):
        kms += step()[1]
    R.barrier()
    el = R.reduce(time.perf_counter() - t0, "max")
    return {"steps": steps, "seconds": round(el, 3), "value": round(file_len * steps / GIB / el, 3),
            "unit": "GiB/s", "ms_per_step": round(el / steps * 1e3, 3), "kernel_ms": round(kms / steps, 3),
            "note": "the timed step repeated after the timed region; not `value`"}


def parity_sample(ctx, L, dptr, tptr, pieces, plan, S, p, fk, ak, C, w, args, cxx, fill):
    """After the timed region: this rank's first and last 1,000 blocks (the
    last rank's include the PRF-only tail block) and >= parity_blocks random
    blocks, GPU tags vs the oracle.  Returns (all equal, blocks checked)."""
    import numpy as np
    from oracle import oracle as O
    nblocks = plan["nblocks"]
    rng = random.Random(0x5A11 + plan["b0"])
    picks = set(range(min(1000, nblocks))) | set(range(max(0, nblocks - 1000), nblocks))
    while len(picks) < min(nblocks, args.parity_blocks + 2000):
        picks.add(rng.randrange(nblocks))
    picks = sorted(picks)
    tags = np.empty(nblocks * w, dtype=np.uint8)
    ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data, tptr.value, nblocks * w, 2))
    enc = O.cxx_encode if cxx else O.encode
    ok = True
    k = 0
    # walk the pieces (refill when there are several: the buffer holds the last one)
    for pi, (off, n) in enumerate(pieces):
        if len(pieces) > 1:
            fill(pi)
        pb0, pb1 = off // C, (nblocks if pi == len(pieces) - 1 else (off + n) // C)
        sel = [b for b in picks if pb0 <= b < pb1]
        # contiguous runs: one copy and one oracle call each
        i = 0
        while i < len(sel):
            j = i
            while j + 1 < len(sel) and sel[j + 1] == sel[j] + 1:
                j += 1
            r0, r1 = sel[i], sel[j] + 1
            lo = (r0 - pb0) * C
            hi = min((r1 - pb0) * C, n)
            data = np.empty(max(hi - lo, 0), dtype=np.uint8)
            if hi > lo:
                ctx.check(L.hb_memcpy(ctx.h, data.ctypes.data, dptr.value + lo, hi - lo, 2))
            want = enc(p, S, fk, ak, data, block_base=plan["b0"] + r0, nblocks=r1 - r0, nthreads=4)
            got = tags[r0 * w:r1 * w].tobytes()
            ok = ok and got == b"".join(t.to_bytes(w, "big") for t in want)
            k += r1 - r0
            i = j + 1
    return ok, k


def host_cpu_info():
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                info["lscpu_model"] = ln.split(":", 1)[1].strip()
    except Exception:
        info["lscpu_model"] = platform.processor() or None
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    return info


def cpu_baseline(ctx, L, dptr, tptr, length, S, p, fk, ak, C, seconds, threads, py_seconds, cxx=False):
    """CPU rows on this process's CPU share, on prefixes of the SAME synthetic
    file (copied from the device in 256 MiB pieces):
      * headline ("cxx Swizzle" counterpart): the native
        multi-threaded encoder baseline/hb_cpu_swizzle.cpp (AES-NI CFB-8,
        SHA-NI, 64-bit-limb Montgomery MAC, std::thread) until `seconds` of
        work; its tags are compared with the GPU's for the same blocks;
      * the test oracle (OpenSSL EVP + BIGNUM per sector) for a third of that;
      * the single-core pure-Python PySwizzle restatement on 1 MiB and a
        bounded prefix of a 64 MiB input.
    The cxx-PRF mode has no native row (the oracle is its headline)."""
    import io
    import numpy as np
    from oracle import oracle as O
    info = host_cpu_info()
    if threads is None:
        # the GPU box gives each GPU a 16-core share and exports it as
        # OMP_NUM_THREADS; nproc there counts the whole machine
        threads = int(os.environ.get("OMP_NUM_THREADS") or info.get("affinity") or os.cpu_count() or 1)
    threads = max(1, threads)
    piece = (256 << 20) // C * C
    host = np.empty(piece, dtype=np.uint8)
    out = np.empty((piece // C) * 32, dtype=np.uint8)
    gpu = np.empty((piece // C) * 32, dtype=np.uint8)

    def timed(encode, budget):
        done = busy = 0.0
        off = 0
        same = True
        while busy < budget and off < length:
            n = min(piece, length - off)
            ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value + off, n, 2))
            nb = n // C
            t = time.perf_counter()
            encode(off // C, n, nb)
            busy += time.perf_counter() - t
            ctx.check(L.hb_memcpy(ctx.h, gpu.ctypes.data, tptr.value + (off // C) * 32, nb * 32, 2))
            same = same and bool(np.array_equal(out[:nb * 32], gpu[:nb * 32]))
            done += n
            off += n
        return done, busy, same

    def oracle_encode(b0, n, nb):
        rc = O.encode_raw(p, S, fk, ak, host.ctypes.data, n, b0, nb, out.ctypes.data, threads, cxx)
        if rc:
            raise RuntimeError("oracle error %d" % rc)

    oracle_budget = seconds if cxx else max(2.0, seconds / 3)
    done, busy, same = timed(oracle_encode, oracle_budget)
    oracle_row = {"value": round(done / GIB / busy, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
                  "sample": "%d MiB prefix of the same synthetic file (%d blocks), oracle/swizzle_oracle.c "
                            "(%s), %d pthreads, %.1f s" % (
                                done // (1 << 20), done // C,
                                "cxx prf: OpenSSL AES-NI CFB-128 + BIGNUM" if cxx else
                                "OpenSSL AES-NI CFB8 + BIGNUM", threads, busy),
                  "tags_equal_gpu": same}
    if cxx:
        return dict(oracle_row, host=info)
    from baseline import cpu as NC
    aesni = bool(NC.lib().hbcpu_aesni())

    def native_encode(b0, n, nb):
        NC.encode_raw(p, S, fk, ak, host.ctypes.data, n, b0, nb, out.ctypes.data, threads)

    native_encode(0, min(piece, length), min(piece, length) // C)      # warm-up (page faults, threads)
    done, busy, same = timed(native_encode, seconds)
    rate = done / GIB / busy
    res = {"value": round(rate, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
           "name": "cxx Swizzle counterpart: native C++ encoder (BASELINE.md 3)",
           "cores_available": info.get("affinity") or info.get("nproc"),
           "per_core_gib_s": round(rate / threads, 4),
           "cores_note": ("%d threads = this process's CPU share ($OMP_NUM_THREADS / affinity; a GPU box leases "
                          "16 host cores per GPU and exports OMP_NUM_THREADS=16), not the whole host's %s "
                          "CPUs; per_core_gib_s = value / cores" % (threads, info.get("affinity") or info.get("nproc"))),
           "sample": "%d MiB prefix of the same synthetic file (%d blocks), baseline/hb_cpu_swizzle.cpp "
                     "(%s, SHA-NI SHA256_Transform, 64-bit-limb Montgomery MAC), %d std::threads, %.1f s" % (
                         done // (1 << 20), done // C,
                         "AES-NI, 8 evaluations interleaved per thread" if aesni else "portable byte AES",
                         threads, busy),
           "tags_equal_gpu": same,
           "oracle_row": oracle_row,
           "host": info}
    # BASELINE.md 3 asks for all host cores; the lease gives this process a
    # share of them, so the whole-host figure is an extrapolation, labelled
    ncpu = info.get("affinity") or info.get("nproc") or threads
    if ncpu > threads:
        res["full_node_extrapolated"] = {
            "value": round(rate / threads * ncpu, 3), "unit": "GiB/s", "cores": ncpu, "kind": "extrapolated",
            "note": "per_core_gib_s x all %d logical CPUs of the host: linear in threads from the measured "
                    "%d-thread share, an upper bound (SMT sharing and host memory bandwidth not modelled); "
                    "not measured" % (ncpu, threads)}
    # the "PySwizzle" row: pure Python, one core, the reference's algorithmic cost
    from oracle import pyswizzle_port as PP
    rows = []
    ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value, min(64 << 20, length, piece), 2))
    for label, size, budget in (("1 MiB input", 1 << 20, None), ("64 MiB input", 64 << 20, py_seconds)):
        size = min(size, length, piece)
        src = io.BytesIO(host[:size].tobytes())
        t = time.perf_counter()
        if budget is None:
            PP.encode(p, S, fk, ak, src)
            nbytes = size
        else:
            # whole blocks until the budget is spent (rate over the processed prefix)
            f = PP.KeyedPRF(fk, p)
            a = PP.KeyedPRF(ak, p)
            nbytes = 0
            blk = 0
            while nbytes + C <= size and time.perf_counter() - t < budget:
                sigma = f.eval(blk)
                for j in range(S):
                    buf = src.read(32)
                    sigma += a.eval(j) * int.from_bytes(buf, "big")
                sigma %= p
                nbytes += C
                blk += 1
        dt = time.perf_counter() - t
        rows.append({"value": round(nbytes / (1 << 20) / dt, 3), "unit": "MiB/s", "cores": 1,
                     "kind": "port", "sample": "%s: %.2f MiB encoded in %.1f s" % (label, nbytes / (1 << 20), dt)})
    rows.append(pyswizzle_test6_row())
    res["pyswizzle_rows"] = rows
    return res


def pyswizzle_test6_row():
    """The "PySwizzle" row on BASELINE.md 3's config 1: the reference's
    tests/files/test6.txt (999,999 B, regenerated) at the PySwizzle defaults
    (10 sectors, 1024-bit prime, PySwizzle.py:233), encode + prove + verify by
    the single-core pure-Python restatement, with the keys, tags and proof of
    the reference-generated golden case (tests/golden/file_cases.json)."""
    import io
    from oracle import pyswizzle_port as PP
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "file_cases.json")))
    c = next(c for c in g["cases"] if c["name"] == "test6.txt/p1024/S10")
    p = int(c["prime"], 16)
    S = int(c["sectors"])
    fk, ak = bytes.fromhex(c["f_key"]), bytes.fromhex(c["alpha_key"])
    line = b"abcdefghijklmnopqrstuvwxyz1234567890\n"
    data = (line * (999999 // len(line) + 1))[:999999]
    w = (p.bit_length() + 7) // 8
    t = time.perf_counter()
    tags = PP.encode(p, S, fk, ak, io.BytesIO(data))
    enc_s = time.perf_counter() - t
    tags_ok = hashlib.sha256(b"".join(x.to_bytes(w, "big") for x in tags)).hexdigest() == c["tags_sha256"]
    f = io.BytesIO(data)
    ch = c["chal"]
    ck, vmax = bytes.fromhex(ch["key"]), int(ch["v_max"], 16)
    t = time.perf_counter()
    mu, sg = PP.prove(p, S, f, ck, ch["chunks"], vmax, tags)
    prove_s = time.perf_counter() - t
    proof_ok = mu == [int(m, 16) for m in c["proof"]["mu"]] and sg == int(c["proof"]["sigma"], 16)
    # the default challenge of gen_challenge: chunks = #tags (PySwizzle.py:329)
    t = time.perf_counter()
    mu2, sg2 = PP.prove(p, S, f, ck, len(tags), vmax, tags)
    prove_all_s = time.perf_counter() - t
    t = time.perf_counter()
    ok = PP.verify(p, S, fk, ak, len(tags), ck, len(tags), vmax, mu2, sg2)
    verify_s = time.perf_counter() - t
    return {"value": round(len(data) / (1 << 20) / enc_s, 3), "unit": "MiB/s", "cores": 1, "kind": "port",
            "sample": "test6.txt (999,999 B), 10 sectors, 1024-bit prime (PySwizzle defaults), golden keys",
            "encode_s": round(enc_s, 3), "tags_equal_golden": tags_ok,
            "prove_s_300_idx": round(prove_s, 3), "proof_equal_golden": proof_ok,
            "prove_s_all_%d_idx" % len(tags): round(prove_all_s, 3),
            "verify_s_all_idx": round(verify_s, 3), "verified": ok}


def host_file_prove(ctx, L, dptr, pys, p, S, path, n, tag):
    """PySwizzle.prove through the drop-in API on a real file with the default
    challenge (gen_challenge: chunks = #tags, PySwizzle.py:316-331): every
    challenged block gathered from the (page-cache warm) mmap by host threads
    into pinned double buffers, summed on the GPU.  Checked against the same
    proof with the file device-resident."""
    import ctypes as ct
    ntags = len(tag)
    key = hashlib.sha256(b"hb-bench-chal").digest()
    chal = pys.Challenge(ntags, p, key)
    beat = pys.PySwizzle(S, b"k" * 32, p)
    with open(path, "rb") as f:
        beat.prove(f, pys.Challenge(1000, p, key), tag)          # warm-up
        t = time.perf_counter()
        proof = beat.prove(f, chal, tag)
        dt = time.perf_counter() - t
    # the same challenge with the file on the device (tags uploaded)
    w = 32
    pb = p.to_bytes(w, "big")
    mu = ct.create_string_buffer(w * S)
    sg = ct.create_string_buffer(w)
    import numpy as np
    traw = np.frombuffer(tag.raw(p), dtype=np.uint8)
    ctx.check(L.hb_prove(ctx.h, pb, w, S, key, 32, ntags, pb, w, traw.ctypes.data, ntags, dptr, n, 1, mu, sg))
    same = [int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(S)] == proof.mu and \
        int.from_bytes(sg.raw, "big") == proof.sigma
    return {"chunks": ntags, "file_bytes": n, "seconds": round(dt, 3),
            "challenged_gib_s": round(ntags * S * 32 / GIB / dt, 3),
            "blocks_per_s": round(ntags / dt, 1),
            "gather_threads": int(os.environ.get("HB_GATHER_THREADS") or os.environ.get("OMP_NUM_THREADS") or
                                  os.cpu_count() or 1),
            "equal_device_resident_proof": same}


def host_path(ctx, L, dptr, length, S, pb, fk, ak, C):
    """Rate with the file and the tags in host memory (the boundary of a
    file-like object in, tag bytes out; north_star: "the rate including pinned
    hipMemcpyAsync of sectors in and tags out"): chunked H2D of sectors +
    encode + D2H of tags, all inside the timed region, on a 4 GiB prefix of
    the same synthetic file.  Never `value`.  Rows:
      raw_*: hb_encode on a host buffer -- pageable (the runtime's staging),
        page-locked read-only in 256 MiB windows by the library itself
        (HB_HOST_REGISTER, registration inside the timed call), and pinned
        beforehand by the caller (hb_host_register, registration not timed);
      api_*: the drop-in API (PySwizzle.py:279-314 -> encode_file) on a BytesIO
        (its buffer, zero copy) and on a real file (read-only mmap, page cache
        warm), each with and without the windowed registration; `api_default`
        names what encode_file does by itself (REGISTER_KINDS);
      api_prove_file: PySwizzle.prove on the real file, default challenge.
    Every run's tags are compared with the first one's."""
    import importlib
    import io
    import tempfile
    import numpy as np
    n = min(length, 4 * GIB) // C * C
    host = np.empty(n, dtype=np.uint8)
    ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value, n, 2))
    nb = n // C
    tags = np.empty(nb * 32, dtype=np.uint8)
    ref = np.empty(nb * 32, dtype=np.uint8)
    out = {"bytes": n, "chunk": "256 MiB of whole blocks, double-buffered, H2D / D2H on a copy stream",
           "note": "PCIe-inclusive rates of the host-memory boundary; never `value` (DESIGN.md 6)"}

    def run(dst, flags=0):
        t = time.perf_counter()
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, host.ctypes.data, n, nb,
                              dst.ctypes.data, flags, None))
        return time.perf_counter() - t

    run(ref)   # warm-up (staging buffers, prefix image allocation)
    out["raw_pageable_gib_s"] = round(n / GIB / run(tags), 3)
    ok = bool(np.array_equal(tags, ref))
    run(tags, _native_flag("HB_HOST_REGISTER"))
    out["raw_register_windows_gib_s"] = round(n / GIB / run(tags, _native_flag("HB_HOST_REGISTER")), 3)
    ok = ok and bool(np.array_equal(tags, ref))
    ctx.check(L.hb_host_register(ctx.h, host.ctypes.data, n))
    ctx.check(L.hb_host_register(ctx.h, tags.ctypes.data, tags.nbytes))
    try:
        run(tags)
        out["raw_pinned_gib_s"] = round(n / GIB / run(tags), 3)
        ok = ok and bool(np.array_equal(tags, ref))
    finally:
        ctx.check(L.hb_host_unregister(ctx.h, tags.ctypes.data))
        ctx.check(L.hb_host_unregister(ctx.h, host.ctypes.data))
    out["raw_tags_equal"] = ok
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    p = int.from_bytes(pb, "big")
    out["api_default"] = {"register_kinds": list(pys.REGISTER_KINDS)}

    def api(src, register, reps=3):
        """Best of `reps` encode_file calls, with the phases of the best one:
        the FileBuffer (mmap), the encode (hb_encode via encode_shards), and
        consume + close (munmap)."""
        from heartbeat_amd import multi
        from heartbeat_amd._filebuf import FileBuffer
        best, same = None, True
        for _ in range(reps):
            src.seek(0)
            t0 = time.perf_counter()
            tag, _ = pys.encode_file(p, S, fk, ak, src, register=register)
            dt = time.perf_counter() - t0
            same = same and tag._raw[:nb * 32] == ref.tobytes()
            del tag
            if best is None or dt < best:
                best = dt
        # the phases of one more call, spelled out as encode_file does them
        src.seek(0)
        t0 = time.perf_counter()
        fb = FileBuffer(src, populate=not register)
        t1 = time.perf_counter()
        tags_out = np.empty((fb.len // C + 1) * 32, dtype=np.uint8)
        multi.encode_shards(p, S, fk, ak, fb.addr, fb.len, fb.len // C + 1, tags_out.ctypes.data,
                            _native_flag("HB_HOST_REGISTER") if register else 0, multi.devices())
        t2 = time.perf_counter()
        fb.consume()
        fb.close()
        t3 = time.perf_counter()
        phases = {"filebuffer_ms": round((t1 - t0) * 1e3, 2), "encode_ms": round((t2 - t1) * 1e3, 2),
                  "close_ms": round((t3 - t2) * 1e3, 2)}
        return n / GIB / best, same, phases

    api_ok = True
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp")) as fh:
        host.tofile(fh.name)
        # a file at rest (written back, page cache warm), not one still being
        # flushed while it is encoded
        with open(fh.name, "rb") as f:
            os.fsync(f.fileno())
            pys.encode_file(p, S, fk, ak, f)
            for reg, key in ((False, "api_file_mmap_gib_s"), (True, "api_file_mmap_register_gib_s")):
                r, same, ph = api(f, reg)
                out[key] = round(r, 3)
                out[key.replace("_gib_s", "_phases")] = ph
                api_ok = api_ok and same
            f.seek(0)
            tag, _ = pys.encode_file(p, S, fk, ak, f)
        out["api_prove_file"] = host_file_prove(ctx, L, dptr, pys, p, S, fh.name, n, tag)
        del tag
    bio = io.BytesIO(host.tobytes())
    pys.encode_file(p, S, fk, ak, bio)          # warm-up
    for reg, key in ((False, "api_bytesio_gib_s"), (True, "api_bytesio_register_gib_s")):
        r, same, _ = api(bio, reg)
        out[key] = round(r, 3)
        api_ok = api_ok and same
    # PySwizzle's default shape (1024-bit prime, S = 10) through the same API
    # on the same bytes: 256 MiB windows of 209,715 blocks, each on the
    # mid-size path (quad PRF + MFMA MAC)
    p1024 = seeded_prime(1024)
    pys.encode_file(p1024, 10, fk, ak, bio)          # warm-up (1024-bit kernels)
    best = None
    for _ in range(3):
        bio.seek(0)
        t0 = time.perf_counter()
        pys.encode_file(p1024, 10, fk, ak, bio)
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    out["api_bytesio_register_p1024_s10_gib_s"] = round(n / GIB / best, 3)
    del bio
    out["api_tags_equal"] = api_ok
    out["unit"] = "GiB/s"
    return out


def verify_timing(ctx, L, pb, S, fk, ak, nblocks, ck, chunks, mu, sg, reps):
    """PySwizzle.verify (PySwizzle.py:372-395) of that proof, timed: the
    right-hand side sum_i v_i F(idx_i) + sum_j alpha_j mu_j on the GPU
    (hb_verify_rhs), compared with sigma."""
    w = len(sg.raw)
    rhs = ctypes.create_string_buffer(w)

    def one():
        ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, len(fk), nblocks, ck, len(ck), chunks, pb, len(pb),
                                  mu.raw, rhs))

    for _ in range(min(10, reps)):
        one()
    t = time.perf_counter()
    for _ in range(reps):
        one()
    return {"ms_per_verify": round((time.perf_counter() - t) / reps * 1e3, 4), "verifies": reps,
            "verified": rhs.raw == sg.raw}


def prove_row(ctx, L, dptr, tptr, length, nblocks, S, p, C, w, args, fk, ak, proofs=200, chunks=10000):
    """configs[4] inside the default run: PySwizzle.prove (PySwizzle.py:333-370)
    of a 10,000-index challenge over the encode's own device-resident file and
    tags -- the same call as `--config c5`, `proofs` timed back to back after
    20 warm-ups.  Checked against the oracle without copying the file back:
    the oracle's KeyedPRF(key, #tags) gives the challenged indices
    (PySwizzle.py:344-345), only those blocks and tags are copied into an
    otherwise untouched (lazily zero) host image, and oracle/swizzle_oracle.c
    and the native CPU prove (baseline/hb_cpu_swizzle.cpp) prove on it."""
    from heartbeat_amd import _native
    pb = _native.be(p)
    ck = hashlib.sha256(b"hb-bench-challenge").digest()
    mu = ctypes.create_string_buffer(w * S)
    sg = ctypes.create_string_buffer(w)

    def one():
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, ck, len(ck), chunks, pb, len(pb), tptr, nblocks, dptr, length,
                             3, mu, sg))

    for _ in range(min(20, proofs)):
        one()
    t = time.perf_counter()
    for _ in range(proofs):
        one()
    ms = (time.perf_counter() - t) / proofs * 1e3
    launches = ctx.last_kernel_ms()[1]
    gib = length / GIB
    row = {"workload": "configs[4]: Swizzle prove() on this run's %g GiB device-resident file and tags, "
                       "10 000-index challenge, 256-bit prime, 16 sectors/block, 1 MI355X%s"
                       % (gib, "" if gib == 64 else " [not configs[4]'s 64 GiB]"),
           "ms_per_proof": round(ms, 4), "proofs": proofs, "chunks": chunks,
           "launches_per_proof": launches,
           "path": "fused PRF + weighted-sum launch (DESIGN.md 5.3)" if launches == 1 else
                   "PRF launch + hb_wsum_kernel"}
    row["verify"] = verify_timing(ctx, L, pb, S, fk, ak, nblocks, ck, chunks, mu, sg, max(2, proofs // 4))
    if args.no_cpu_baseline:
        return row
    import numpy as np
    from oracle import oracle as O
    idx = sorted({O.prf_eval(ck, nblocks, i) for i in range(chunks)})
    host = np.zeros(length, dtype=np.uint8)          # untouched pages stay unallocated
    tags = np.zeros(nblocks * w, dtype=np.uint8)
    for ix in idx:
        a = ix * C
        if a < length:
            ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data + a, dptr.value + a, min(C, length - a), 2))
        ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data + ix * w, tptr.value + ix * w, w, 2))
    ref_mu = ctypes.create_string_buffer(w * S)
    ref_sg = ctypes.create_string_buffer(w)
    rc = O.lib().hbo_prove(pb, len(pb), S, ck, len(ck), chunks, pb, len(pb), nblocks,
                           ctypes.cast(tags.ctypes.data, ctypes.c_char_p), w, host.ctypes.data, length, ref_mu, ref_sg)
    if rc:
        raise RuntimeError("oracle prove error %d" % rc)
    row["proof_equal_oracle"] = ref_mu.raw == mu.raw and ref_sg.raw == sg.raw
    row["oracle_check"] = ("%d distinct challenged blocks and tags copied back; oracle/swizzle_oracle.c proves on "
                           "them (indices from its own KeyedPRF)" % len(idx))
    from baseline import cpu as NC
    info = host_cpu_info()
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or info.get("affinity") or
                                      os.cpu_count() or 1)
    want_mu = [int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(S)]
    for th in sorted({1, threads}):
        NC.prove_raw(p, S, ck, chunks, p, nblocks, tags.ctypes.data, host.ctypes.data, length, th)   # warm-up
        t = time.perf_counter()
        k = 0
        while k < 3 or time.perf_counter() - t < 1.0:
            nmu, nsg = NC.prove_raw(p, S, ck, chunks, p, nblocks, tags.ctypes.data, host.ctypes.data, length, th)
            k += 1
        row["cpu_native_%d_threads_ms" % th] = round((time.perf_counter() - t) / k * 1e3, 4)
        row["cpu_native_equal_gpu"] = nmu == want_mu and nsg == int.from_bytes(sg.raw, "big")
    row["cpu_native"] = ("baseline/hb_cpu_swizzle.cpp prove (the cxx Swizzle counterpart) on the same host image, "
                         "1 and %d std::threads" % threads)
    return row


def _native_flag(name):
    from heartbeat_amd import _native
    return getattr(_native, name)


def bench_prove(args, cfg, R):
    """configs[4]: one step = one PySwizzle.prove (PySwizzle.py:333-370) over
    the device-resident file and tags: idx / v PRFs for `chunks` indices, the
    gathered weighted sums of the S sector columns and of the tags, and the
    mod-p reductions, with mu and sigma copied back to the host."""
    from heartbeat_amd import _native
    L = _native.lib()
    ctx = _native.context(R.device)
    S = cfg["sectors"]
    p = P256
    pb = _native.be(p)
    C = 32 * S
    w = 32
    length = int(args.gib * GIB) if args.gib is not None else cfg["gib_per_rank"] * GIB
    nblocks = length // C + 1
    fk = hashlib.sha256(b"hb-bench-f").digest()
    ak = hashlib.sha256(b"hb-bench-alpha").digest()
    dptr = ctypes.c_void_p()
    tptr = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, length, ctypes.byref(dptr)))
    ctx.check(L.hb_device_malloc(ctx.h, nblocks * w, ctypes.byref(tptr)))
    ctx.check(L.hb_fill_random(ctx.h, dptr, length, 0x5EED0000 + 3 + R.rank))
    chunks = cfg["prove_chunks"]
    cxx = args.prf == "cxx"
    pflags = 3 | (_native.HB_PRF_CXX if cxx else 0)
    ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, dptr, length, nblocks, tptr, pflags, None))
    ck = hashlib.sha256(b"hb-bench-challenge").digest()
    vb = pb                                   # v_max = p, as gen_challenge (PySwizzle.py:329)
    mu = ctypes.create_string_buffer(w * S)
    sg = ctypes.create_string_buffer(w)

    def step():
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, ck, len(ck), chunks, vb, len(vb), tptr, nblocks,
                             dptr, length, pflags, mu, sg))

    for _ in range(max(1, args.warmup)):
        step()
    steps = max(args.steps, 20)
    R.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    R.barrier()
    ms = R.reduce((time.perf_counter() - t0) / steps * 1e3, "max")
    line = {
        "metric": "Swizzle prove() latency, ms per proof (device-resident file and tags)",
        "value": round(ms, 4), "unit": "ms", "n_gpus": R.world,
        **R.device_report(_native.pci_bus_id(R.device)), "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": False, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (SplitMix64 random file bytes, seeded keys)",
        "config": {"workload": workload_name(args, cfg), "file_bytes": length, "blocks_total": nblocks,
                   "sectors": S, "prime_bits": 256, "chunks": chunks,
                   "prf": "cxx prf, cxx prove (parity unpinned)" if cxx else "PySwizzle KeyedPRF"},
        "gathered_bytes_per_proof": chunks * (C + w),
        "build": _native.build_info(),
    }
    if not cxx:
        line["verify"] = verify_timing(ctx, L, pb, S, fk, ak, nblocks, ck, chunks, mu, sg, max(2, steps // 4))
    if R.rank == 0 and not args.no_cpu_baseline and not cxx:
        import numpy as np
        from oracle import oracle as O
        host = np.empty(length, dtype=np.uint8)
        ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value, length, 2))
        tags = np.empty(nblocks * w, dtype=np.uint8)
        ctx.check(L.hb_memcpy(ctx.h, tags.ctypes.data, tptr.value, nblocks * w, 2))
        t = time.perf_counter()
        n = 0
        while n < 3 or time.perf_counter() - t < min(args.cpu_seconds, 5.0):
            ref_mu = ctypes.create_string_buffer(w * S)
            ref_sg = ctypes.create_string_buffer(w)
            rc = O.lib().hbo_prove(pb, len(pb), S, ck, len(ck), chunks, vb, len(vb), nblocks,
                                   ctypes.cast(tags.ctypes.data, ctypes.c_char_p), w,
                                   host.ctypes.data, length, ref_mu, ref_sg)
            if rc:
                raise RuntimeError("oracle prove error %d" % rc)
            n += 1
        cpu_ms = (time.perf_counter() - t) / n * 1e3
        oracle_row = {"value": round(cpu_ms, 3), "unit": "ms", "cores": 1, "kind": "port",
                      "sample": "%d proofs of the same challenge, oracle/swizzle_oracle.c (OpenSSL BIGNUM), "
                                "1 thread" % n}
        line["proof_equal_oracle"] = ref_mu.raw == mu.raw and ref_sg.raw == sg.raw
        # the "cxx Swizzle" counterpart (idx/s prove on configs[4]):
        # the native prove of baseline/hb_cpu_swizzle.cpp on the same host copy
        from baseline import cpu as NC
        info = host_cpu_info()
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or info.get("affinity") or
                                          os.cpu_count() or 1)
        nrow = {}
        for th in sorted({1, threads}):
            NC.prove_raw(p, S, ck, chunks, p, nblocks, tags.ctypes.data, host.ctypes.data, length, th)   # warm-up
            t = time.perf_counter()
            k = 0
            while k < 3 or time.perf_counter() - t < min(args.cpu_seconds, 5.0):
                nmu, nsg = NC.prove_raw(p, S, ck, chunks, p, nblocks, tags.ctypes.data, host.ctypes.data, length, th)
                k += 1
            nrow[th] = ((time.perf_counter() - t) / k * 1e3, k)
        want_mu = [int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(S)]
        ms_n, k_n = nrow[threads]
        line["cpu_baseline"] = {
            "value": round(ms_n, 4), "unit": "ms", "cores": threads, "kind": "port",
            "name": "cxx Swizzle counterpart: native prove (baseline/hb_cpu_swizzle.cpp, AES-NI index/v PRFs, "
                    "gather, 64-bit-limb MAC; reference loop cxx/shacham_waters_private.cxx:731-789)",
            "sample": "%d proofs of the same 10,000-index challenge on the host copy of the file, %d std::threads"
                      % (k_n, threads),
            "idx_per_s": round(chunks / (ms_n * 1e-3), 1),
            "one_thread_ms": round(nrow[1][0], 4),
            "cores_available": info.get("affinity") or info.get("nproc"),
            "proof_equal_gpu": nmu == want_mu and nsg == int.from_bytes(sg.raw, "big"),
            "oracle_row": oracle_row,
            "host": info}
        line["idx_per_s"] = round(chunks / (ms * 1e-3), 1)
        del host, tags
    if R.rank == 0:
        print(json.dumps(line), flush=True)
    ctx.check(L.hb_device_free(ctx.h, dptr))
    ctx.check(L.hb_device_free(ctx.h, tptr))


if __name__ == "__main__":
    main()
