#!/usr/bin/env python3
"""Swizzle encode benchmark (BASELINE.json metric: GiB/s of file bytes tagged,
Swizzle encode, device-resident).

One step = one pass of the encode hot path (hb_encode: alpha PRF + Montgomery
conversion + the encode kernel) over every block of this rank's device-resident
synthetic file.  Workload (BASELINE.json configs):
  c3 (default): configs[2], 64 GiB random file, 256-bit prime, 16 sectors per
                block -- the largest single-GPU configuration; for N > 1 every
                rank encodes its own 64 GiB block-range shard of an N*64 GiB file
                (weak scaling, no collective: blocks are independent).
  c2:           configs[1], 1 GiB, 256-bit prime, 1 sector per block.
  c4:           configs[3], 256 GiB file sharded over the N ranks (256/N GiB each).
Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run, one rank per GPU (RCCL is used only for the barrier and
the max-over-ranks time).

Besides the contract fields the JSON line carries
  roofline:     the encode kernel's algorithmic file bytes per launch / its mean
                duration (HIP events on the kernel's stream) against the HBM
                read peak; traffic from the rocprofv3 PMC pass when recorded in
                profiles/ for this workload, else null; plus the LDS-lookup
                rate, the resource that actually binds.
  cpu_baseline: the repo's C oracle (OpenSSL AES-NI + BIGNUM, pthreads) timed on
                this host on a bounded prefix of the same file (rank 0, N = 1).
"""
import argparse
import ctypes
import hashlib
import json
import os
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
                    "16 sectors/block, block ranges sharded over N GPUs",
               gib_total=256, sectors=16, weak=False),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--gib", type=float, default=None, help="override file GiB per rank")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--single-pass", action="store_true",
                    help="one-pass PRF engine instead of prefix-image first pass + retry pass")
    ap.add_argument("--prf", default="pyswizzle", choices=["pyswizzle", "cxx"],
                    help="pyswizzle: KeyedPRF, tags bit-exact vs PySwizzle (the headline); cxx: the "
                         "cxx Swizzle extension's PRF (cxx/prf.hxx, CFB-128), parity unpinned")
    ap.add_argument("--host-path", action="store_true",
                    help="also time the pinned/pageable host path on a 4 GiB prefix (DESIGN.md)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from heartbeat_amd import _native
    L = _native.lib()
    ctx = _native.context(local)

    cfg = CONFIGS[args.config]
    S = cfg["sectors"]
    p = P256
    pb = _native.be(p)
    ss, w = 32, 32
    C = ss * S
    if args.gib is not None:
        file_len = int(args.gib * GIB) * world
    elif cfg["weak"]:
        file_len = cfg["gib_per_rank"] * GIB * world
    else:
        file_len = cfg["gib_total"] * GIB
    # rank r encodes its block range of one file of file_len bytes
    from heartbeat_amd.shard import shard_plan
    plan = shard_plan(file_len, C, rank, world)
    global_blocks = plan["total_blocks"]
    b0 = plan["b0"]
    nblocks = plan["nblocks"]
    length = plan["byte_len"]                        # this rank's bytes

    fk = hashlib.sha256(b"hb-bench-f").digest()
    ak = hashlib.sha256(b"hb-bench-alpha").digest()

    dptr = ctypes.c_void_p()
    tptr = ctypes.c_void_p()
    ctx.check(L.hb_device_malloc(ctx.h, length, ctypes.byref(dptr)))
    ctx.check(L.hb_device_malloc(ctx.h, nblocks * w, ctypes.byref(tptr)))
    # each rank fills its shard from its own seeded stream (bytes do not affect the work)
    ctx.check(L.hb_fill_random(ctx.h, dptr, length, 0x5EED0000 + 3 + rank))
    if "prove_chunks" in cfg:
        return bench_prove(args, cfg, ctx, L, dptr, tptr, length, nblocks, S, p, pb, fk, ak, C, rank)

    tries = ctypes.c_uint64()
    cxx = args.prf == "cxx"
    flags = 3 | (_native.HB_ENCODE_SINGLE_PASS if args.single_pass else 0) | (_native.HB_PRF_CXX if cxx else 0)

    def step():
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, b0, dptr, length, nblocks, tptr,
                              flags, ctypes.byref(tries)))
        return ctx.last_kernel_ms()[0]

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        kms.append(step())
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_bytes = file_len * args.steps
    value = total_bytes / GIB / elapsed
    kernel_ms = sum(kms) / len(kms)
    achieved_gbs = length / (kernel_ms * 1e-3) / 1e9
    tries_per_block = tries.value / nblocks
    # nb = 32 byte-0 AES-256 per try (197 LDS lookups each); the two-pass
    # encode replaces the first 4 of every block's first try by prefix-image
    # loads and builds that image (2^24 + 2^16 + 2^8 AES) once per step
    if cxx:
        # cxx prf: 2 full AES-256 per try (CFB-128 over 32 bytes), 16 * 14 lookups each
        aes = tries.value * 2
        lookups = aes * 16 * 14
    else:
        aes = tries.value * 32
        if not args.single_pass:
            aes += (1 << 24) + (1 << 16) + (1 << 8) - 4 * nblocks
        lookups = aes * (16 * 12 + 5)
    lds_rate = lookups / (kernel_ms * 1e-3)
    lds_peak = NUM_CUS * CLOCK_GHZ * 1e9 * LDS_LOOKUPS_PER_CLK_CU

    traffic = None
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            rec = json.load(open(prof)).get(args.config + ("_cxx" if cxx else ""))
            if rec and rec.get("file_bytes") == length:
                traffic = rec["hbm_bytes_per_launch"]
        except (ValueError, KeyError):
            traffic = None

    line = {
        "metric": "GiB/s file bytes tagged (Swizzle encode, device-resident) at 1/2/4/8 GPUs",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak" if cfg["weak"] else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (SplitMix64 random file bytes, seeded keys)",
        "config": {
            "workload": cfg["name"],
            "file_bytes": file_len,
            "file_bytes_per_rank": length,
            "blocks_total": global_blocks,
            "sectors": S,
            "prime_bits": 256,
            "prime": hex(p),
            "expected_tries_per_prf": round(2.0 ** 256 / p, 4),
            "prf": "cxx Swizzle prf (cxx/prf.hxx:125-176, CFB-128 over SHA256(LE32 i)); parity unpinned"
                   if cxx else "PySwizzle KeyedPRF (util.py:83-96, CFB-8 over SHA256(str(i))); bit-exact",
            "parallelism": "dp%d block-range shards, no collective" % world,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": "hb_cxx_encode_kernel" if cxx else "hb_encode_kernel" if args.single_pass else
                      "hb_prefix_kernel + hb_encode_first_kernel + hb_encode_retry_kernel",
            "kernel_ms": round(kernel_ms, 3),
            "algorithmic_bytes_per_launch": length,
            "binding_resource": {
                "resource": "LDS ds_read_b32 T-table lookups",
                "achieved_per_s": lds_rate,
                "peak_per_s": lds_peak,
                "frac": round(lds_rate / lds_peak, 4),
            },
        },
        "prf_tries_per_block": round(tries_per_block, 4),
        "aes_per_block": round(aes / nblocks, 3),
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(ctx, L, dptr, length, S, p, fk, ak, C,
                                            args.cpu_seconds, args.cpu_threads, cxx)
    if rank == 0 and args.host_path:
        line["host_path"] = host_path(ctx, L, dptr, length, S, pb, fk, ak, C)

    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.check(L.hb_device_free(ctx.h, dptr))
    ctx.check(L.hb_device_free(ctx.h, tptr))
    if dist is not None:
        dist.destroy_process_group()


def bench_prove(args, cfg, ctx, L, dptr, tptr, length, nblocks, S, p, pb, fk, ak, C, rank):
    """configs[4]: one step = one PySwizzle.prove (PySwizzle.py:333-370) over
    the device-resident file and tags: idx / v PRFs for `chunks` indices, the
    gathered weighted sums of the S sector columns and of the tags, and the
    mod-p reductions, with mu and sigma copied back to the host."""
    chunks = cfg["prove_chunks"]
    # --prf cxx: the cxx extension's prove (shacham_waters_private.cxx:731-789)
    from heartbeat_amd import _native
    cxx = args.prf == "cxx"
    pflags = 3 | (_native.HB_PRF_CXX if cxx else 0)
    ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, dptr, length, nblocks, tptr, pflags, None))
    ck = hashlib.sha256(b"hb-bench-challenge").digest()
    vb = pb                                   # v_max = p, as gen_challenge (PySwizzle.py:329)
    w = 32
    mu = ctypes.create_string_buffer(w * S)
    sg = ctypes.create_string_buffer(w)

    def step():
        ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, ck, len(ck), chunks, vb, len(vb), tptr, nblocks,
                             dptr, length, pflags, mu, sg))

    for _ in range(max(1, args.warmup)):
        step()
    steps = max(args.steps, 20)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ms = (time.perf_counter() - t0) / steps * 1e3
    line = {
        "metric": "Swizzle prove() latency, ms per proof (device-resident file and tags)",
        "value": round(ms, 4), "unit": "ms", "n_gpus": 1, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": False, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (SplitMix64 random file bytes, seeded keys)",
        "config": {"workload": cfg["name"], "file_bytes": length, "blocks_total": nblocks,
                   "sectors": S, "prime_bits": 256, "chunks": chunks,
                   "prf": "cxx prf, cxx prove (parity unpinned)" if cxx else "PySwizzle KeyedPRF"},
        "gathered_bytes_per_proof": chunks * (C + w),
    }
    if rank == 0 and not args.no_cpu_baseline and not cxx:
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
        line["cpu_baseline"] = {"value": round(cpu_ms, 3), "unit": "ms", "cores": 1, "kind": "port",
                                "sample": "%d proofs of the same challenge, oracle/swizzle_oracle.c "
                                          "(OpenSSL), 1 thread" % n}
        line["proof_equal_oracle"] = ref_mu.raw == mu.raw and ref_sg.raw == sg.raw
        del host, tags
    print(json.dumps(line), flush=True)
    ctx.check(L.hb_device_free(ctx.h, dptr))
    ctx.check(L.hb_device_free(ctx.h, tptr))


def cpu_baseline(ctx, L, dptr, length, S, p, fk, ak, C, seconds, threads, cxx=False):
    """Oracle (kind "port") on successive 256 MiB prefixes of the same file
    until `seconds` of CPU work, on `threads` host threads."""
    import numpy as np
    from oracle import oracle as O
    threads = max(1, min(threads, os.cpu_count() or 1))
    piece = (256 << 20) // C * C
    host = np.empty(piece, dtype=np.uint8)
    out = np.empty((piece // C) * 32, dtype=np.uint8)
    done = 0
    busy = 0.0
    off = 0
    while busy < seconds and off < length:
        n = min(piece, length - off)
        ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value + off, n, 2))
        nb = n // C
        t = time.perf_counter()
        rc = O.encode_raw(p, S, fk, ak, host.ctypes.data, n, off // C, nb, out.ctypes.data, threads, cxx)
        busy += time.perf_counter() - t
        if rc:
            raise RuntimeError("oracle error %d" % rc)
        done += n
        off += n
    return {"value": round(done / GIB / busy, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": "%d MiB prefix of the same synthetic file (%d blocks), oracle/swizzle_oracle.c "
                      "(%s), %d pthreads, %.1f s" % (
                          done >> 20, done // C,
                          "cxx prf: OpenSSL AES-NI CFB-128 + BIGNUM" if cxx else
                          "OpenSSL AES-NI CFB8 + BIGNUM", threads, busy)}


def host_path(ctx, L, dptr, length, S, pb, fk, ak, C):
    """Rate with the file and the tags in host memory (the boundary of a
    file-like object in, tag bytes out): chunked H2D of sectors + encode + D2H
    of tags, all inside the timed region, once from a pageable buffer and once
    from the same buffer page-locked with hb_host_register (pinned DMA)."""
    import numpy as np
    n = min(length, 4 * GIB) // C * C
    host = np.empty(n, dtype=np.uint8)
    ctx.check(L.hb_memcpy(ctx.h, host.ctypes.data, dptr.value, n, 2))
    nb = n // C
    tags = np.empty(nb * 32, dtype=np.uint8)
    ref = np.empty(nb * 32, dtype=np.uint8)
    out = {"bytes": n, "chunk": "256 MiB of whole blocks, double-buffered, H2D / D2H on a copy stream"}

    def run(dst):
        t = time.perf_counter()
        ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, host.ctypes.data, n, nb,
                              dst.ctypes.data, 0, None))
        return time.perf_counter() - t

    run(ref)   # warm-up (staging buffers, prefix image allocation)
    out["pageable_gib_s"] = round(n / GIB / run(tags), 3)
    ok = bool(np.array_equal(tags, ref))
    ctx.check(L.hb_host_register(ctx.h, host.ctypes.data, n))
    ctx.check(L.hb_host_register(ctx.h, tags.ctypes.data, tags.nbytes))
    try:
        run(tags)
        out["pinned_gib_s"] = round(n / GIB / run(tags), 3)
        ok = ok and bool(np.array_equal(tags, ref))
    finally:
        ctx.check(L.hb_host_unregister(ctx.h, tags.ctypes.data))
        ctx.check(L.hb_host_unregister(ctx.h, host.ctypes.data))
    out["pinned_tags_equal_pageable"] = ok
    out["unit"] = "GiB/s"
    return out


if __name__ == "__main__":
    main()
