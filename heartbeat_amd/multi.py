"""Multi-GPU encode / prove inside the drop-in API (BASELINE.json north_star:
"shard block ranges across the 8 GPUs of one node and concatenate per-GPU
tags on the host").

Blocks are independent (tag_i depends on the global index i, block i's bytes
and the keys; PySwizzle.py:296-309), so an encode over G devices gives device g
the contiguous block range of ``shard.shard_plan(len, C, g, G)`` with
``block_base`` = its first block, and every device writes its tags straight
into its slice of the one output buffer: the concatenation is free.  A prove
splits the challenge indices [0, chunks) the same way (hb_prove_range) and adds
the S + 1 partial sums mod p on the host.  No collective, no peer copies: each
device reads only its own part of the (host or device) file.

One host thread per device; ctypes releases the GIL during the calls, so the
devices run concurrently (and, for host-resident files, so do their PCIe
links).

Device selection, first match wins: ``set_devices([...])``; $HB_DEVICES
("0,1,2,3" or "all"); $HB_DEVICE (one device: the process is pinned); under a
launcher ($LOCAL_RANK) the rank's device; otherwise every visible device.
Every call of the drop-in API -- encode, prove, verify, KeyedPRF, Merkle --
uses ``devices()[0]`` as its single device, so one flow never touches a GPU
outside the selection.  Small jobs stay on one device: a shard gets at least
MIN_SHARD_BYTES of file (encode) or MIN_SHARD_CHUNKS challenge indices
(prove).  Device-resident buffers (HB_DATA_ON_DEVICE / HB_TAGS_ON_DEVICE) are
one device's memory: they are refused with more than one distinct device.
"""
import ctypes
import os
import threading

from . import _native
from .exc import HeartbeatError
from .shard import block_range, shard_plan

MIN_SHARD_BYTES = 256 << 20
MIN_SHARD_CHUNKS = 1 << 20

_devices = None


def set_devices(devices):
    """Devices used by encode / prove: a list of ordinals (repeats allowed:
    each entry is its own context), or None for the default."""
    global _devices
    _devices = None if devices is None else [int(d) for d in devices]


def visible_device_count():
    n = ctypes.c_int(0)
    rc = _native.lib().hb_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def devices(explicit=None):
    if explicit is not None:
        return [int(d) for d in explicit]
    if _devices is not None:
        return list(_devices)
    env = os.environ.get("HB_DEVICES", "").strip()
    if env and env != "all":
        return [int(x) for x in env.split(",") if x.strip()]
    pinned = any(os.environ.get(v, "").strip() for v in ("HB_DEVICE", "LOCAL_RANK"))
    if env == "all" or not pinned:
        n = visible_device_count()
        if n > 0:
            return list(range(n))
    return [_native.default_device()]


def primary_context():
    """The context of the first selected device: single-device calls
    (verify, KeyedPRF, Merkle) run where encode and prove run."""
    return _native.context(devices()[0])


def check_resident(flags, devs):
    """Device-resident input or output is one device's memory: no peer access
    is set up, so it cannot be split over several devices."""
    if flags & (_native.HB_DATA_ON_DEVICE | _native.HB_TAGS_ON_DEVICE) and len(set(devs)) > 1:
        raise HeartbeatError("device-resident buffers cannot be sharded over devices %s: "
                             "pass one device, or host buffers" % sorted(set(devs)))


def contexts(devs):
    """One context per entry of devs (a repeated ordinal gets a second context)."""
    seen = {}
    out = []
    for d in devs:
        k = seen.get(d, 0)
        seen[d] = k + 1
        out.append(_native.context(d, k))
    return out


def shard_count(ndev, amount, minimum):
    return max(1, min(ndev, amount // minimum if minimum else ndev))


def run_parallel(fns):
    """Run the callables on one thread each; re-raise the first error."""
    if len(fns) == 1:
        return [fns[0]()]
    res = [None] * len(fns)
    err = []

    def wrap(k):
        try:
            res[k] = fns[k]()
        except BaseException as e:   # noqa: BLE001 -- re-raised below
            err.append(e)

    ts = [threading.Thread(target=wrap, args=(k,)) for k in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    return res


def encode_shards(p, sectors, fk, ak, addr, length, nblocks, out_addr, flags, devs, min_bytes=MIN_SHARD_BYTES):
    """hb_encode of a whole file (host or device memory at addr) over devs;
    tags written to out_addr (nblocks * width bytes).  Returns PRF tries."""
    w = _native.width_of(p)
    C = (p.bit_length() // 8) * sectors
    G = shard_count(len(devs), length, min_bytes)
    check_resident(flags, devs[:G])
    ctxs = contexts(devs[:G])
    pb = _native.be(p)
    L = _native.lib()

    def job(g):
        plan = shard_plan(length, C, g, G)
        if plan["nblocks"] == 0:
            return 0
        ctx = ctxs[g]
        tries = ctypes.c_uint64(0)
        data = (addr + plan["byte_off"]) if (addr and plan["byte_len"]) else None
        with ctx.lock:
            ctx.check(L.hb_encode(ctx.h, pb, len(pb), sectors, fk, ak, len(fk), plan["b0"], data,
                                  plan["byte_len"], plan["nblocks"], out_addr + plan["b0"] * w, flags,
                                  ctypes.byref(tries)))
        return tries.value

    assert sum(shard_plan(length, C, g, G)["nblocks"] for g in range(G)) == nblocks
    return sum(run_parallel([lambda g=g: job(g) for g in range(G)]))


def prove_shards(p, sectors, key, chunks, vmax_be, tags_addr, ntags, data_addr, length, flags, devs,
                 min_chunks=MIN_SHARD_CHUNKS):
    """hb_prove over devs: challenge indices split into ranges, partial
    (mu, sigma) added mod p.  Returns (mu list, sigma)."""
    w = _native.width_of(p)
    G = shard_count(len(devs), chunks, min_chunks)
    check_resident(flags, devs[:G])
    ctxs = contexts(devs[:G])
    pb = _native.be(p)
    L = _native.lib()

    def job(g):
        i0, i1 = block_range(chunks, g, G)
        ctx = ctxs[g]
        mu = ctypes.create_string_buffer(w * sectors)
        sg = ctypes.create_string_buffer(w)
        with ctx.lock:
            ctx.check(L.hb_prove_range(ctx.h, pb, len(pb), sectors, key, len(key), chunks, i0, i1,
                                       vmax_be, len(vmax_be), tags_addr, ntags, data_addr, length, flags,
                                       mu, sg))
        return ([int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(sectors)],
                int.from_bytes(sg.raw, "big"))

    parts = run_parallel([lambda g=g: job(g) for g in range(G)])
    mu = [sum(pt[0][j] for pt in parts) % p for j in range(sectors)]
    sigma = sum(pt[1] for pt in parts) % p
    return mu, sigma
