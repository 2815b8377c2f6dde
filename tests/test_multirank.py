"""N > 1 path on CPU: two gloo ranks shard one encode by block range
(heartbeat_amd.shard) and their tags, gathered in rank order, equal the
single-process tags.  The per-rank compute here is the CPU oracle (no GPU in
this container); on the GPU each rank runs hb_encode on the same plan
(bench.py, tests/test_gpu_parity.py::test_shards_concatenate)."""
import os
import socket

import pytest

P256 = int("db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b", 16)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data(n):
    import hashlib
    out = b""
    i = 0
    while len(out) < n:
        out += hashlib.sha256(b"mr%d" % i).digest()
        i += 1
    return out[:n]


def _worker(rank, world, port, L, S, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from heartbeat_amd.shard import shard_plan
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            init_method="tcp://127.0.0.1:%d" % port)
    data = _data(L)
    C = 32 * S
    plan = shard_plan(L, C, rank, world)
    part = data[plan["byte_off"]:plan["byte_off"] + plan["byte_len"]]
    tags = O.encode(P256, S, b"f" * 32, b"a" * 32, part, block_base=plan["b0"],
                    nblocks=plan["nblocks"])
    got = [None] * world
    dist.all_gather_object(got, tags)
    if rank == 0:
        q.put([t for r in got for t in r])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("L,S", [(512 * 1001 + 7, 16), (512 * 1000, 16), (32 * 777, 1)])
def test_two_rank_shards_equal_single(L, S):
    import torch.multiprocessing as mp
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, L, S, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = O.encode(P256, S, b"f" * 32, b"a" * 32, _data(L))
    assert merged == full


def test_shard_plan_covers_file():
    from heartbeat_amd.shard import shard_plan
    for L, C, N in ((0, 512, 2), (511, 512, 3), (512 * 8, 512, 8), (10 ** 6 + 3, 1280, 7)):
        plans = [shard_plan(L, C, r, N) for r in range(N)]
        assert sum(p["nblocks"] for p in plans) == L // C + 1
        assert sum(p["byte_len"] for p in plans) == L
        for a, b in zip(plans, plans[1:]):
            assert a["b0"] + a["nblocks"] == b["b0"]
            assert a["byte_off"] + a["byte_len"] == b["byte_off"] or b["byte_len"] == 0


def test_multi_device_selection(monkeypatch):
    """heartbeat_amd.multi: device list resolution and shard counts."""
    from heartbeat_amd import multi
    monkeypatch.setenv("HB_DEVICES", "0,0,1")
    assert multi.devices() == [0, 0, 1]
    assert multi.devices([3]) == [3]
    multi.set_devices([2, 5])
    try:
        assert multi.devices() == [2, 5]
    finally:
        multi.set_devices(None)
    # small files stay on one device; large ones use every device
    assert multi.shard_count(8, 10 << 20, multi.MIN_SHARD_BYTES) == 1
    assert multi.shard_count(8, 3 * multi.MIN_SHARD_BYTES, multi.MIN_SHARD_BYTES) == 3
    assert multi.shard_count(8, 64 << 30, multi.MIN_SHARD_BYTES) == 8
    assert multi.shard_count(2, 0, multi.MIN_SHARD_CHUNKS) == 1


def test_multi_run_parallel_order_and_errors():
    from heartbeat_amd import multi
    assert multi.run_parallel([lambda k=k: k * k for k in range(5)]) == [0, 1, 4, 9, 16]

    def boom():
        raise ValueError("x")
    with pytest.raises(ValueError):
        multi.run_parallel([lambda: 1, boom])


def test_prove_partition_sums_mod_p(oracle):
    """hb_prove_range's contract on the oracle: partial proofs over a partition
    of the challenge indices add mod p to the whole proof (PySwizzle.py:351-368
    sums over i)."""
    import hashlib
    p = P256
    S = 3
    data = b"".join(hashlib.sha256(b"pp%d" % i).digest() for i in range(200))
    tags = oracle.encode(p, S, b"f" * 32, b"a" * 32, data)
    key = b"k" * 32
    mu, sg = oracle.prove(p, S, key, 40, p, tags, data)
    # the oracle proves whole challenges only; restate the partition on ints
    from oracle import oracle as O
    idx = [O.prf_eval(key, len(tags), i) for i in range(40)]
    v = [O.prf_eval(key, p, i) for i in range(40)]
    C = 32 * S

    def part(a, b):
        m = [sum(v[i] * int.from_bytes(data[idx[i] * C + j * 32: idx[i] * C + (j + 1) * 32], "big")
                 for i in range(a, b)) % p for j in range(S)]
        return m, sum(v[i] * tags[idx[i]] for i in range(a, b)) % p

    parts = [part(0, 13), part(13, 27), part(27, 40)]
    assert [sum(x[0][j] for x in parts) % p for j in range(S)] == mu
    assert sum(x[1] for x in parts) % p == sg


def test_hb_device_pins_every_call(monkeypatch):
    """$HB_DEVICE pins the process to one device: encode, prove and the
    single-device calls (verify, KeyedPRF, Merkle: multi.primary_context)
    all resolve to it, whatever the visible device count."""
    from heartbeat_amd import multi
    monkeypatch.delenv("HB_DEVICES", raising=False)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.setattr(multi, "visible_device_count", lambda: 8)
    assert multi.devices() == list(range(8))          # unpinned: every device
    monkeypatch.setenv("HB_DEVICE", "3")
    assert multi.devices() == [3]
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert multi.devices() == [3]                     # HB_DEVICE before LOCAL_RANK
    monkeypatch.delenv("HB_DEVICE")
    assert multi.devices() == [5]
    monkeypatch.setenv("HB_DEVICES", "6,7")
    assert multi.devices() == [6, 7]                  # an explicit list wins
    opened = []
    monkeypatch.setattr(multi._native, "context", lambda d=None, k=0: opened.append(d) or d)
    assert multi.primary_context() == 6 and opened == [6]


def test_device_resident_buffers_refuse_several_devices():
    """HB_DATA_ON_DEVICE / HB_TAGS_ON_DEVICE pointers belong to one device:
    sharding them over distinct devices is refused before any call."""
    from heartbeat_amd import multi, _native
    from heartbeat_amd.exc import HeartbeatError
    for flags in (_native.HB_DATA_ON_DEVICE, _native.HB_TAGS_ON_DEVICE,
                  _native.HB_DATA_ON_DEVICE | _native.HB_TAGS_ON_DEVICE):
        with pytest.raises(HeartbeatError, match="device-resident"):
            multi.check_resident(flags, [0, 1])
        with pytest.raises(HeartbeatError):
            multi.encode_shards(P256, 16, b"f" * 32, b"a" * 32, 1 << 20, 4 << 30, (4 << 30) // 512 + 1,
                                1 << 20, flags, [0, 1, 0, 1])
        with pytest.raises(HeartbeatError):
            multi.prove_shards(P256, 16, b"k" * 32, 1 << 22, P256.to_bytes(32, "big"), 1 << 20, 100,
                               1 << 20, 4 << 30, flags, [2, 3])
        multi.check_resident(flags, [1, 1])            # one device (two contexts): fine
    multi.check_resident(0, [0, 1])                    # host buffers shard freely
