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
