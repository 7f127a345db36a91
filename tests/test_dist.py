"""Image-parallel multi-process path (ccmi.dist) with world_size 2 on the gloo backend (CPU):
sharding covers every image exactly once, records gather to every rank, counters reduce."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from ccmi import dist as cd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        images = [f"kodim{i:02d}" for i in range(1, 25)]
        mine = cd.shard(images, rank, world)
        recs = [{"name": n, "rank": rank, "pixels": 768 * 512} for n in mine]
        allrec = cd.gather_records(recs)
        tot = cd.reduce_counters({"pixels": sum(r["pixels"] for r in recs), "frames": len(recs)})
        mx = cd.reduce_counters({"seconds": 1.0 + rank}, op="max")
        q.put((rank, mine, allrec, tot, mx))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_aggregation():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [set(r[1]) for r in res]
    assert not shards[0] & shards[1]
    assert len(shards[0] | shards[1]) == 24
    for rank, _, allrec, tot, mx in res:
        assert sorted(r["name"] for r in allrec) == sorted(f"kodim{i:02d}" for i in range(1, 25))
        assert tot == {"frames": 24.0, "pixels": 24.0 * 768 * 512}
        assert mx == {"seconds": 2.0}


def test_shard_validates_rank():
    from ccmi import dist as cd
    with pytest.raises(ValueError):
        cd.shard([1, 2], 2, 2)
    assert cd.shard(list(range(5)), 1, 2) == [1, 3]
