"""N > 1 path on CPU: world-size-2 gloo processes run the sharding + the per-batch pose
all-gather exactly as bench.py does over RCCL (the front-end kernels themselves need a GPU and
are covered by the gpu tests)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_seq, q):
    import sys
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(here, "ssf-slam_amd"))
    from ssf import dist as sd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = sd.sequence_shard(n_seq, world, rank)
        B = len(mine)
        pose_abs = torch.zeros((B, 7), dtype=torch.float64)
        pose_abs[:, 3] = 1.0
        pose_abs[:, 4] = torch.tensor([float(s) for s in mine])       # t.x = sequence id
        mask_out = torch.zeros((B, 32), dtype=torch.float64)
        mask_out[:, 0] = torch.tensor([100.0 + s for s in mine])
        rec = sd.pose_record(pose_abs, mask_out)
        allp = sd.gather_poses(rec)
        # max-over-ranks timing reduction used by bench.py
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, list(mine), allp.numpy().tolist(), float(t.item())))
    finally:
        dist.destroy_process_group()


def test_sequence_shard_covers_all():
    import ssf.dist as sd
    for n in (1, 7, 8, 256, 1000):
        for w in (1, 2, 3, 8):
            got = [s for r in range(w) for s in sd.sequence_shard(n, w, r)]
            assert got == list(range(n))


@pytest.mark.timeout(120)
def test_gloo_world2_pose_allgather():
    world, n_seq = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_seq, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    res.sort()
    for rank, mine, allp, tmax in res:
        assert tmax == 2.0
        assert len(allp) == n_seq
        assert [row[4] for row in allp] == [float(s) for s in range(n_seq)]
        assert [row[7] for row in allp] == [100.0 + s for s in range(n_seq)]
