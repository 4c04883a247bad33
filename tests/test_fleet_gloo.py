"""Multi-process stream sharding + score gather on the gloo backend
(world_size 2, CPU): the N>1 path of bench.py without a GPU."""
import os
import socket

import numpy as np
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


def test_shard_range_partitions(rt):
    from rtap_amd.fleet import shard_range
    for n in [0, 1, 7, 1024, 1025]:
        for world in [1, 2, 3, 8]:
            got = [shard_range(n, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(got[r][1] == got[r + 1][0] for r in range(world - 1))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _worker(rank, world, port, n_total, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _pkg
    fleet = _pkg.load().fleet
    g = fleet.ScoreGather(n_total)
    a, b = g.local_range
    out = []
    for t in range(steps):
        # stream s at step t scores (s * 7 + t) % 41 / 40 (float32, like k/40)
        local = torch.tensor([((s * 7 + t) % 41) / 40.0 for s in range(a, b)], dtype=torch.float32)
        h, staging = g.gather(local)
        h.wait()
        if rank == 0:
            out.append(g.unpad(staging).numpy())
    # the same scores as one block of all steps (bench.py run mode: one gather per chunk)
    blk = torch.tensor([[((s * 7 + t) % 41) / 40.0 for s in range(a, b)] for t in range(steps)], dtype=torch.float32)
    h, staging = g.gather_rows(blk)
    h.wait()
    if rank == 0:
        q.put(np.stack(out))
        q.put(g.unpad_rows(staging).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [8, 11])
def test_score_gather_two_ranks(rt, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 5
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    got_rows = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = np.array([[((s * 7 + t) % 41) / 40.0 for s in range(n_total)] for t in range(steps)], np.float32)
    assert np.array_equal(got, want)
    assert np.array_equal(got_rows, want)
