"""bench.py's N>1 path on the gloo backend (world_size 2, CPU): the timed
replay with its per-step / per-chunk score gathers (staging layouts,
unpad, all_reduce(MAX) timing) driven by deterministic CPU "engines", and the
one-time model broadcast from rank 0 (fleet.broadcast_state) -- the code the
8-GPU scaling run executes, minus the GPU."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _score(s, t):
    return ((s * 7 + t) % 41) / 40.0


class FakeEngine:
    """Stands in for HTMEngine on the CPU: step/run write deterministic
    float32 scores for this rank's global streams [s0, s1); state regions are
    host byte arrays (export/import by stream)."""

    def __init__(self, s0, s1, regions=None, delay=0.0):
        self.s0, self.s1 = s0, s1
        self.delay = delay
        self.regions = regions or {}

    def step(self, vals, out):
        t = int(vals[0].item())
        out[:] = torch.tensor([_score(s, t) for s in range(self.s0, self.s1)], dtype=torch.float32)
        if self.delay:
            import time
            time.sleep(self.delay)

    def run(self, vals, out):
        for k in range(vals.shape[0]):
            self.step(vals[k], out[k])

    def state_bytes(self, r):
        return self.regions[r].shape[1]

    def export_state(self, r, s0, n):
        return self.regions[r][s0:s0 + n].copy()

    def import_state(self, r, data, s0=0):
        self.regions[r][s0:s0 + data.shape[0]] = data


def _worker(rank, world, port, n_total, steps, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import _pkg
    import bench
    fleet = _pkg.load().fleet
    g = fleet.ScoreGather(n_total)
    a, b = g.local_range
    n = b - a
    # rank 1 is slower: the reported time must be the max over ranks
    eng = FakeEngine(a, b, delay=0.02 if rank == 1 else 0.0)
    warm = 3
    vals = torch.arange(warm + steps, dtype=torch.float64)[:, None].repeat(1, n)  # value = step index
    scores = torch.zeros((warm + steps, n), dtype=torch.float32)
    gathered = None
    if rank == 0:
        gathered = (torch.empty((world, steps, g.width)) if mode == "run" else torch.empty((steps, world, g.width)))
    dt, gathered = bench.timed_replay(eng, vals, scores, warm, steps, mode, 2, g, gathered, rank, world, "cpu")
    if rank == 0:
        rows = g.unpad_rows(gathered) if mode == "run" else torch.stack([g.unpad(gathered[k]) for k in range(steps)])
        q.put((dt, rows.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,n_total", [("step", 8), ("step", 11), ("run", 8), ("run", 11)])
def test_timed_replay_two_ranks(mode, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 5
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, steps, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    dt, rows = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = np.array([[_score(s, 3 + t) for s in range(n_total)] for t in range(steps)], np.float32)
    assert np.array_equal(rows, want)  # every rank's scores, in global stream order, on rank 0
    assert dt >= steps * 0.02  # rank 1's sleeps: the max over ranks, not rank 0's own time


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import _pkg
    fleet = _pkg.load().fleet
    rng = np.random.default_rng(5)
    trained = {"sp_perm": rng.integers(0, 256, (1, 4096), dtype=np.uint8),
               "tm_seg_meta": rng.integers(0, 256, (1, 999), dtype=np.uint8),
               "tm_header": rng.integers(0, 256, (1, 300), dtype=np.uint8)}
    # rank 0 holds the trained model, the others a blank engine of the same config
    regions = {k: (v.copy() if rank == 0 else np.zeros_like(v)) for k, v in trained.items()}
    eng = FakeEngine(0, 1, regions=regions)
    nb = fleet.broadcast_state(eng, list(trained), src=0)
    ok = nb == sum(v.size for v in trained.values()) and all(np.array_equal(eng.regions[k], trained[k])
                                                              for k in trained)
    t = torch.tensor([0.0 if ok else 1.0])
    dist.all_reduce(t)
    if rank == 0:
        q.put(float(t.item()))
    dist.barrier()
    dist.destroy_process_group()


def test_model_broadcast_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    bad = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert bad == 0.0
