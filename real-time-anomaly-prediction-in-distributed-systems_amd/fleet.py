"""Streams across GPUs: one process per GPU, streams sharded by rank, and the
per-step gather of anomaly scores to rank 0.

The reference runs one model per process with no collectives at all
(ML/HTM/ModelTesting.py:194-213); its only cross-host channel is Kafka.  Here
the N independent streams are split into contiguous blocks, one per rank
(weak scaling: no data-path exchange, each rank steps its own engine), and
the only collective is a gather of each step's float32 scores to rank 0 --
the input of the SLO alerting (`ModelTesting.py:75-99`).  On ROCm the
`torch.distributed` "nccl" backend is RCCL over xGMI; the same code runs on
"gloo" for CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous stream block [s0, s1) of `rank`: the first n_total % world
    ranks own one extra stream."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    s0 = rank * base + min(rank, extra)
    return s0, s0 + base + (1 if rank < extra else 0)


class ScoreGather:
    """Per-step gather of every rank's scores [n_local] to rank `dst`.

    Shards may be uneven; each rank's block is padded to the largest one so
    one fixed-size collective serves every step.  `gather(scores, out_row)`
    is asynchronous (returns the work handle); after `wait()` rank `dst`'s
    `out_row` ([n_total] view) holds the scores in global stream order."""

    def __init__(self, n_total: int, group=None, dst: int = 0):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst = dst
        self.n_total = n_total
        self.ranges = [shard_range(n_total, self.world, r) for r in range(self.world)]
        self.width = max(b - a for a, b in self.ranges)
        self._pending = []
        self._pads = {}  # uneven shards: reused padded send buffers (a small ring per shape)

    PAD_RING = 4

    def _padded(self, x):
        """x [..., n_local] copied into a reused [..., width] zero-padded send
        buffer.  A ring of PAD_RING buffers per shape: a slot is reused only
        after the collective that read it last has completed (its handle is
        waited for), so the async gathers in flight never see a later copy."""
        import torch
        key = (tuple(x.shape), x.dtype, str(x.device))
        ring = self._pads.get(key)
        if ring is None:
            shape = tuple(x.shape[:-1]) + (self.width,)
            ring = self._pads[key] = [[torch.zeros(shape, dtype=x.dtype, device=x.device), None, 0]
                                      for _ in range(self.PAD_RING)]
            ring.append(0)  # next slot
        i = ring[-1]
        ring[-1] = (i + 1) % self.PAD_RING
        slot = ring[i]
        if slot[1] is not None:
            slot[1].wait()
            slot[1] = None
        slot[0][..., :x.shape[-1]].copy_(x)
        return slot

    @staticmethod
    def _track(slot, h):
        if slot is not None:
            slot[1] = h

    @property
    def local_range(self):
        return self.ranges[self.rank]

    def gather(self, scores, staging=None):
        """Start gathering this rank's `scores` (device or CPU tensor).
        `staging` ([world, width], rank dst only) receives the padded blocks;
        returns (handle, staging)."""
        import torch
        n = scores.numel()
        if n != self.ranges[self.rank][1] - self.ranges[self.rank][0]:
            raise ValueError("scores do not match this rank's shard")
        src, slot = scores, None
        if n != self.width:
            slot = self._padded(scores)
            src = slot[0]
        if self.rank == self.dst:
            if staging is None:
                staging = torch.empty((self.world, self.width), dtype=scores.dtype, device=scores.device)
            gl = list(staging.unbind(0))
        else:
            gl = None
        h = self.dist.gather(src.contiguous(), gather_list=gl, dst=self.dst, group=self.group, async_op=True)
        self._track(slot, h)
        return h, staging

    def gather_rows(self, block, staging=None):
        """Start gathering a block of steps at once: this rank's `block`
        [m, n_local] (one htm_run chunk of scores) -> rank dst's `staging`
        [world, m, width] (allocated if None).  One collective per chunk
        instead of one per step.  Returns (handle, staging)."""
        import torch
        m, n = block.shape
        if n != self.ranges[self.rank][1] - self.ranges[self.rank][0]:
            raise ValueError("block does not match this rank's shard")
        src, slot = block, None
        if n != self.width:
            slot = self._padded(block)
            src = slot[0]
        gl = None
        if self.rank == self.dst:
            if staging is None:
                staging = torch.empty((self.world, m, self.width), dtype=block.dtype, device=block.device)
            gl = [staging[r] for r in range(self.world)]
            if not all(t.is_contiguous() and t.shape == (m, self.width) for t in gl):
                raise ValueError("staging must hold a contiguous [m, width] block per rank")
        h = self.dist.gather(src.contiguous(), gather_list=gl, dst=self.dst, group=self.group, async_op=True)
        self._track(slot, h)
        return h, staging

    def unpad_rows(self, staging):
        """[world, m, width] padded blocks -> [m, n_total] in global stream order."""
        import torch
        return torch.cat([staging[r, :, : b - a] for r, (a, b) in enumerate(self.ranges)], dim=1)

    def unpad(self, staging):
        """[world, width] padded blocks -> [n_total] in global stream order."""
        import torch
        return torch.cat([staging[r, : b - a] for r, (a, b) in enumerate(self.ranges)])


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """The slowest rank's time (the bench contract's max over ranks): one
    all_reduce(MAX) of a float64 on `device` (CPU tensor for gloo)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(seconds)
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def broadcast_state(engine, regions, src: int = 0, stream: int = 0, device=None, group=None) -> int:
    """Broadcast stream `stream`'s state from rank `src` into stream `stream`
    of every other rank's engine: each region exported to host bytes
    (htm_export_state), packed into ONE uint8 tensor, one `dist.broadcast`
    (RCCL over xGMI when `device` is a GPU), imported (htm_import_state).

    This is the one-time shared-model distribution of fleet mode (SURVEY.md
    §5, §8(e)): rank 0 trains the model, the other ranks receive it instead of
    re-training.  `engine` needs state_bytes / export_state / import_state;
    `regions` names the regions to send (their sizes agree on every rank,
    since the engines share a config).  Returns the bytes broadcast."""
    import torch
    import torch.distributed as dist
    sizes = [int(engine.state_bytes(r)) for r in regions]
    total = sum(sizes)
    rank = dist.get_rank(group)
    if rank == src:
        host = np.concatenate([engine.export_state(r, stream, 1).reshape(-1) for r in regions])
        buf = torch.from_numpy(host).to(device) if device is not None else torch.from_numpy(host)
    else:
        buf = torch.empty(total, dtype=torch.uint8, device=device)
    dist.broadcast(buf, src=src, group=group)
    if rank != src:
        host = buf.cpu().numpy()
        off = 0
        for r, n in zip(regions, sizes):
            engine.import_state(r, host[off:off + n].reshape(1, n), s0=stream)
            off += n
    return total
