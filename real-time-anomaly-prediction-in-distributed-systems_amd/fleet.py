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
        src = scores
        if n != self.width:
            src = torch.zeros(self.width, dtype=scores.dtype, device=scores.device)
            src[:n] = scores
        if self.rank == self.dst:
            if staging is None:
                staging = torch.empty((self.world, self.width), dtype=scores.dtype, device=scores.device)
            gl = list(staging.unbind(0))
        else:
            gl = None
        h = self.dist.gather(src.contiguous(), gather_list=gl, dst=self.dst, group=self.group, async_op=True)
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
        src = block
        if n != self.width:
            src = torch.zeros((m, self.width), dtype=block.dtype, device=block.device)
            src[:, :n] = block
        gl = None
        if self.rank == self.dst:
            if staging is None:
                staging = torch.empty((self.world, m, self.width), dtype=block.dtype, device=block.device)
            gl = [staging[r] for r in range(self.world)]
            if not all(t.is_contiguous() and t.shape == (m, self.width) for t in gl):
                raise ValueError("staging must hold a contiguous [m, width] block per rank")
        h = self.dist.gather(src.contiguous(), gather_list=gl, dst=self.dst, group=self.group, async_op=True)
        return h, staging

    def unpad_rows(self, staging):
        """[world, m, width] padded blocks -> [m, n_total] in global stream order."""
        import torch
        return torch.cat([staging[r, :, : b - a] for r, (a, b) in enumerate(self.ranges)], dim=1)

    def unpad(self, staging):
        """[world, width] padded blocks -> [n_total] in global stream order."""
        import torch
        return torch.cat([staging[r, : b - a] for r, (a, b) in enumerate(self.ranges)])
