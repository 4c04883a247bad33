"""CPU stand-in for HTMEngine in bench.py's launcher test (bench.py
--cpu-standin, tests/test_bench_launch.py).  It does no HTM compute: step/run
write a deterministic function of (global stream, input value) so the test
can check that every rank stepped its own shard of the streams; the counters
and profile calls return the neutral values bench.py's line expects.  Never
used for a measurement (the line's "data" field says so)."""
import torch


def standin_score(stream, value):
    return ((int(stream) * 7 + int(value)) % 41) / 40.0


class StandInEngine:
    n_columns = 2048
    cells_per_column = 12
    fused = True

    def __init__(self, n_streams, s0):
        self.n_streams = n_streams
        self.s0 = s0
        self.steps = 0

    def set_run_chunk(self, steps):
        self.chunk = steps

    def set_run_unit(self, steps):
        pass

    def step(self, values, out):
        g = torch.arange(self.s0, self.s0 + self.n_streams, dtype=torch.float64)
        out.copy_(((g * 7 + values.to(torch.float64).floor()) % 41 / 40.0).to(torch.float32))
        self.steps += 1

    def run(self, values, out):
        for k in range(values.shape[0]):
            self.step(values[k], out[k])

    def flush(self):
        pass

    def counters(self):
        return dict(tm_bytes=0, inf_phase2=self.steps, inf_backtracks=0, lrn_phase2=0, lrn_backtracks=0,
                    seg_live=0, seg_hwm=0, error=0)

    def profile(self, on):
        pass

    def profile_read(self):
        return dict(sp_ms=0.0, tm_ms=0.0, steps=0, launches=0)

    def close(self):
        pass
