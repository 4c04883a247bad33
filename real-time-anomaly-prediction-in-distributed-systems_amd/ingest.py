"""Ingestion of the reference's aggregate records into batched engine inputs
(SURVEY.md §8(f)-4).

The reference's StreamAggregator joins each node's `stats` (cpu%, mem%) and
`responsetime` messages per epoch and emits one JSON record per epoch
(StreamEngine/StreamAggregator.py:101-115): count, mem, max, timestamp,
summation, violations, cpu, mean.  ModelTraining/ModelTesting read cpu (and
mem for the skip test), mean and violations from it (ModelTraining.py:26-32,
ModelTesting.py:46-60).  Here many nodes' records are gathered per epoch
into the [n_streams, n_fields] value array `HTMEngine.step` takes, plus the
per-stream violation/mean/valid arrays `SLOHarness.record` takes.  Kafka
itself stays out of scope: callers feed lines from any transport.
"""
from __future__ import annotations

import json

import numpy as np

AGGREGATE_FIELDS = ("count", "mem", "max", "timestamp", "summation", "violations", "cpu", "mean")
_NULLS = (None, "None", "null", "")


def parse_aggregate(line) -> dict:
    """One aggregate record (JSON text or dict); null metrics become NaN."""
    rec = json.loads(line) if isinstance(line, (str, bytes)) else dict(line)
    out = {}
    for k in AGGREGATE_FIELDS:
        v = rec.get(k)
        out[k] = np.nan if v in _NULLS else float(v)
    return out


class AggregateBatcher:
    """Per-epoch batches of many nodes' aggregate records.

    `nodes` fixes the stream order (stream s = nodes[s]); `fields` the model's
    input fields in the engine's (sorted, MultiEncoder) order -- ("cpu",) for
    Model 1, ("cpu", "mem") for the two-field Model-3 shape.  A node without a
    record for an epoch, or with a null cpu/mem, is invalid for that epoch: its
    values are NaN (the encoder's missing value) and SLO evaluation skips it
    (ModelTraining.py:29-32, ModelTesting.py:51-53)."""

    def __init__(self, nodes, fields=("cpu",)):
        self.nodes = list(nodes)
        self.index = {n: i for i, n in enumerate(self.nodes)}
        self.fields = tuple(sorted(fields))
        self.pending = {}  # timestamp -> {node: record}

    def push(self, node, line):
        rec = parse_aggregate(line)
        if node not in self.index:
            raise KeyError("unknown node %r" % (node,))
        ts = rec["timestamp"]
        if np.isnan(ts):
            raise ValueError("aggregate record without a timestamp")
        self.pending.setdefault(int(ts), {})[node] = rec

    def epochs(self):
        return sorted(self.pending)

    def pop_epoch(self, ts=None) -> dict:
        """The oldest (or given) epoch as arrays: values [n, fields] float64,
        violations int32 [n], means int32 [n] (int(mean), as ModelTesting.py:58
        truncates), valid bool [n], timestamp."""
        if not self.pending:
            raise KeyError("no pending epoch")
        ts = min(self.pending) if ts is None else int(ts)
        recs = self.pending.pop(ts)
        n = len(self.nodes)
        values = np.full((n, len(self.fields)), np.nan)
        viol = np.zeros(n, np.int32)
        mean = np.zeros(n, np.int32)
        valid = np.zeros(n, bool)
        for node, r in recs.items():
            s = self.index[node]
            ok = not (np.isnan(r["cpu"]) or np.isnan(r["mem"]))
            valid[s] = ok
            if ok:
                values[s] = [r[f] for f in self.fields]
            else:
                values[s] = np.nan
            viol[s] = 0 if np.isnan(r["violations"]) else int(r["violations"])
            mean[s] = 0 if np.isnan(r["mean"]) else int(r["mean"])
        return dict(timestamp=ts, values=values, violations=viol, means=mean, valid=valid)
