"""Aggregate-record ingestion (StreamAggregator.py:101-115 format) into
batched engine / SLO inputs -- host logic, no GPU."""
import json

import numpy as np
import pytest


def rec(ts, cpu, mem=16, mean=120, violations=0):
    return json.dumps({"count": 77, "mem": mem, "max": 4708, "timestamp": ts, "summation": 31570,
                       "violations": violations, "cpu": cpu, "mean": mean})


def test_parse_nulls_become_nan(rt):
    r = rt.ingest.parse_aggregate('{"count": 1, "mem": null, "max": 3, "timestamp": 5, "summation": 2, '
                                  '"violations": 0, "cpu": "None", "mean": 70}')
    assert np.isnan(r["cpu"]) and np.isnan(r["mem"]) and r["mean"] == 70.0


def test_batcher_orders_nodes_and_epochs(rt):
    b = rt.ingest.AggregateBatcher(["web1", "db1", "web2"], fields=("mem", "cpu"))
    assert b.fields == ("cpu", "mem")  # MultiEncoder order
    b.push("db1", rec(101, 40, mean=71))
    b.push("web1", rec(100, 22))
    b.push("web2", rec(100, 14, violations=2))
    b.push("web1", rec(101, None))
    assert b.epochs() == [100, 101]
    e = b.pop_epoch()
    assert e["timestamp"] == 100
    assert e["values"][0].tolist() == [22.0, 16.0] and np.isnan(e["values"][1]).all()
    assert e["valid"].tolist() == [True, False, True] and e["violations"].tolist() == [0, 0, 2]
    e = b.pop_epoch()
    assert e["valid"].tolist() == [False, True, False] and e["means"][1] == 71
    with pytest.raises(KeyError):
        b.push("nope", rec(1, 1))
