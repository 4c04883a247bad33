"""Extract the reference's input traces into tests/golden/model1_traces.npz.

Source: /root/reference/ML/Data/TrainingData.txt and TestingData.txt (JSON
lines written by StreamEngine/StreamAggregator.py:101-115).  Only the fields
the Model-1 path reads are kept (ModelTraining.py:26-32, ModelTesting.py:46-60):
cpu, mem, mean, violations.  A null cpu/mem becomes NaN (the record is then
skipped by the harness, as the reference does).  Run once here; the .npz is
committed so the GPU box (no /root/reference) has the data.
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference/ML/Data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "model1_traces.npz")
SWEEP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "result_model1_sweep.json")


def load(path):
    rows = [json.loads(line) for line in open(path)]

    def f(v):
        return np.nan if v in (None, "None", "null") else float(v)

    return (np.array([f(r["cpu"]) for r in rows]), np.array([f(r["mem"]) for r in rows]),
            np.array([int(r["mean"]) for r in rows]), np.array([int(r["violations"]) for r in rows]),
            np.array([int(r["max"]) for r in rows]), np.array([int(r["count"]) for r in rows]))


def main():
    if not os.path.isdir(REF):
        sys.exit("reference data not present")
    tr = load(os.path.join(REF, "TrainingData.txt"))
    te = load(os.path.join(REF, "TestingData.txt"))
    np.savez_compressed(OUT, train_cpu=tr[0], train_mem=tr[1], train_mean=tr[2], train_violations=tr[3],
                        train_max=tr[4], train_count=tr[5],
                        test_cpu=te[0], test_mem=te[1], test_mean=te[2], test_violations=te[3],
                        test_max=te[4], test_count=te[5])
    print("wrote", OUT, len(tr[0]), len(te[0]))
    write_sweep()


def write_sweep():
    """The reference's published threshold sweep (ML/Data/result_model1.txt,
    101 blocks 'T / TP: a FP: b TN: c FN: d / Avg leadtime / Model accuracy')
    as data.  The 0.0 block is all-alarm (TP 53 FP 2221), which the harness's
    strict '>' cannot produce once any window is all-zero, so it
    is flagged and left out of distances."""
    import re
    txt = open(os.path.join(REF, "result_model1.txt")).read()
    blocks = re.findall(r"^([01](?:\.\d+)?)\nTP: (\d+) FP: (\d+) TN: (\d+) FN: (\d+)\nAvg leadtime ([\d.]+)", txt, re.M)
    out = []
    for t, tp, fp, tn, fn, lead in blocks:
        out.append(dict(threshold=float(t), tp=int(tp), fp=int(fp), tn=int(tn), fn=int(fn),
                        avg_lead=float(lead), excluded=float(t) == 0.0))
    assert len(out) == 101, len(out)
    with open(SWEEP, "w") as f:
        json.dump({"source": "ML/Data/result_model1.txt", "blocks": out}, f, indent=0)
    print("wrote", SWEEP, len(out))


if __name__ == "__main__":
    main()
