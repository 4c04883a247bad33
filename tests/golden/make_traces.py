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


def load(path):
    rows = [json.loads(line) for line in open(path)]

    def f(v):
        return np.nan if v in (None, "None", "null") else float(v)

    return (np.array([f(r["cpu"]) for r in rows]), np.array([f(r["mem"]) for r in rows]),
            np.array([int(r["mean"]) for r in rows]), np.array([int(r["violations"]) for r in rows]))


def main():
    if not os.path.isdir(REF):
        sys.exit("reference data not present")
    tr = load(os.path.join(REF, "TrainingData.txt"))
    te = load(os.path.join(REF, "TestingData.txt"))
    np.savez_compressed(OUT, train_cpu=tr[0], train_mem=tr[1], train_mean=tr[2], train_violations=tr[3],
                        test_cpu=te[0], test_mem=te[1], test_mean=te[2], test_violations=te[3])
    print("wrote", OUT, len(tr[0]), len(te[0]))


if __name__ == "__main__":
    main()
