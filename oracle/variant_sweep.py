"""A/B the oracle's Appendix-A [L]/[M] choices against the only end-to-end
numbers the reference publishes: the 100 threshold blocks of
ML/Data/result_model1.txt (TP/FP/TN/FN of ModelTesting.getModelStats,
ModelTesting.py:148-171, swept over the anomaly threshold of :75-77).

TEST INFRASTRUCTURE (part of the oracle): it replays the reference's Model-1
experiment (ModelTraining.py:21-56 on TrainingData, save before record 2185
per NetworkModel.py:123-127, then ModelTesting.py:36-107 on TestingData with
1+7 steps per record, SP learning on, TM learning off) through the C
restatement under each variant, scores every window with the literal
harness (oracle/slo_reference.py) at every threshold of result_model1.txt and
reports the distance to the reference's counts.

Usage:  python oracle/variant_sweep.py [--jobs 8] [--out oracle/variant_sweep.json]

The reference data files are read from tests/golden/model1_traces.npz (the
inputs) and tests/golden/result_model1_sweep.json (the reference's counts,
extracted by tests/golden/make_traces.py), so the script runs without
/root/reference.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import oracle  # noqa: E402
import slo_reference  # noqa: E402

# variant flags (htm_oracle.h ORC_VAR_*)
V = dict(SP_TIE_LOW=0x001, SP_NO_TIEBREAKER=0x002, SP_INIT_DOUBLE=0x004, SP_POOL_ASCEND=0x008,
         TM_BMC_SEG_GE=0x010, TM_DC_TIERS=0x020, TM_DC_READONLY=0x040, TM_FREE_LATE=0x080,
         TM_BT_LAST_START=0x100)

# name -> (oracle variant flags, harness options)
VARIANTS = {
    "frozen (current restatement)": ([], {}),
    "SP ties -> lower index": (["SP_TIE_LOW"], {}),
    "SP init without tieBreaker draw": (["SP_NO_TIEBREAKER"], {}),
    "SP connected init summed in double": (["SP_INIT_DOUBLE"], {}),
    "SP pool population ascending": (["SP_POOL_ASCEND"], {}),
    "TM best cell: last segment >=": (["TM_BMC_SEG_GE"], {}),
    "TM duty-cycle tier refresh": (["TM_DC_TIERS"], {}),
    "TM phase-2 duty cycle read-only": (["TM_DC_READONLY"], {}),
    "TM freeNSynapses later-first": (["TM_FREE_LATE"], {}),
    "TM backtrack: closest start": (["TM_BT_LAST_START"], {}),
    "SP lower ties + no tieBreaker": (["SP_TIE_LOW", "SP_NO_TIEBREAKER"], {}),
    # harness alternatives (what the off-repo sweep script might have done)
    "harness: TM learning on in test": ([], {"tm_learn_test": True}),
    "harness: TM reset at load": ([], {"reset_at_load": True}),
    "harness: SP learning off in test": ([], {"sp_learn_test": False}),
    "harness: train all 2185 records": ([], {"train_n": 2185}),
    "harness: 2 training epochs": ([], {"epochs": 2}),
    "harness: 4 training epochs": ([], {"epochs": 4}),
    # seed noise: the frozen restatement under other seeds -- how far the sweep
    # moves when only the random draws change (the yardstick for the above)
    "seed 2046": ([], {"seed": 2046}),
    "seed 2047": ([], {"seed": 2047}),
    "seed 2048": ([], {"seed": 2048}),
    "seed 2049": ([], {"seed": 2049}),
    "harness: SP learning off in test, seed 2046": ([], {"sp_learn_test": False, "seed": 2046}),
    "harness: SP learning off in test, seed 2047": ([], {"sp_learn_test": False, "seed": 2047}),
    "harness: SP learning off in test, seed 2048": ([], {"sp_learn_test": False, "seed": 2048}),
    "harness: SP learning off in test, seed 2049": ([], {"sp_learn_test": False, "seed": 2049}),
}


def load_inputs():
    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    train = [float(c) for c, mm in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(mm))]
    with open(os.path.join(ROOT, "tests", "golden", "result_model1_sweep.json")) as f:
        ref = [b for b in json.load(f)["blocks"] if not b["excluded"]]
    return train, d["test_cpu"], d["test_mean"], d["test_violations"], ref


def run_variant(args):
    name, flags, opt = args
    train, test_cpu, _, _, _ = load_inputs()
    var = 0
    for f in flags:
        var |= V[f]
    seeds = {"sp_seed": opt["seed"], "tm_seed": opt["seed"]} if "seed" in opt else {}
    m = oracle.OracleModel(variant=var, **seeds)
    t0 = time.time()
    n_train = opt.get("train_n", 2184)
    for _ in range(opt.get("epochs", 1)):
        for v in train[:n_train]:
            m.step(v, True, True)
    if opt.get("reset_at_load"):
        m.tm_reset()
    sp_l = opt.get("sp_learn_test", True)
    tm_l = opt.get("tm_learn_test", False)
    wins = np.zeros((len(test_cpu), 8), np.float32)
    for r, v in enumerate(test_cpu):
        for j in range(8):
            wins[r, j] = m.step(float(v), sp_l, tm_l)
    sc = m.tm_scalars()
    return name, var, opt, wins, sc["n_segments"], time.time() - t0


def score(wins, means, viol, ref):
    rows = []
    for blk in ref:
        t = blk["threshold"]
        g = slo_reference.evaluate(wins, means, viol, t)[:4]
        rows.append((t, g, (blk["tp"], blk["fp"], blk["tn"], blk["fn"])))
    l1 = np.mean([sum(abs(a - b) for a, b in zip(g, r)) for _, g, r in rows])
    a_mae = np.mean([abs((g[0] + g[1]) - (r[0] + r[1])) for _, g, r in rows])
    return rows, float(l1), float(a_mae)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--out", default=os.path.join(HERE, "variant_sweep.json"))
    ap.add_argument("--only", default=None, help="';'-separated subset of variant names")
    a = ap.parse_args()
    oracle.build()
    train, test_cpu, means, viol, ref = load_inputs()
    names = list(VARIANTS) if not a.only else [n for n in VARIANTS if n in a.only.split(";")]
    work = [(n, VARIANTS[n][0], VARIANTS[n][1]) for n in names]
    out = {"reference": "ML/Data/result_model1.txt", "n_blocks": len(ref), "variants": []}
    with mp.Pool(a.jobs) as pool:
        for name, var, opt, wins, nseg, dt in pool.imap_unordered(run_variant, work):
            rows, l1, a_mae = score(wins, means, viol, ref)
            k = np.rint(wins.astype(np.float64) * 40).astype(int)
            rec = {"name": name, "variant": var, "harness": opt, "segments_after": int(nseg),
                   "mean_l1_per_block": round(l1, 2), "mean_abs_alarm_count_error": round(a_mae, 2),
                   "windows_all_zero": int((k.max(1) == 0).sum()),
                   "sweep": {str(t): list(g) for t, g, _ in rows}, "seconds": round(dt, 1)}
            out["variants"].append(rec)
            print("%-40s L1/block %8.2f  alarmMAE %8.2f  zero-windows %4d  segs %6d  %.0fs"
                  % (name, l1, a_mae, rec["windows_all_zero"], nseg, dt), flush=True)
    out["variants"].sort(key=lambda r: r["mean_l1_per_block"])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
