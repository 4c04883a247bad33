"""Which SLO labelling rule produced the reference's threshold sweep?

TEST INFRASTRUCTURE (analysis of the oracle's pins).  At threshold 1.0 no
window alarms (scores are float32(k/40) <= 1.0, compared with '>'), so the
T = 1.0 block of ML/Data/result_model1.txt (TN 2221 / FN 53, :501-502) depends
on the SLO labels and the prediction-list bookkeeping only -- not on the
model.  The committed harness (ML/HTM/ModelTesting.py: violation = mean >= 70
or violations > 0, :57-60; _MAX_LEAD_TIME 50, :31; processpredictionList
:113-146; getModelStats over predictionList[:-50], :148-171) gives TN 2202 /
FN 72 on the committed TestingData.txt.  This script enumerates simple
variants of the rule -- the response-time threshold and comparison, the field
it reads, the lead window (the tail cut stays 50: the sweep's blocks all total
2,274 = 2,324 - 50), a label shift, labels ignored in a warm-up prefix -- and
keeps those that reproduce TN 2221 / FN 53 exactly.  Each survivor is then
scored on the whole 100-block sweep with the oracle's ModelTesting windows
(tests/golden/model1_golden.npz: the restatement as frozen, seed 2045) and,
when oracle/variant_sweep.json is present, with every variant's windows.

Usage: python oracle/label_rule_search.py [--out oracle/label_rule_search.json]
Reads only tests/golden/ fixtures (no /root/reference at run time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import slo_reference  # noqa: E402

CUT = 50
N_REC = 2324


def t1_counts(labels, lead):
    """(TN, FN) of the all-'N' prediction list (threshold 1.0): item i is FN
    iff a violation falls in [i, i + lead] (ModelTesting.py:113-146)."""
    v = np.nonzero(labels)[0]
    fn = 0
    for i in range(N_REC - CUT):
        j = np.searchsorted(v, i)
        if j < len(v) and v[j] <= i + lead:
            fn += 1
    return N_REC - CUT - fn, fn


def candidate_rules(d):
    mean, viol = d["test_mean"], d["test_violations"]
    mx, cnt = d["test_max"], d["test_count"]
    base = (viol > 0) | (mean >= 70)
    for lead in range(1, 101):
        for m in range(40, 401):
            yield f"mean >= {m}, lead {lead}", (viol > 0) | (mean >= m), lead
            yield f"mean > {m}, lead {lead}", (viol > 0) | (mean > m), lead
        for shift in (-2, -1, 1, 2):
            lab = np.zeros_like(base)
            if shift > 0:
                lab[shift:] = base[:-shift]
            else:
                lab[:shift] = base[-shift:]
            yield f"mean >= 70 shifted {shift:+d}, lead {lead}", lab, lead
        for k in range(1, 40):
            lab = base.copy()
            lab[:k] = False
            yield f"mean >= 70 ignoring records 1..{k}, lead {lead}", lab, lead
    for x in range(500, 10001, 50):
        yield f"max >= {x}, lead 50", (viol > 0) | (mx >= x), 50
    for c in range(50, 501, 5):
        yield f"mean >= 70 and count >= {c}, lead 50", (viol > 0) | ((mean >= 70) & (cnt >= c)), 50


def sweep_l1(wins, d, labels, lead, ref):
    rows = []
    for b in ref:
        g = slo_reference.evaluate(wins, d["test_mean"], d["test_violations"], b["threshold"], max_lead=lead,
                                   cut=CUT, labels=labels)[:4]
        rows.append(sum(abs(a - r) for a, r in zip(g, (b["tp"], b["fp"], b["tn"], b["fn"]))))
    return float(np.mean(rows))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(HERE, "label_rule_search.json"))
    a = ap.parse_args()
    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    with open(os.path.join(ROOT, "tests", "golden", "result_model1_sweep.json")) as f:
        blocks = json.load(f)["blocks"]
    ref = [b for b in blocks if not b["excluded"]]
    t1 = [b for b in blocks if b["threshold"] == 1.0][0]
    want = (t1["tn"], t1["fn"])
    literal = (d["test_violations"] > 0) | (d["test_mean"] >= 70)
    out = {"reference_t1": list(want), "literal_rule_t1": list(t1_counts(literal, 50)), "matches": []}
    seen = set()
    for name, lab, lead in candidate_rules(d):
        key = (lab.tobytes(), lead)
        if key in seen:
            continue
        seen.add(key)
        if t1_counts(lab, lead) == want:
            out["matches"].append({"rule": name, "lead": lead, "labels": [int(i) + 1 for i in np.nonzero(lab)[0]]})
    g = np.load(os.path.join(ROOT, "tests", "golden", "model1_golden.npz"))
    wins = {"oracle as frozen (seed 2045)": g["test_windows"]}
    out["literal_rule_l1"] = {"oracle as frozen (seed 2045)": round(sweep_l1(g["test_windows"], d, literal, 50, ref), 1)}
    for m in out["matches"]:
        lab = np.zeros(N_REC, bool)
        lab[np.array(m["labels"]) - 1] = True
        m["sweep_l1_per_block"] = {k: round(sweep_l1(w, d, lab, m["lead"], ref), 1) for k, w in wins.items()}
    out["matches"].sort(key=lambda m: m["sweep_l1_per_block"]["oracle as frozen (seed 2045)"])
    print("literal rule at T=1.0: TN %d FN %d (reference TN %d FN %d); sweep L1/block %.1f"
          % (*out["literal_rule_t1"], *want, out["literal_rule_l1"]["oracle as frozen (seed 2045)"]))
    print("%d simple rules reproduce the T=1.0 block exactly:" % len(out["matches"]))
    for m in out["matches"][:40]:
        print("  %-55s labels %-40s L1/block %s" % (m["rule"], m["labels"][:6] + (["..."] if len(m["labels"]) > 6 else []),
                                                     m["sweep_l1_per_block"]))
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
