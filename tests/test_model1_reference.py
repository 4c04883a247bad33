"""Statistical comparison of the oracle's Model-1 replay with the only
end-to-end numbers the reference publishes (ML/Data/result_model1.txt).

The reference's sweep came from an off-repo script and a NuPIC build that
the as-written code cannot reproduce, so exact counts
are not expected: this is a sanity band, documented as such.  What IS pinned
exactly: every score is float32(k/40) with 40 active columns
and the harness arithmetic (float32 score vs double threshold).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

# (threshold, TP, FP, TN, FN) from ML/Data/result_model1.txt:206-209 (0.5),
# :426-429 (0.85), :451-454 (0.9)
REFERENCE = [(0.5, 16, 465, 1785, 8), (0.85, 10, 161, 2094, 9), (0.9, 4, 108, 2139, 23)]


def sweep_blocks():
    """The reference's 101 threshold blocks (tests/golden/result_model1_sweep.json,
    extracted from ML/Data/result_model1.txt by tests/golden/make_traces.py)."""
    with open(os.path.join(GOLDEN, "result_model1_sweep.json")) as f:
        return json.load(f)["blocks"]


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "model1_golden.npz"))


def test_scores_are_float32_k_over_40(golden):
    w = golden["test_windows"].ravel()
    k = np.round(w.astype(np.float64) * 40)
    assert np.array_equal(w, (k / 40.0).astype(np.float32))
    t = golden["train_scores"]
    assert np.array_equal(t, (np.round(t.astype(np.float64) * 40) / 40.0).astype(np.float32))


def test_float32_threshold_comparison_semantics():
    # float32(0.35) < 0.35 and float32(0.1) > 0.1: the sweep boundaries in
    # result_model1.txt move exactly there
    assert not (float(np.float32(14 / 40)) > 0.35)
    assert float(np.float32(4 / 40)) > 0.1


def test_sweep_in_reference_band(golden, traces):
    import slo_reference
    w = golden["test_windows"]
    total = len(w) - 50
    for th, tp, fp, tn, fn in REFERENCE:
        g = slo_reference.evaluate(w, traces["test_mean"], traces["test_violations"], th)
        assert sum(g[:4]) == total == tp + fp + tn + fn  # 2274 records scored, like the reference
        # same regime: false positives within 40 % of the reference, accuracy within 5 points
        assert abs(g[1] - fp) <= 0.4 * fp, (th, g, (tp, fp, tn, fn))
        acc_g = (g[0] + g[2]) / total
        acc_r = (tp + tn) / total
        assert abs(acc_g - acc_r) < 0.05, (th, acc_g, acc_r)


def test_train_fixture_prefix_reproduces(oracle_mod, golden, traces):
    m = oracle_mod.OracleModel()
    for k in range(120):
        s = m.step(traces["train"][k], True, True)
        assert s == golden["train_scores"][k]
        if k < 300:
            assert np.array_equal(m.active_columns(), golden["train_active"][k])


def test_reference_sweep_moves_only_at_float32_k_over_40():
    """SURVEY.md §0.4 on the reference's own data: wherever the reference's
    counts change between adjacent thresholds a < b, a score float32(k/40)
    lies in (a, b] (the harness alarms on score > T, ModelTesting.py:76).
    Float64 k/40 scores would put no score in 11 of those intervals."""
    blocks = [b for b in sweep_blocks() if not b["excluded"]]
    f32 = [float(np.float32(k / 40.0)) for k in range(41)]
    f64 = [k / 40.0 for k in range(41)]
    changes, miss64 = 0, 0
    for a, b in zip(blocks, blocks[1:]):
        ca = (a["tp"], a["fp"], a["tn"], a["fn"])
        cb = (b["tp"], b["fp"], b["tn"], b["fn"])
        if ca == cb:
            continue
        changes += 1
        lo, hi = a["threshold"], b["threshold"]
        assert any(lo < s <= hi for s in f32), (lo, hi)
        miss64 += not any(lo < s <= hi for s in f64)
    assert changes >= 30 and miss64 >= 10


# The documented band of the full curve (oracle/variant_sweep.json):
# the off-repo sweep is not reproducible exactly (unknown NuPIC build and random
# draws; the seed ensemble alone moves the curve by this much or more), so the
# test pins the regime and the known gap, on every one of the 100 blocks.
BAND_SPLIT = 0.45      # operating range: the code's 0.85 and the README's 0.98 / 0.99
BAND_HI_REL = 0.30     # T >= 0.45: |alarms - ref| <= 0.30 ref + 15
BAND_HI_ABS = 15
BAND_HI_TP = 8         # T >= 0.45: |TP - ref TP| <= 8
BAND_LO_RATIO = 2.0    # T < 0.45: ref <= alarms <= 2.0 ref (the restatement predicts
                       # fewer windows perfectly: 112 all-zero windows vs the reference's 725)


def test_full_sweep_in_documented_band(golden, traces):
    import slo_reference
    w = golden["test_windows"]
    for b in sweep_blocks():
        if b["excluded"]:
            continue  # the 0.0 block is all-alarm, unreachable with '>' 
        t = b["threshold"]
        tp, fp, tn, fn, _ = slo_reference.evaluate(w, traces["test_mean"], traces["test_violations"], t)
        assert tp + fp + tn + fn == 2274
        alarms, ref_alarms = tp + fp, b["tp"] + b["fp"]
        if t >= BAND_SPLIT:
            assert abs(alarms - ref_alarms) <= BAND_HI_REL * ref_alarms + BAND_HI_ABS, (t, alarms, ref_alarms)
            assert abs(tp - b["tp"]) <= BAND_HI_TP, (t, tp, b["tp"])
        else:
            assert ref_alarms <= alarms <= BAND_LO_RATIO * ref_alarms, (t, alarms, ref_alarms)


def test_slo_labels_differ_from_the_reference_sweep(traces):
    """Model-independent pin: at threshold 1.0 nothing alarms, so TN/FN depend
    only on the SLO labels.  ModelTesting.py's rule (mean >= 70 or violations
    > 0, :57-60) on the committed TestingData.txt labels 72 records as
    within-lead-time positives (15 violating records: rows 0-16 and
    1579-1583); the reference's sweep reports 53 (TN 2221 / FN 53,
    result_model1.txt:501-502).  Its sweep did not label the committed data the
    way the committed harness does -- the TP/FN part of the gap is not the model's."""
    import slo_reference
    w0 = np.zeros((len(traces["test_mean"]), 8), np.float32)
    assert slo_reference.evaluate(w0, traces["test_mean"], traces["test_violations"], 1.0)[:4] == (0, 0, 2202, 72)
    last = [b for b in sweep_blocks() if b["threshold"] == 1.0][0]
    assert (last["tn"], last["fn"]) == (2221, 53)


RECOVERED_RULES = [  # oracle/label_rule_search.py: simple rules that give TN 2221 / FN 53 at T = 1.0
    ("mean >= 70 and count >= 340, lead 50", lambda t: (t["test_violations"] > 0) |
     ((t["test_mean"] >= 70) & (t["raw"]["test_count"] >= 340)), 50),
    ("mean >= 70 ignoring records 1..17, lead 48", lambda t: ((t["test_violations"] > 0) | (t["test_mean"] >= 70)) &
     (np.arange(len(t["test_mean"])) >= 17), 48),
    ("mean >= 70, lead 31", lambda t: (t["test_violations"] > 0) | (t["test_mean"] >= 70), 31),
]


@pytest.mark.parametrize("name,rule,lead", RECOVERED_RULES, ids=[r[0] for r in RECOVERED_RULES])
def test_recovered_label_rules_reproduce_the_t1_block(traces, name, rule, lead):
    """The labelling search (oracle/label_rule_search.py, oracle/label_rule_search.json)
    finds 35 one-parameter variants of ModelTesting.py:57-60 / :113-146 that
    reproduce the model-independent T = 1.0 block exactly (result_model1.txt:501-502);
    three of them, re-checked here.  The block alone cannot choose between them."""
    import slo_reference
    w0 = np.zeros((len(traces["test_mean"]), 8), np.float32)
    lab = rule(traces)
    got = slo_reference.evaluate(w0, traces["test_mean"], traces["test_violations"], 1.0, max_lead=lead, cut=50,
                                 labels=lab)[:4]
    assert got == (0, 0, 2221, 53)


def test_no_recovered_label_rule_explains_the_gap():
    """Scored with the oracle's ModelTesting windows on all 100 blocks, every
    rule that fits T = 1.0 lands within 3 % of the literal rule's distance to
    the reference (354.6 L1/block): the labels are not where the restatement
    and the off-repo sweep differ; the all-zero windows are (oracle 112 vs the
    reference's 725)."""
    import json
    d = json.load(open(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "label_rule_search.json")))
    base = d["literal_rule_l1"]["oracle as frozen (seed 2045)"]
    assert d["reference_t1"] == [2221, 53] and d["literal_rule_t1"] == [2202, 72]
    assert len(d["matches"]) >= 3
    for m in d["matches"]:
        l1 = m["sweep_l1_per_block"]["oracle as frozen (seed 2045)"]
        assert abs(l1 - base) <= 0.03 * base, (m["rule"], l1, base)

