"""CPU checks of the SDRClassifier restatement (oracle/sdr_classifier_reference.py).

Parity w.r.t. NuPIC is unpinned (NuPIC is not installable here and the
reference holds no classifier fixtures).  What can be pinned is the float64
arithmetic order the restatement claims for numpy, which NuPIC's 'py'
classifier runs on: these tests hold the explicit restatement against numpy
itself.  Behavioural checks follow the expectations of NuPIC's published
sdr_classifier unit tests (a repeated value is predicted with high
probability; the actual-value EMA uses actValueAlpha 0.3)."""
import numpy as np
import pytest

import sdr_classifier_reference as scr


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 15, 16, 17, 127, 128, 129, 255, 256, 257, 479, 480, 1000])
def test_pairwise_sum_is_numpys(n):
    rng = np.random.default_rng(n)
    for _ in range(20):
        a = rng.random(n) * np.exp(rng.normal(size=n) * 4)
        assert scr.numpy_pairwise_sum(a) == np.sum(a)


@pytest.mark.parametrize("nb", [2, 3, 17, 480])
def test_axis0_row_order_is_numpys(nb):
    rng = np.random.default_rng(nb)
    W = rng.normal(size=(500, nb)) * 1e-2
    pnz = np.sort(rng.choice(500, size=120, replace=False))
    act = W[pnz[0]].copy()
    for b in pnz[1:]:
        act = act + W[b]
    assert np.array_equal(act, W[pnz].sum(axis=0))
    p = scr.infer_single_step(pnz, W)
    a2 = W[pnz].sum(axis=0)
    e = np.exp(a2 - a2.max())
    assert np.array_equal(p, e / np.sum(e))


def test_repeated_value_is_predicted():
    c = scr.SDRClassifier(steps=[1], alpha=0.1)
    prev = 0.0
    for rec in range(10):
        r = c.compute(rec, [1, 5, 9], 4, 34.7, True, True)
        if rec >= 2:
            assert int(np.argmax(r[1])) == 4 and r[1][4] > prev
            prev = r[1][4]
    assert prev > 0.5
    assert r["actualValues"][4] == pytest.approx(34.7)


def test_actual_value_ema_and_default():
    c = scr.SDRClassifier(steps=[1], alpha=0.1)
    c.compute(0, [1], 3, 10.0, True, True)
    c.compute(1, [2], 3, 20.0, True, True)
    assert c.actual_values[3] == 0.7 * 10.0 + 0.3 * 20.0
    r = c.compute(2, [3], 0, 5.0, False, True)
    # buckets without a value report actValueList[0]
    assert r["actualValues"][:3] == [5.0, 5.0, 5.0]


def test_multi_step_learning_shapes_and_growth():
    c = scr.SDRClassifier(steps=[1, 2, 3], alpha=0.05)
    rng = np.random.default_rng(0)
    seq = [3, 7, 11, 7]
    for rec in range(60):
        b = seq[rec % 4]
        pnz = sorted(rng.choice(100, size=10, replace=False) + 100 * b)
        c.compute(rec, pnz, b, float(b), True, True)
    assert c.max_bucket == 11 and c.weights[2].shape == (c.max_input + 1, 12)
    assert len(c.history) == 4


def test_region_outputs_and_prediction_results():
    reg = scr.SDRClassifierRegion(steps="1,2", alpha=0.1)
    x = np.zeros(64, np.float32)
    x[[3, 9, 40]] = 1
    for _ in range(20):
        reg.compute(x, 5, 50.0)
    res, conf = scr.prediction_results(reg.actualValues, reg.probabilities, reg.stepsList)
    assert res == [50.0, 50.0] and all(c > 0.5 for c in conf)
    reg.learningMode = False
    reg.compute(x, 5, 50.0)
    assert reg.recordNum == 21
