"""The batched SLO-prediction harness (csrc/slo.hip) against the literal
restatement of ModelTesting.py (oracle/slo_reference.py), and the batched
ModelTraining/ModelTesting drivers against the golden Model-1 replay."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)


def ref_stats(windows, means, violations, th):
    """(TP, FP, TN, FN, avg lead) as getModelStats prints them."""
    import slo_reference
    return tuple(slo_reference.evaluate(windows, means, violations, th))


def gpu_stats(row):
    """the kernel's (TP, FP, TN, FN, lead sum) -> getModelStats' form (leadTime / tp
    in double, like the reference's float accumulation of integer leads)"""
    tp, fp, tn, fn, lead = (int(x) for x in row)
    return tp, fp, tn, fn, (float(lead) / tp if tp else None)


def synthetic(n_streams, n_rec, seed):
    """score windows quantised like the engine's (k/40), violation runs of
    every length (incl. > 64 records, exercising the ring's pending path)."""
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 41, size=(n_rec, 8, n_streams))
    k = np.where(rng.random(k.shape) < 0.7, np.minimum(k, 30), k)
    w = (k / 40.0).astype(np.float32)
    viol = np.zeros((n_rec, n_streams), np.int32)
    mean = rng.integers(10, 69, size=(n_rec, n_streams)).astype(np.int32)
    for s in range(n_streams):
        t = 0
        while t < n_rec:
            t += int(rng.integers(5, 200))
            run = int(rng.choice([1, 3, 20, 55, 70, 130]))
            if s % 2:
                viol[t:t + run, s] = 1
            else:
                mean[t:t + run, s] = 70 + rng.integers(0, 30)
            t += run
    return w, viol, mean


@pytest.mark.parametrize("th", [0.85, 0.98, 0.35, 0.1])
def test_slo_kernel_matches_reference(rt, th):
    n, n_rec = 24, 700
    w, viol, mean = synthetic(n, n_rec, seed=int(th * 100))
    slo = rt.SLOHarness(n, threshold=th)
    dw = torch.tensor(w, device="cuda")
    dv = torch.tensor(viol, device="cuda")
    dm = torch.tensor(mean, device="cuda")
    for r in range(n_rec):
        slo.record(dw[r], dv[r], dm[r])
    got = slo.stats()
    for s in range(n):
        want = ref_stats([w[r, :, s] for r in range(n_rec)], mean[:, s], viol[:, s], th)
        assert gpu_stats(got[s]) == want, (s, tuple(got[s]), want)


def test_slo_skipped_records(rt):
    n, n_rec = 8, 300
    w, viol, mean = synthetic(n, n_rec, seed=3)
    rng = np.random.default_rng(4)
    valid = rng.random((n_rec, n)) > 0.1
    slo = rt.SLOHarness(n, threshold=0.85)
    for r in range(n_rec):
        slo.record(torch.tensor(w[r], device="cuda"), viol[r], mean[r], valid=valid[r])
    got = slo.stats()
    for s in range(n):
        keep = np.nonzero(valid[:, s])[0]
        want = ref_stats([w[r, :, s] for r in keep], mean[keep, s], viol[keep, s], 0.85)
        assert gpu_stats(got[s]) == want


def test_model1_experiment_through_the_batched_drivers(rt, traces, tmp_path):
    """ModelTraining then ModelTesting for 3 replicated
    streams: the saved network has seen 2184 records, the test windows equal
    the golden replay, and the SLO counts equal the literal harness's."""
    g = np.load(os.path.join(GOLDEN, "model1_golden.npz"))
    raw = traces["raw"]
    ok = rt.harness.valid_records(raw["train_cpu"], raw["train_mem"])
    n = 3
    eng = rt.HTMEngine(n, seg_capacity=72 * 1024)
    p = str(tmp_path / "network1.htm")
    sc = rt.harness.model_training(eng, np.repeat(raw["train_cpu"][ok][:, None], n, axis=1), save_path=p)
    assert np.array_equal(sc[:2184, 0].cpu().numpy(), g["train_scores"])
    saved = rt.HTMEngine.load(p)
    windows, stats = rt.harness.model_testing(saved, traces["test"], traces["test_violations"],
                                              traces["test_mean"], threshold=0.85)
    assert np.array_equal(windows[:, :, 0], g["test_windows"])
    assert np.array_equal(windows[:, :, 2], g["test_windows"])
    want = ref_stats(list(g["test_windows"]), traces["test_mean"], traces["test_violations"], 0.85)
    for s in range(n):
        assert gpu_stats(stats[s]) == want
