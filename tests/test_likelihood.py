"""AnomalyLikelihood kernel (csrc/likelihood.hip) against the CPU restatement
of NuPIC's algorithm (oracle/likelihood_reference.py).  Parity w.r.t. NuPIC is
unpinned (the reference never computes a likelihood); the tolerance is the
north star's 1e-6 relative."""
import numpy as np
import pytest

import likelihood_reference as lr

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)


def series(n_streams, T, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 41, size=(T, n_streams))
    k = np.where(rng.random(k.shape) < 0.8, np.minimum(k, 4), k)  # mostly-predicted streams
    scores = (k / 40.0).astype(np.float32)
    values = rng.integers(0, 101, size=(T, n_streams)).astype(np.float64)
    values[:, 0] = 42.0  # a constant metric: the null distribution
    spikes = rng.random((T, n_streams)) < 0.01
    scores[spikes] = 1.0
    return values, scores


@pytest.mark.parametrize("params", [dict(learning_period=288, estimation_samples=100, historic_window=8640,
                                         reestimation_period=100),
                                    dict(learning_period=30, estimation_samples=20, historic_window=120,
                                         reestimation_period=25)])
def test_likelihood_matches_restatement(rt, params):
    n = 6
    T = 1200 if params["historic_window"] == 8640 else 700
    values, scores = series(n, T, seed=params["historic_window"])
    lk = rt.AnomalyLikelihood(n, **params)
    dv, ds = torch.tensor(values, device="cuda"), torch.tensor(scores, device="cuda")
    got = np.stack([lk.anomaly_probability(dv[t], ds[t]).cpu().numpy() for t in range(T)])
    refs = [lr.AnomalyLikelihood(params["learning_period"], params["estimation_samples"], params["historic_window"],
                                 params["reestimation_period"]) for _ in range(n)]
    want = np.array([[refs[s].anomaly_probability(values[t, s], float(scores[t, s])) for s in range(n)]
                     for t in range(T)])
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=0)
    assert np.all(got[: params["learning_period"] + params["estimation_samples"]] == 0.5)
