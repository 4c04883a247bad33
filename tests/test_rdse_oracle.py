"""CPU checks of the model.yaml-shape additions to the oracle (no GPU).

* The C oracle's RandomDistributedScalarEncoder (oracle/htm_oracle.c rdse_*)
  against the independent pure-Python restatement kept in NuPIC's own shape
  (oracle/rdse_reference.py): bucket indices and bit sets on sequences that
  grow the map in both directions, jump, clip at both ends, hit Python 2's
  half-away-from-zero rounding, and start with a missing value.
* NuPIC's RDSE invariants on the grown map: neighbours at distance d < w share
  exactly w - d bits, all others at most 2 (_overlapOK).
* The boost factor's exp (exp_det) is the correctly rounded exp on the range
  updateBoostFactorsGlobal_ sees.
Parity w.r.t. NuPIC is unpinned (NuPIC is absent).
"""
import math

import numpy as np
import pytest

import rdse_reference as ref


def test_python_random_matches_the_c_oracle(oracle_mod):
    for seed in (1, 42, 1956, 2045):
        r = ref.NupicRandom(seed)
        assert [r._raw() for _ in range(500)] == oracle_mod.rng_stream(seed, 500).tolist()


SEQS = {
    "walk": [50, 52, 55, 49, 47, 60, 61, 30, 31, 90, 10, 0, 100, 50.4, 50.5],
    "nan_first": [float("nan"), 20.0, 21.0, float("nan"), 19.0, 80.0],
    "halves": [10.0, 11.32, 9.12, 12.2, 8.24, 10.44],  # (x - 10) / 0.88 = +-1.5, +-2.5, 0.5
    "clip": [0.0, 100.0, 0.0, 55.0],
}


@pytest.mark.parametrize("name", sorted(SEQS))
@pytest.mark.parametrize("res,seed", [(0.88, 1), (1.0, 42), (0.1, 7)])
def test_c_oracle_rdse_equals_python_restatement(oracle_mod, name, res, seed):
    p = oracle_mod.model_yaml_params(rdse_resolution=res, rdse_seed=seed)
    m = oracle_mod.OracleModel(p)
    py = ref.RDSE(res, w=21, n=400, seed=seed)
    for x in SEQS[name]:
        bits = m.encode([x])
        pb, pidx = py.encode(x)
        assert m.bucket() == (-1 if pidx is None else pidx), x
        assert bits.tolist() == pb, x
    st = m.rdse_state()
    assert (st["min_idx"], st["max_idx"], st["num_tries"]) == (py.minIndex, py.maxIndex, py.numTries)
    for i in range(py.minIndex, py.maxIndex + 1):
        assert st["map"][i].tolist() == py.bucketMap[i]


def test_rdse_overlap_invariants(oracle_mod):
    m = oracle_mod.OracleModel(oracle_mod.model_yaml_params())
    for x in np.linspace(0, 100, 41):
        m.encode([float(x)])
    st = m.rdse_state()
    lo, hi, w = st["min_idx"], st["max_idx"], 21
    assert hi - lo >= 100
    sets = {i: set(st["map"][i].tolist()) for i in range(lo, hi + 1)}
    for i in range(lo, hi + 1):
        assert len(sets[i]) == w
        for j in range(i + 1, hi + 1):
            ov = len(sets[i] & sets[j])
            assert ov == w - (j - i) if j - i < w else ov <= 2, (i, j, ov)


def test_exp_det_is_correctly_rounded(oracle_mod):
    xs = np.float32(np.linspace(-3.5, 0.5, 20001))
    for x in xs:
        assert oracle_mod.exp_det(x) == np.float32(math.exp(float(x))), x
    assert oracle_mod.exp_det(0.0) == 1.0


def test_boosting_changes_the_winners(oracle_mod):
    """boostStrength 3 (model.yaml:41) vs 0 on the same stream: the boost
    factors move away from 1 after learning steps and change the SP output."""
    p3 = oracle_mod.model_yaml_params()
    p0 = oracle_mod.model_yaml_params(sp_boost_strength=0.0)
    a, b = oracle_mod.OracleModel(p3), oracle_mod.OracleModel(p0)
    rng = np.random.default_rng(3)
    differ = 0
    for _ in range(120):
        v = [float(rng.integers(0, 101))]
        a.step(v, True, False)
        b.step(v, True, False)
        differ += not np.array_equal(a.active_columns(), b.active_columns())
    sa = a.sp_state()
    assert np.all(sa["boost"] > 0) and np.any(sa["boost"] != 1.0)
    target = np.float32(40 / 2048)
    want = np.array([oracle_mod.exp_det(np.float32((target - d) * np.float32(3.0))) for d in sa["active_dc"]])
    assert np.array_equal(sa["boost"], want)
    assert differ > 0
