"""GPU parity of north_star's 32-cell target shape: the reference's model.yaml.

ML/HTM/params/model.yaml (unused by the reference's scripts, the parameter
set north_star's "2048-column/32-cell" target is quoted on): the
RandomDistributedScalarEncoder (:15-21, resolution 0.88, seed 1), the SP with
boostStrength 3.0, potentialPct 0.85, inc 0.04, dec 0.005, seed 1956
(:28-41) and a 32-cell BacktrackingTM, activationThreshold 16, minThreshold
12, pamLength 1, seed 1960 (:45-63).  The HIP engine is held bit-exact to the
oracle (oracle/htm_oracle.c, its RDSE cross-checked by the pure-Python
restatement in tests/test_rdse_oracle.py) through learning (boosted
inhibition, RDSE bucket growth), the frozen test phase in lockstep (deferred
duty writes) and fleet mode.  Parity w.r.t. NuPIC is unpinned (NuPIC absent,
SURVEY.md §8(c)).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from test_gpu_parity import sp_equal, tm_equal  # noqa: E402


def yaml_engine(rt, n, **kw):
    kw.setdefault("seg_capacity", 1 << 15)
    return rt.HTMEngine(n, config=rt._lib.model_yaml_config(**kw))


def streams(traces, n, T, seed=11):
    rng = np.random.default_rng(seed)
    tr = np.asarray(traces["train"], np.float64)
    idx = (np.arange(T)[:, None] + 173 * np.arange(n)[None, :]) % len(tr)
    v = np.clip(tr[idx] + rng.integers(-3, 4, size=idx.shape), 0, 100)
    v[rng.random(v.shape) < 0.01] = np.nan  # missing records: empty SDR, offset untouched
    return v


def check_rdse(eng, s, orc):
    a, b = eng.rdse_state(s), orc.rdse_state()
    for k in ("min_idx", "max_idx", "has_offset", "num_tries", "offset"):
        assert a[k] == b[k], k
    assert np.array_equal(a["map"], b["map"])


def test_model_yaml_learning_then_frozen_vs_oracle(rt, oracle_mod, traces):
    """Two streams (different inputs, seed_stride 0 as the yaml) learn 320
    records with SP+TM learning on -- boosted inhibition, RDSE map growth --
    then 96 records with TM learning off and SP learning on (ModelTesting's
    test phase) stepped in lockstep with the deferred duty writes: scores,
    active columns and encoder buckets every step; SP (boost factors
    included), TM and RDSE state at the end."""
    n, T1, T2 = 2, 320, 96
    vals = streams(traces, n, T1 + T2)
    eng = yaml_engine(rt, n)
    orcs = [oracle_mod.OracleModel(oracle_mod.model_yaml_params()) for _ in range(n)]
    for k in range(T1 + T2):
        tm_learn = k < T1
        if k in (0, T1):
            eng.set_learning(True, tm_learn)
        g = eng.step(torch.tensor(vals[k], device="cuda")).cpu().numpy()
        act = eng.get_output("active_columns").cpu().numpy()
        bk = eng.get_output("buckets").cpu().numpy()
        for s in range(n):
            o = orcs[s].step([vals[k, s]], True, tm_learn)
            assert g[s] == o, f"step {k} stream {s}: gpu {g[s]} oracle {o}"
            ao = np.zeros(eng.n_columns, np.uint8)
            ao[orcs[s].active_columns()] = 1
            assert np.array_equal(act[s], ao), f"active columns, step {k} stream {s}"
            assert bk[s, 0] == orcs[s].bucket(), f"bucket, step {k} stream {s}"
    eng.status()
    for s in range(n):
        sp_equal(eng, s, orcs[s])
        assert np.array_equal(eng.sp_state(s)["boost"], orcs[s].sp_state()["boost"])
        tm_equal(eng, s, orcs[s])
        check_rdse(eng, s, orcs[s])
    assert np.any(eng.sp_state(0)["boost"] != 1.0)  # boosting is live
    eng.close()


def test_model_yaml_fleet_131072_streams_vs_oracle(rt, oracle_mod, traces):
    """Fleet mode at north_star's per-GPU share of its 1M-stream target
    (131,072 streams sharing one frozen model.yaml model, 32 cells per column,
    each stream with its own TM state and RDSE encoder): 6 sampled streams
    against oracle clones of the trained model over 48 lockstep steps."""
    train = streams(traces, 1, 400, seed=3)[:, 0]
    model = yaml_engine(rt, 1)
    model.run(torch.tensor(train, device="cuda").reshape(-1, 1))
    model.status()
    orc = oracle_mod.OracleModel(oracle_mod.model_yaml_params())
    for v in train:
        orc.step([v], True, True)
    n, T = 131072, 48
    fleet = rt.HTMEngine.fleet(model, n, q_capacity=4096)
    rng = np.random.default_rng(9)
    test = np.asarray(traces["test"], np.float64)
    sample = [0, 1, 4097, 65536, 99999, n - 1]
    orcs = {s: orc.clone() for s in sample}
    got = np.zeros((T, len(sample)), np.float32)
    for k in range(T):
        v = np.clip(test[(k + 7 * np.arange(n)) % len(test)] + rng.integers(-2, 3, size=n), 0, 100)
        g = fleet.step(torch.tensor(v, device="cuda")).cpu().numpy()
        for j, s in enumerate(sample):
            got[k, j] = g[s]
            assert g[s] == orcs[s].step([v[s]], False, False), f"step {k} stream {s}"
    fleet.status()
    # (the shared segment records hold every stream's dutyCycle() writes: the
    # per-stream state is what a clone must match)
    for s in (sample[0], sample[-1]):
        a, b = fleet.tm_states(s), orcs[s].tm_states()
        for k in a:
            assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(fleet.col_confidence(s), orcs[s].col_confidence())
        check_rdse(fleet, s, orcs[s])
    fleet.close()
    model.close()
