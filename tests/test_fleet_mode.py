"""Fleet mode (config 4): streams sharing one frozen SP+TM model give exactly
the results of an ordinary engine holding a copy of the model per stream."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)


@pytest.fixture(scope="module")
def model(rt, traces):
    eng = rt.HTMEngine(1, seg_capacity=1 << 15)
    eng.run(torch.tensor(traces["train"][:500], dtype=torch.float64, device="cuda").reshape(-1, 1))
    eng.status()
    return eng


def replicas(rt, model, n):
    eng = rt.HTMEngine(n, seg_capacity=1 << 15)
    for region in rt._lib.ST:
        eng.import_state(region, model.export_state(region, 0, 1), s0=0)
    eng.replicate(0)
    eng.set_learning(False, False)
    return eng


@pytest.mark.parametrize("pid_lists", [True, False])
def test_fleet_equals_replicated_engines(rt, model, traces, pid_lists, monkeypatch):
    """pid_lists False: the frozen index without pid lists (HTM_FX_PID=0, read
    at engine creation), phase 2 reading the qualifying segments' synapse rows."""
    n, T = 16, 120
    if not pid_lists:
        monkeypatch.setenv("HTM_FX_PID", "0")
    rep = replicas(rt, model, n)
    fl = rt.HTMEngine.fleet(model, n, q_capacity=4096)
    monkeypatch.delenv("HTM_FX_PID", raising=False)
    assert fl.is_fleet and fl.device_bytes() < rep.device_bytes() / 4
    rng = np.random.default_rng(17)
    base = np.asarray(traces["test"][:T], np.float64)
    vals = np.clip(base[:, None] + rng.integers(-3, 4, size=(T, n)), 0, 100)
    vals[rng.random(vals.shape) < 0.02] = np.nan
    v = torch.tensor(vals, device="cuda")
    a = rep.run(v).cpu().numpy()
    b = fl.run(v[:60]).cpu().numpy()
    b = np.concatenate([b, np.stack([fl.step(v[k]).cpu().numpy() for k in range(60, T)])])
    assert np.array_equal(a, b)
    for s in [0, n - 1]:
        sa, sb = rep.tm_states(s), fl.tm_states(s)
        for k in sa:
            assert np.array_equal(sa[k], sb[k])
        assert np.array_equal(rep.col_confidence(s), fl.col_confidence(s))
    # the shared model is read-only except for the segments' dutyCycle cache:
    # at the frozen iteration, Segment::dutyCycle() stores the value it
    # returns, so the fleet's cache holds the updates of every stream and
    # stream 0's replica only its own -- entries differ only where the
    # fleet's was refreshed at the frozen iteration (outputs are unaffected)
    ga, gb = rep.tm_segments(0), fl.tm_segments(0)
    for k in ["cell", "nsyn", "src", "perm", "pos_act"]:
        assert np.array_equal(ga[k], gb[k])
    it = fl.tm_header(0).lrn_iter
    diff = (ga["last_dc"] != gb["last_dc"]) | (ga["last_dc_iter"] != gb["last_dc_iter"])
    assert np.all(gb["last_dc_iter"][diff] == it)
    fl.status()


def test_fleet_refuses_learning(rt, model):
    fl = rt.HTMEngine.fleet(model, 4)
    with pytest.raises(rt.HtmError):
        fl.set_learning(True, False)
    with pytest.raises(rt.HtmError):  # the pool scan would race on the shared segment records
        fl.use_frozen_index(False)


def test_fleet_save_load_round_trip(rt, model, traces, tmp_path):
    """A fleet saved mid-run (htm_save: the shared model once, every stream's
    state) loads back as a fleet and continues exactly like the unsaved one;
    the file holds one model, not one per stream."""
    n, T = 64, 80
    rng = np.random.default_rng(23)
    base = np.asarray(traces["test"][:T], np.float64)
    v = torch.tensor(np.clip(base[:, None] + rng.integers(-3, 4, size=(T, n)), 0, 100), device="cuda")
    fl = rt.HTMEngine.fleet(model, n, q_capacity=4096)
    for k in range(40):
        fl.step(v[k])
    path = str(tmp_path / "fleet.htm")
    fl.save(path)
    re = rt.HTMEngine.load(path)
    assert re.is_fleet and re.n_streams == n and not re.sp_learn and not re.tm_learn
    a = np.stack([fl.step(v[k]).cpu().numpy() for k in range(40, T)])
    b = np.stack([re.step(v[k]).cpu().numpy() for k in range(40, T)])
    assert np.array_equal(a, b)
    for s in (0, n - 1):
        for k, x in fl.tm_states(s).items():
            assert np.array_equal(x, re.tm_states(s)[k]), k
    for region in ("tm_seg_duty", "tm_seg_meta", "sp_perm"):  # the shared model: one instance
        assert np.array_equal(fl.export_state(region, 0, 1), re.export_state(region, 0, 1)), region
    # (the header's last 8 bytes count algorithmic bytes: the loaded fleet's
    # deferred log starts empty, so it logs sets the saved one deduplicated)
    assert np.array_equal(fl.export_state("tm_header")[:, :-8], re.export_state("tm_header")[:, :-8])
    import os
    model_bytes = sum(fl.state_bytes(r) for r in ("sp_perm", "sp_potmask", "sp_connT", "tm_seg_src", "tm_seg_perm"))
    assert os.path.getsize(path) < 2 * model_bytes + n * 64 * 1024
