"""The headline configuration beside the oracle, at full size.

BASELINE.json configs[1] / SURVEY.md §8(d) config 2, run exactly as bench.py
times it: 1,024 replicas of the GPU-trained Model-1 state
(bench.trained_engine: the reference's 2,184 training records,
ModelTraining.py:88-93 with NetworkModel.py:123-127's save-before-step),
SP+TM learning off, bench.make_inputs' synthetic streams, the untimed warm-up
as one htm_run chunk, then lockstep htm_step with the deferred dutyCycle()
writes on (HTM_OPT_DEFER_DUTY, flushed beside the steps on the engine's own
stream).  Sampled streams -- including both sides of the 768-workgroup
residency boundary (3 per CU x 256 CUs) and the last stream -- are held
against independent oracle clones on every step: the score, the SP active
columns, the TM output cells and the predicted-column set (nonzero
colConfidence) of each step; after htm_flush the full TM
state of two streams (segment dutyCycle records included) must equal the
oracle's.  Oracle parity w.r.t. NuPIC itself is unpinned.

Also the round-2 advisor's case: a frozen -> TM-learning -> frozen cycle must
not let a set logged before the learning phase suppress a write after it.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from test_gpu_parity import tm_equal  # noqa: E402

SAMPLED = [0, 1, 97, 511, 767, 768, 1000, 1023]


def test_config2_lockstep_1024_replicas_vs_oracle(rt, oracle_mod, traces):
    import bench
    n, warm, T = 1024, 64, 128
    train = np.asarray(traces["train"][:2184], np.float64)
    eng, _, _, _ = bench.trained_engine(rt, n, 72 * 1024, 0, train)
    eng.set_learning(False, False)
    trace = np.asarray(traces["test"], np.float64)
    vals = torch.tensor(bench.make_inputs(n, 0, n, 0, warm + T, trace), device="cuda")
    base = oracle_mod.OracleModel()
    for v in train:
        base.step([v], True, True)
    orcs = {s: base.clone() for s in SAMPLED}
    host = vals.cpu().numpy()
    scores = torch.empty((warm + T, n), dtype=torch.float32, device="cuda")
    eng.run(vals[:warm], out=scores[:warm])  # bench: the untimed warm-up
    g = scores[:warm].cpu().numpy()
    for s, o in orcs.items():
        for k in range(warm):
            assert g[k, s] == o.step([host[k, s]], False, False), f"warm-up step {k} stream {s}"
    c0 = eng.counters()
    idx = torch.tensor(SAMPLED, device="cuda")
    for k in range(warm, warm + T):
        eng.step(vals[k], out=scores[k])  # bench's timed region: lockstep
        # the SDR state of every sampled stream at this step (north_star: bit-exact
        # SDR state per step): SP active columns, TMRegion bottomUpOut (infActive |
        # infPredicted cells) and the predicted-column set nonzero(colConfidence(t))
        # the next score reads -- read without touching the packed state
        act = eng.get_output("active_columns").index_select(0, idx).cpu().numpy()
        out = eng.bitmap_to_dense(eng.get_output("tm_output").index_select(0, idx))
        pred = eng.get_output("pred_columns").index_select(0, idx).cpu().numpy()
        got = scores[k].cpu().numpy()
        for i, (s, o) in enumerate(orcs.items()):
            assert got[s] == o.step([host[k, s]], False, False), f"lockstep step {k} stream {s}: score"
            ao = np.zeros(eng.n_columns, np.uint8)
            ao[o.active_columns()] = 1
            assert np.array_equal(act[i], ao), f"lockstep step {k} stream {s}: active columns"
            assert np.array_equal(out[i], o.tm_output()), f"lockstep step {k} stream {s}: TM output cells"
            po = (o.col_confidence() != 0).astype(np.uint8)
            assert np.array_equal(pred[i], po), f"lockstep step {k} stream {s}: predicted columns"
    eng.flush()
    c1 = eng.counters()
    assert c1["error"] == 0
    assert c1["inf_backtracks"] - c0["inf_backtracks"] > n  # the deferred (discarded) phase 2s happened
    for s in (SAMPLED[0], SAMPLED[5]):
        tm_equal(eng, s, orcs[s])
    eng.status()
    eng.close()


def _replicas(rt, model, n):
    e = rt.HTMEngine(n, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        e.import_state(region, model.export_state(region, 0, 1), s0=0)
    e.replicate(0)
    return e


def test_frozen_learn_frozen_cycle_keeps_duty_writes(rt, oracle_mod, traces):
    """Lockstep frozen steps (deferred writes), then TM learning, then frozen
    again: the segment records (dutyCycle cache, meta) equal the undeferred
    engine's and the oracle's -- the deferred log is emptied when the index is
    rebuilt, so a recurring active set still finds its writes made at the new
    iteration.  The steps run on a non-default torch stream (the host-side
    state reads must still see every write)."""
    n = 24
    train = np.asarray(traces["train"][:2184], np.float64)
    model = rt.HTMEngine(1, seg_capacity=72 * 1024)
    model.run(torch.tensor(train, device="cuda").reshape(-1, 1))
    model.status()
    a, b = _replicas(rt, model, n), _replicas(rt, model, n)
    b.defer_duty(False)
    orc = oracle_mod.OracleModel()
    for v in train:
        orc.step([v], True, True)
    test = np.asarray(traces["test"], np.float64)
    rng = np.random.default_rng(5)
    phases = [(False, 48), (True, 24), (False, 64), (True, 8), (False, 40)]
    T = sum(p[1] for p in phases)
    idx = (np.arange(T)[:, None] + 41 * np.arange(n)[None, :]) % len(test)
    host = np.clip(test[idx] + rng.integers(-2, 3, size=idx.shape), 0, 100).astype(np.float64)
    vals = torch.tensor(host, device="cuda")
    side = torch.cuda.Stream()
    k = 0
    for tm_learn, steps in phases:
        for e in (a, b):
            e.set_learning(False, tm_learn)
        with torch.cuda.stream(side):
            ga = torch.stack([a.step(vals[k + j]) for j in range(steps)])
            gb = torch.stack([b.step(vals[k + j]) for j in range(steps)])
        side.synchronize()
        ga, gb = ga.cpu().numpy(), gb.cpu().numpy()
        assert np.array_equal(ga, gb)
        for j in range(steps):
            assert ga[j, 0] == orc.step([host[k + j, 0]], False, tm_learn), f"step {k + j}"
        for region in ("tm_seg_duty", "tm_seg_meta"):
            assert np.array_equal(a.export_state(region), b.export_state(region)), (region, k)
        k += steps
    tm_equal(a, 0, orc)
    for e in (a, b):
        e.status()
        e.close()
    model.close()
