"""Deferred dutyCycle() writes in frozen lockstep steps (HTM_OPT_DEFER_DUTY).

A frozen phase 2 whose confidences the step discards (backtrack replays,
out-of-sequence results) computes only the predicted cells; the first
dutyCycle() record write of its qualifying segments is logged and replayed by
the flush kernel.  Everything observable must equal the undeferred engine and
the oracle: scores at every step, segment records (dutyCycle cache included)
after any export, the phase-2 / backtrack counters -- with the log flushed on
its cadence, and with a log that fills (the step then counts in full).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)


@pytest.fixture(scope="module")
def model1(rt, traces):
    eng = rt.HTMEngine(1, seg_capacity=72 * 1024)
    eng.run(torch.tensor(traces["train"][:2184], dtype=torch.float64, device="cuda").reshape(-1, 1))
    eng.status()
    return eng


def replicas(rt, model1, n, flush_every=0):
    e = rt.HTMEngine(n, seg_capacity=72 * 1024)
    if flush_every:
        e.flush_every(flush_every)  # (HTM_OPT_FLUSH_EVERY: past the log ring, the log fills)
    for region in rt._lib.ST:
        e.import_state(region, model1.export_state(region, 0, 1), s0=0)
    e.replicate(0)
    return e


def lockstep(e, vals):
    return np.stack([e.step(vals[k]).cpu().numpy() for k in range(vals.shape[0])])


@pytest.mark.parametrize("sp_learn", [False, True])
@pytest.mark.parametrize("flush_every", [0, 100000], ids=["cadence", "log_fills"])
def test_deferred_equals_undeferred(rt, model1, traces, sp_learn, flush_every):
    n, T = 96, 160
    rng = np.random.default_rng(17)
    test = np.asarray(traces["test"], np.float64)
    t = np.arange(T)[:, None]
    s = np.arange(n)[None, :]
    vals = torch.tensor(np.clip(test[(t + 53 * s) % len(test)] + rng.integers(-2, 3, size=(T, n)), 0, 100),
                        device="cuda")
    a = replicas(rt, model1, n, flush_every)
    b = replicas(rt, model1, n)
    b.defer_duty(False)
    for e in (a, b):
        e.set_learning(sp_learn, False)
    ga, gb = lockstep(a, vals), lockstep(b, vals)
    assert np.array_equal(ga, gb)
    ca, cb = a.counters(), b.counters()
    for k in ("inf_phase2", "inf_backtracks", "seg_live", "error"):
        assert ca[k] == cb[k], k
    assert ca["inf_backtracks"] > 0
    for region in ("tm_seg_duty", "tm_seg_meta", "tm_bitmaps", "tm_colconf", "tm_header", "sp_perm"):
        xa, xb = a.export_state(region), b.export_state(region)
        if region == "tm_header":  # the algorithmic byte counter differs by design
            xa, xb = xa[:, :-8], xb[:, :-8]
        assert np.array_equal(xa, xb), region


def test_lockstep_test_phase_matches_golden(rt, model1, traces):
    """ModelTesting's 1+7 steps per record (ModelTesting.py:66-72), SP learning
    on, TM learning off, one htm_step per step with deferral on: the golden
    windows of the oracle, and the oracle's segment records after a save."""
    g = np.load(os.path.join(GOLDEN, "model1_golden.npz"))
    e = replicas(rt, model1, 1)
    e.set_learning(True, False)
    n_rec = 300
    v = torch.tensor(np.repeat(traces["test"][:n_rec], 8).reshape(-1, 1), device="cuda")
    out = lockstep(e, v).reshape(n_rec, 8)
    assert np.array_equal(out, g["test_windows"][:n_rec])
    ref = replicas(rt, model1, 1)
    ref.defer_duty(False)
    ref.set_learning(True, False)
    lockstep(ref, v)
    sa, sb = e.tm_segments(0), ref.tm_segments(0)
    for k in ("last_dc", "last_dc_iter", "pos_act"):
        assert np.array_equal(sa[k], sb[k]), k


def test_frozen_learn_frozen_cycle(rt, model1, traces):
    """Deferred writes across a frozen -> TM learning -> frozen cycle: the
    re-frozen index starts an empty log (engine.cpp build_fx), so an active
    set logged before the learning phase is not taken for one already written
    at the new iteration.  Scores, counters and the segment records (dutyCycle
    cache included) equal the undeferred engine in every phase."""
    n, T = 32, 48
    rng = np.random.default_rng(29)
    test = np.asarray(traces["test"], np.float64)
    t = np.arange(3 * T)[:, None]
    s = np.arange(n)[None, :]
    vals = torch.tensor(np.clip(test[(t + 31 * s) % len(test)] + rng.integers(-2, 3, size=(3 * T, n)), 0, 100),
                        device="cuda")
    a = replicas(rt, model1, n)
    b = replicas(rt, model1, n)
    b.defer_duty(False)
    for k, tm_learn in enumerate((False, True, False)):
        for e in (a, b):
            e.set_learning(False, tm_learn)
        ga, gb = lockstep(a, vals[k * T:(k + 1) * T]), lockstep(b, vals[k * T:(k + 1) * T])
        assert np.array_equal(ga, gb), k
        for region in ("tm_seg_duty", "tm_seg_meta"):
            assert np.array_equal(a.export_state(region), b.export_state(region)), (k, region)
    ca, cb = a.counters(), b.counters()
    for key in ("inf_phase2", "inf_backtracks", "lrn_phase2", "seg_live", "error"):
        assert ca[key] == cb[key], key
    assert ca["inf_backtracks"] > 0


def test_flush_overlapping_snapshots(rt, model1, traces):
    """A flush beside the steps (HTM_OPT_FLUSH_MODE 0) enqueued after every
    step (HTM_OPT_FLUSH_EVERY 1) with 2,048 streams: each flush takes longer
    than a step, so later snapshots land while earlier flushes run -- the
    case the per-flush bound (fx_dupto) exists for.  Scores, counters and the
    segment records (dutyCycle cache included) equal the undeferred engine."""
    n, T = 2048, 48
    rng = np.random.default_rng(43)
    test = np.asarray(traces["test"], np.float64)
    t = np.arange(T)[:, None]
    s = np.arange(n)[None, :]
    vals = torch.tensor(np.clip(test[(t + 37 * s) % len(test)] + rng.integers(-2, 3, size=(T, n)), 0, 100),
                        device="cuda")
    a = replicas(rt, model1, n, flush_every=1)
    a.flush_mode(0)
    b = replicas(rt, model1, n)
    b.defer_duty(False)
    for e in (a, b):
        e.set_learning(False, False)
    ga, gb = lockstep(a, vals), lockstep(b, vals)
    assert np.array_equal(ga, gb)
    ca, cb = a.counters(), b.counters()
    for k in ("inf_phase2", "inf_backtracks", "seg_live", "error"):
        assert ca[k] == cb[k], k
    assert ca["error"] == 0 and ca["inf_backtracks"] > 0
    for region in ("tm_seg_duty", "tm_seg_meta"):
        assert np.array_equal(a.export_state(region), b.export_state(region)), region

