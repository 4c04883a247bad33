"""Ordered lockstep launches (HTM_OPT_ORDERED).

A frozen lockstep launch runs every stream's SP first, then the TM steps in
order of their predicted cost, each on whichever workgroup takes it.  Streams
are independent, so everything observable must equal the one-workgroup-per-
stream launch: scores at every step, the phase-2 / backtrack counters and the
byte counter, and the exported state -- with SP learning on and off (the
fused SP+learning kernel), deferral on and off, and stream counts below and
above the resident workgroups.
"""
import numpy as np
import pytest

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


def replicas(rt, model1, n):
    e = rt.HTMEngine(n, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        e.import_state(region, model1.export_state(region, 0, 1), s0=0)
    e.replicate(0)
    return e


def lockstep(e, vals):
    return np.stack([e.step(vals[k]).cpu().numpy() for k in range(vals.shape[0])])


@pytest.mark.parametrize("n,sp_learn,defer", [(300, False, True), (1024, False, True), (1024, True, True),
                                              (300, False, False), (2000, True, False)])
def test_ordered_equals_stream_order(rt, model1, traces, n, sp_learn, defer):
    T = 64
    rng = np.random.default_rng(7 + n)
    test = np.asarray(traces["test"], np.float64)
    t = np.arange(T)[:, None]
    s = np.arange(n)[None, :]
    vals = torch.tensor(np.clip(test[(t + 53 * s) % len(test)] + rng.integers(-2, 3, size=(T, n)), 0, 100),
                        device="cuda")
    a = replicas(rt, model1, n)
    b = replicas(rt, model1, n)
    b.ordered_steps(False)
    for e in (a, b):
        e.set_learning(sp_learn, False)
        e.defer_duty(defer)
        e.flush_mode(1)  # (the flush after the steps: the byte counter's fresh-record writes are then exact)
    ga, gb = lockstep(a, vals), lockstep(b, vals)
    assert np.array_equal(ga, gb)
    ca, cb = a.counters(), b.counters()
    for k in ("tm_bytes", "inf_phase2", "inf_backtracks", "seg_live", "error"):
        assert ca[k] == cb[k], k
    assert ca["error"] == 0 and ca["inf_backtracks"] > 0
    for region in ("tm_seg_duty", "tm_bitmaps", "tm_colconf", "tm_header", "sp_perm", "sp_duty"):
        assert np.array_equal(a.export_state(region), b.export_state(region)), region


def test_retired_options_are_refused(rt, model1):
    """ABI 6 removed HTM_OPT_WIDE (15) and flush mode 2 (both measured
    slower): setting them fails loudly."""
    e = replicas(rt, model1, 4)
    with pytest.raises(RuntimeError):
        e.set_option(15, 1)
    with pytest.raises(RuntimeError):
        e.flush_mode(2)
    e.flush_mode(1)
    e.flush_mode(0)
