"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Integer/index state must be bit-exact (active columns, cell states, segment
and synapse tables, RNG state); float32 state (permanences, duty cycles,
column confidences, scores) is compared bit-exactly as well -- both sides
run the same float32 operation order with FMA contraction off.  Oracle
parity w.r.t. NuPIC itself is unpinned (oracle/htm_oracle.h).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)


def sp_equal(eng, s, orc):
    a, b = eng.sp_state(s), orc.sp_state()
    for k in ["potential", "perm", "connected", "overlap_dc", "active_dc"]:
        assert np.array_equal(a[k], b[k]), f"SP {k} differs"
    assert (a["iter"], a["iter_learn"]) == (b["iter"], b["iter_learn"])
    assert a["min_overlap_dc"] == b["min_overlap_dc"][0]


def tm_equal(eng, s, orc):
    a, b = eng.tm_states(s), orc.tm_states()
    for k in a:
        assert np.array_equal(a[k], b[k]), f"TM {k} differs"
    assert np.array_equal(eng.col_confidence(s), orc.col_confidence())
    sa, sb = eng.tm_segments(s), orc.tm_segments(32)
    assert len(sa["cell"]) == len(sb["cell"])
    for k in ["cell", "is_seq", "pos_act", "last_dc_iter", "nsyn", "last_dc", "src", "perm"]:
        assert np.array_equal(sa[k], sb[k]), f"segment {k} differs"
    h, sc = eng.tm_header(s), orc.tm_scalars()
    assert (h.lrn_iter, h.iter, h.pam_counter, h.learned_seq_length, h.n_inf_pat, h.n_lrn_pat, h.n_upd) == (
        sc["lrn_iter"], sc["iter"], sc["pam_counter"], sc["learned_seq_length"], sc["n_prev_inf"],
        sc["n_prev_lrn"], sc["n_updates"])
    assert h.avg_input_density == sc["avg_input_density"]
    r = orc.tm_rng_state()
    assert list(h.rng_state) == list(r[:31]) and (h.rng_f, h.rng_r) == (r[31], r[32])
    inf_g, lrn_g = eng.tm_patterns(s)
    assert h.error == 0


def run_pair(eng, orcs, values, sp_learn, tm_learn, check_active=True):
    eng.set_learning(sp_learn, tm_learn)
    n = len(orcs)
    nf = eng.n_fields
    for k in range(values.shape[0]):
        v = values[k].reshape(n, nf)
        g = eng.step(torch.tensor(v.ravel(), device="cuda")).cpu().numpy()
        act = eng.get_output("active_columns").cpu().numpy() if check_active else None
        for s in range(n):
            o = orcs[s].step(v[s], sp_learn, tm_learn)
            assert g[s] == o, f"step {k} stream {s}: gpu {g[s]} oracle {o}"
            if check_active:
                ao = np.zeros(eng.n_columns, np.uint8)
                ao[orcs[s].active_columns()] = 1
                assert np.array_equal(act[s], ao), f"active columns differ at step {k} stream {s}"


def test_init_parity_per_stream_seeds(rt, oracle_mod):
    eng = rt.HTMEngine(3, seed_stride=7, seg_capacity=1024)
    for s in range(3):
        orc = oracle_mod.OracleModel(sp_seed=2045 + 7 * s, tm_seed=2045 + 7 * s)
        sp_equal(eng, s, orc)
        r = orc.tm_rng_state()
        h = eng.tm_header(s)
        assert list(h.rng_state) == list(r[:31]) and (h.rng_f, h.rng_r) == (r[31], r[32])


def test_model1_training_prefix(rt, oracle_mod, traces):
    eng = rt.HTMEngine(1, seg_capacity=1 << 14)
    orc = oracle_mod.OracleModel()
    vals = traces["train"][:400].reshape(-1, 1)
    run_pair(eng, [orc], vals[:200], True, True)
    sp_equal(eng, 0, orc)
    tm_equal(eng, 0, orc)
    run_pair(eng, [orc], vals[200:400], True, True, check_active=False)
    sp_equal(eng, 0, orc)
    tm_equal(eng, 0, orc)
    # inference (TM learning off, SP on) through the frozen index, then the scan
    te = traces["test"][:120].reshape(-1, 1)
    run_pair(eng, [orc], te[:60], True, False)
    assert eng.frozen_index_valid()
    tm_equal(eng, 0, orc)
    eng.use_frozen_index(False)
    run_pair(eng, [orc], te[60:], True, False)
    tm_equal(eng, 0, orc)
    sp_equal(eng, 0, orc)


def digest_sp(st):
    h = hashlib.sha256()
    for k in ["perm", "potential", "connected", "overlap_dc", "active_dc"]:
        h.update(np.ascontiguousarray(st[k]).tobytes())
    return h.hexdigest()


def digest_tm(seg):
    h = hashlib.sha256()
    for k in ["cell", "is_seq", "pos_act", "last_dc_iter", "nsyn", "last_dc", "src", "perm"]:
        h.update(np.ascontiguousarray(seg[k]).tobytes())
    return h.hexdigest()


@pytest.fixture(scope="module")
def trained(rt, traces):
    """Model 1 trained on the GPU over the 2184 records the saved network saw."""
    eng = rt.HTMEngine(1, seg_capacity=72 * 1024)
    v = torch.tensor(traces["train"][:2184], dtype=torch.float64, device="cuda").reshape(-1, 1)
    scores = eng.run(v).cpu().numpy().ravel()
    eng.status()
    return eng, scores


def test_model1_full_training_matches_golden(trained):
    g = np.load(os.path.join(GOLDEN, "model1_golden.npz"))
    eng, scores = trained
    assert np.array_equal(scores, g["train_scores"])
    assert digest_sp(eng.sp_state(0)) == str(g["sp_digest"])
    seg = eng.tm_segments(0)
    assert len(seg["cell"]) == int(g["n_segments"])
    assert int(seg["nsyn"].sum()) == int(g["n_synapses"])
    assert digest_tm({k: v for k, v in seg.items() if k != "slots"}) == str(g["tm_digest"])


@pytest.mark.parametrize("frozen", [True, False])
def test_model1_test_phase_matches_golden(rt, trained, traces, frozen, tmp_path):
    """ModelTesting: 1+7 steps per record, SP learning on, TM learning off."""
    g = np.load(os.path.join(GOLDEN, "model1_golden.npz"))
    base, _ = trained
    p = str(tmp_path / "network1.htm")
    base.save(p)  # the reference loads network1.nta (ModelTesting.py:176)
    eng = rt.HTMEngine.load(p)
    eng.set_learning(True, False)
    eng.use_frozen_index(frozen)
    n_rec = 2324 if frozen else 400
    v = np.repeat(traces["test"][:n_rec], 8).reshape(-1, 1)
    out = eng.run(torch.tensor(v, device="cuda")).cpu().numpy().reshape(n_rec, 8)
    assert np.array_equal(out, g["test_windows"][:n_rec])
    eng.status()


def test_multistream_learning_with_missing_values(rt, oracle_mod):
    n = 6
    eng = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 13)
    orcs = [oracle_mod.OracleModel(sp_seed=2045 + s, tm_seed=2045 + s) for s in range(n)]
    rng = np.random.default_rng(5)
    base = rng.integers(0, 101, size=(60, 1)).astype(np.float64)
    vals = np.clip(np.tile(base, (3, n)) + rng.integers(-3, 4, size=(180, n)), 0, 100).astype(np.float64)
    vals[rng.random(vals.shape) < 0.03] = np.nan
    run_pair(eng, orcs, vals, True, True)
    for s in [0, n - 1]:
        sp_equal(eng, s, orcs[s])
        tm_equal(eng, s, orcs[s])


def test_two_field_encoder_model3_shape(rt, oracle_mod):
    eng = rt.HTMEngine(2, n_fields=2, seed_stride=3, seg_capacity=1 << 12)
    orcs = [oracle_mod.OracleModel(n_fields=2, sp_seed=2045 + 3 * s, tm_seed=2045 + 3 * s) for s in range(2)]
    rng = np.random.default_rng(9)
    vals = rng.integers(0, 101, size=(80, 4)).astype(np.float64)
    run_pair(eng, orcs, vals, True, True)
    tm_equal(eng, 1, orcs[1])


def test_config5_shape_4096_columns_cpu_mem(rt, oracle_mod):
    """BASELINE config 5 shape: cpu+mem MultiEncoder (NetworkUtils.py:89-107,
    1000 input bits) into a 4096-column SP, Model-1 TM.  Learning on over the
    reference's training records, then TM learning off (frozen index) on the
    test records, the ModelTesting.py:40-44 switch."""
    tr = np.stack([np.asarray(traces_np()["train_cpu"]), np.asarray(traces_np()["train_mem"])], axis=1)
    tr = tr[~np.isnan(tr).any(axis=1)][:150]
    te = np.stack([traces_np()["test_cpu"], traces_np()["test_mem"]], axis=1)[:60].astype(np.float64)
    eng = rt.HTMEngine(1, n_fields=2, sp_columns=4096, seg_capacity=1 << 13)
    orc = oracle_mod.OracleModel(n_fields=2, sp_columns=4096)
    sp_equal(eng, 0, orc)
    run_pair(eng, [orc], tr, True, True)
    tm_equal(eng, 0, orc)
    run_pair(eng, [orc], te, True, False)
    sp_equal(eng, 0, orc)
    tm_equal(eng, 0, orc)


def traces_np():
    return np.load(os.path.join(GOLDEN, "model1_traces.npz"))


def test_32_cells_per_column(rt, oracle_mod):
    eng = rt.HTMEngine(1, tm_cells_per_col=32, seg_capacity=1 << 13)
    orc = oracle_mod.OracleModel(tm_cells_per_col=32)
    seq = np.array([10.0, 30.0, 50.0, 70.0, 90.0, 30.0, 10.0])
    vals = np.tile(seq, 20).reshape(-1, 1)
    run_pair(eng, [orc], vals, True, True)
    tm_equal(eng, 0, orc)


def test_reset(rt, oracle_mod):
    eng = rt.HTMEngine(1, seg_capacity=1 << 12)
    orc = oracle_mod.OracleModel()
    vals = np.tile([10.0, 20.0, 30.0, 40.0], 15).reshape(-1, 1)
    run_pair(eng, [orc], vals[:30], True, True)
    eng.tm_reset()
    orc.tm_reset()
    run_pair(eng, [orc], vals[30:], True, True)
    tm_equal(eng, 0, orc)


def test_save_load_roundtrip(rt, tmp_path):
    eng = rt.HTMEngine(2, seed_stride=1, seg_capacity=1 << 12)
    rng = np.random.default_rng(1)
    vals = torch.tensor(rng.integers(0, 101, size=(60, 2)).astype(np.float64), device="cuda")
    eng.run(vals[:40])
    p = str(tmp_path / "e.htm")
    eng.save(p)
    eng2 = rt.HTMEngine.load(p)
    a = eng.run(vals[40:]).cpu().numpy()
    b = eng2.run(vals[40:]).cpu().numpy()
    assert np.array_equal(a, b)
    for s in range(2):
        assert digest_tm({k: v for k, v in eng.tm_segments(s).items() if k != "slots"}) == \
            digest_tm({k: v for k, v in eng2.tm_segments(s).items() if k != "slots"})


def test_replicated_streams_are_independent_and_identical(rt, trained, traces):
    """Full-size property (config-2 shape): 1024 replicas of the trained
    state; streams fed identical inputs produce identical scores, and a
    stream's result does not depend on what the others are fed."""
    base, _ = trained
    n = 1024
    eng = rt.HTMEngine(n, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        eng.import_state(region, base.export_state(region, 0, 1), s0=0)
    eng.replicate(0)
    eng.set_learning(False, False)
    rng = np.random.default_rng(3)
    T = 40
    vals = np.repeat(traces["test"][:T, None], n, axis=1).astype(np.float64)
    noisy = np.clip(vals + rng.integers(-2, 3, size=vals.shape), 0, 100)
    vals[:, n // 2:] = noisy[:, n // 2:]
    out = eng.run(torch.tensor(vals, device="cuda")).cpu().numpy()
    assert np.all(out[:, : n // 2] == out[:, :1])
    # stream n-1 alone (replica engine of one stream) gives the same scores
    one = rt.HTMEngine(1, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        one.import_state(region, base.export_state(region, 0, 1), s0=0)
    one.set_learning(False, False)
    solo = one.run(torch.tensor(vals[:, n - 1:], device="cuda")).cpu().numpy().ravel()
    assert np.array_equal(out[:, n - 1], solo)
    eng.status()


def test_capacity_overflow_is_reported(rt):
    eng = rt.HTMEngine(1, seg_capacity=320)
    rng = np.random.default_rng(2)
    vals = torch.tensor(rng.integers(0, 101, size=(40, 1)).astype(np.float64), device="cuda")
    eng.run(vals)
    with pytest.raises(rt.HtmError):
        eng.status()


@pytest.mark.parametrize("unit", [0, 1, 5, 64])
def test_run_units_equal_lockstep_steps(rt, unit):
    """htm_run through the work queue (units of `unit` steps handed between
    workgroups; 0 = auto) equals one htm_step launch per step (the direct,
    queue-free path), learning on then TM frozen."""
    rng = np.random.default_rng(11)
    vals = rng.integers(0, 101, size=(90, 5)).astype(np.float64)
    a = rt.HTMEngine(5, seed_stride=1, seg_capacity=1 << 12)
    b = rt.HTMEngine(5, seed_stride=1, seg_capacity=1 << 12)
    a.set_run_unit(unit)
    for lo, hi, tm_learn in [(0, 60, True), (60, 90, False)]:
        a.set_learning(True, tm_learn)
        b.set_learning(True, tm_learn)
        ra = a.run(torch.tensor(vals[lo:hi], device="cuda")).cpu().numpy()
        rb = np.stack([b.step(torch.tensor(vals[k], device="cuda")).cpu().numpy() for k in range(lo, hi)])
        assert np.array_equal(ra, rb), f"unit {unit}: run and step differ in [{lo}, {hi})"
    for s in range(5):
        sa, sb = a.tm_states(s), b.tm_states(s)
        for k in sa:
            assert np.array_equal(sa[k], sb[k])


def test_deferred_learn_phase2_completed_anywhere(rt, oracle_mod):
    """A learning step leaves its final learn phase 2 pending (tm_core.h
    lp2_finish: the next step's first pool scan counts it).  Completing it
    early -- a state export (tm_lp2_finish_kernel) in the middle of lockstep
    learning, a mid-run save/load, an htm_run chunk boundary -- changes no
    result: scores at every step and the final SP/TM state equal an engine
    that never stops, and both equal the oracle."""
    n = 3
    rng = np.random.default_rng(5)
    vals = np.clip(np.tile(rng.integers(0, 101, size=(12, 1)), (8, n)) + rng.integers(-3, 4, size=(96, n)), 0, 100)
    vals = vals.astype(np.float64)
    v = torch.tensor(vals, device="cuda")
    a = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 12)
    b = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 12)
    orcs = [oracle_mod.OracleModel(sp_seed=2045 + s, tm_seed=2045 + s) for s in range(n)]
    for e in (a, b):
        e.set_learning(True, True)
    got_a, got_b = [], []
    for k in range(96):
        got_a.append(a.step(v[k]).cpu().numpy())
        if k % 7 == 3:
            a.export_state("tm_header")  # completes the pending phase mid-run
        if k == 50:
            got_b.append(b.run(v[50:70]).cpu().numpy())
        elif not 50 < k < 70:
            got_b.append(b.step(v[k]).cpu().numpy()[None])
    ga, gb = np.stack(got_a), np.concatenate(got_b)
    assert np.array_equal(ga, gb)
    for s in range(n):
        want = np.array([orcs[s].step([vals[k, s]], True, True) for k in range(96)], np.float32)
        assert np.array_equal(ga[:, s], want), f"stream {s}"
        tm_equal(a, s, orcs[s])
        tm_equal(b, s, orcs[s])
        assert a.tm_header(s).lp2_pending == 0
