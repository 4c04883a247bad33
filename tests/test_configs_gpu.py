"""BASELINE.json configs 3, 4 and 5 at (or near) their stated sizes, against
independent oracle models on sampled streams, plus the size-independent
properties the domain offers (identical inputs -> identical outputs; a stream
is unaffected by the other streams of its launch).

Config 3: 65,536 streams learning on (BASELINE configs[2]) with the paged SP
          permanences the bench uses (htm_config.sp_perm_rows): 512 fresh
          streams with per-stream seeds, every step of 8 sampled streams
          checked against the oracle and the full SP/TM state of two; and the
          full 65,536 streams over config 3's 256 steps, 5 sampled streams
          against the oracle every step.
Config 4: fleet mode, 131,072 streams sharing one frozen model (configs[3]).
Config 5: the cpu / mem / mean / max response-time aggregate
          (StreamEngine/StreamAggregator.py:101-115) through a 4-field
          MultiEncoder into a 4096-column SP (configs[4]).
"""
import os

import numpy as np
import pytest

from test_gpu_parity import sp_equal, tm_equal

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

TRAIN = 300  # training records of the fleet's model (the oracle replays them too)


@pytest.fixture(scope="module")
def fleet_model(rt, oracle_mod, traces):
    """Model 1 trained on the first TRAIN records, on the GPU and in the oracle
    (bit-exact to each other: test_gpu_parity), then TM learning off as in
    ModelTesting (NetworkModel.py:40-44)."""
    tr = np.asarray(traces["train"][:TRAIN], np.float64)
    eng = rt.HTMEngine(1, seg_capacity=1 << 14)
    eng.run(torch.tensor(tr, device="cuda").reshape(-1, 1))
    eng.status()
    orc = oracle_mod.OracleModel()
    for x in tr:
        orc.step([x], True, True)
    return eng, orc


def fleet_inputs(traces, n, T, seed=29):
    rng = np.random.default_rng(seed)
    test = np.asarray(traces["test"], np.float64)
    t = np.arange(T)[:, None]
    s = np.arange(n)[None, :]
    v = np.clip(test[(t + 37 * s) % len(test)] + rng.integers(-2, 3, size=(T, n)), 0, 100)
    v[rng.random(v.shape) < 0.01] = np.nan
    return v


def test_config4_fleet_131072_streams_vs_oracle(rt, fleet_model, traces):
    """131,072 streams share the frozen model (SP and TM learning off); 8
    sampled streams replayed by independent oracle clones of the trained
    model over 64 lockstep steps; streams 2^16.. repeat the inputs of streams
    0.. and must repeat their scores; a one-stream fleet on one stream's
    inputs gives that stream's scores (no cross-stream interference)."""
    model, orc = fleet_model
    n, T = 131072, 64
    vals = fleet_inputs(traces, n // 2, T)
    vals = np.concatenate([vals, vals], axis=1)  # identical-input pairs s, s + 65536
    fl = rt.HTMEngine.fleet(model, n, q_capacity=4096)
    v = torch.tensor(vals, device="cuda")
    got = np.stack([fl.step(v[k]).cpu().numpy() for k in range(T)])
    fl.status()
    assert np.array_equal(got[:, : n // 2], got[:, n // 2:])
    sample = [0, 1, 4097, 20011, 33333, 65535, 65536 + 777, n - 1]
    for s in sample:
        o = orc.clone()
        want = np.array([o.step([vals[k, s]], False, False) for k in range(T)], np.float32)
        assert np.array_equal(got[:, s], want), f"stream {s}"
    solo = rt.HTMEngine.fleet(model, 1, q_capacity=4096)
    s = 20011
    one = np.array([solo.step(torch.tensor(vals[k, s:s + 1], device="cuda")).cpu().numpy()[0] for k in range(T)])
    assert np.array_equal(one, got[:, s])
    # the score distribution is not degenerate (the model predicts something)
    assert 0 < np.count_nonzero(got == 0) < got.size


def test_config4_fleet_flush_beside_the_steps(rt, fleet_model, traces):
    """The deferred-write flush beside the steps (HTM_OPT_FLUSH_MODE 0) at fleet
    scale: 131,072 streams, 8-entry logs, a flush enqueued every 4 steps, each
    flush slower than those 4 steps -- so snapshots are taken while earlier
    flushes still run (the round-3 overlap).  96 lockstep steps: 8 sampled
    streams equal oracle clones at every step, the flush reports no error flag
    (ring / job-list / job checks, tm.hip), and the shared model's segment
    records (dutyCycle cache included) equal those of the same fleet flushed on
    the step stream -- no deferred write is lost."""
    model, orc = fleet_model
    n, T = 131072, 96
    vals = fleet_inputs(traces, n, T, seed=31)
    v = torch.tensor(vals, device="cuda")
    out = {}
    for mode in (0, 1):
        fl = rt.HTMEngine.fleet(model, n, q_capacity=4096)
        fl.flush_mode(mode)
        scores = torch.empty((T, n), dtype=torch.float32, device="cuda")
        for k in range(T):
            fl.step(v[k], out=scores[k])
        fl.flush()
        torch.cuda.synchronize()
        c = fl.counters()
        assert c["error"] == 0, f"mode {mode}: error flags {c['error']:#x}"
        fl.status()
        out[mode] = (scores.cpu().numpy(), fl.export_state("tm_seg_duty", 0, 1), fl.export_state("tm_seg_meta", 0, 1),
                     c)
        fl.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1]), "segment dutyCycle records differ: deferred writes lost"
    assert np.array_equal(out[0][2], out[1][2])
    for key in ("inf_phase2", "inf_backtracks"):
        assert out[0][3][key] == out[1][3][key], key
    got = out[0][0]
    for s in [0, 5, 4097, 33333, 65536 + 777, n - 1]:
        o = orc.clone()
        want = np.array([o.step([vals[k, s]], False, False) for k in range(T)], np.float32)
        assert np.array_equal(got[:, s], want), f"stream {s}"


def test_config4_fleet_131072_save_resume(rt, fleet_model, traces, tmp_path):
    """Checkpoint / resume at fleet scale (NetworkModel.py:123-125 saves the
    network before the step, ModelTesting.py:176 reloads it): a 131,072-stream
    fleet saved after 40 lockstep steps (deferred writes pending) and loaded
    back continues bit-exactly like the fleet that was not saved -- every
    stream's scores, sampled streams' cell states, the shared model's segment
    records -- and sampled streams equal oracle clones throughout."""
    model, orc = fleet_model
    n, T, cut = 131072, 72, 40
    vals = fleet_inputs(traces, n, T, seed=37)
    v = torch.tensor(vals, device="cuda")
    fl = rt.HTMEngine.fleet(model, n, q_capacity=4096)
    head = np.stack([fl.step(v[k]).cpu().numpy() for k in range(cut)])
    path = str(tmp_path / "fleet131072.htm")
    fl.save(path)
    re = rt.HTMEngine.load(path)
    assert re.is_fleet and re.n_streams == n
    a = np.stack([fl.step(v[k]).cpu().numpy() for k in range(cut, T)])
    b = np.stack([re.step(v[k]).cpu().numpy() for k in range(cut, T)])
    assert np.array_equal(a, b)
    fl.status()
    re.status()
    for s in (0, 77777, n - 1):
        sa, sb = fl.tm_states(s), re.tm_states(s)
        for k in sa:
            assert np.array_equal(sa[k], sb[k]), (s, k)
    for region in ("tm_seg_duty", "tm_seg_meta"):  # the shared model: one instance
        assert np.array_equal(fl.export_state(region, 0, 1), re.export_state(region, 0, 1)), region
    got = np.concatenate([head, b])
    for s in (3, 65536 + 11, n - 2):
        o = orc.clone()
        want = np.array([o.step([vals[k, s]], False, False) for k in range(T)], np.float32)
        assert np.array_equal(got[:, s], want), f"stream {s}"
    re.close()
    fl.close()
    os.remove(path)


def test_config3_many_fresh_streams_learning(rt, oracle_mod):
    """512 fresh streams (seed per stream) with SP+TM learning on: 8 sampled
    streams match independent oracle models at every step; two of them match
    in their whole SP/TM state at the end."""
    n, T = 512, 120
    eng = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 13, sp_perm_rows=1536)
    rng = np.random.default_rng(41)
    base = rng.integers(0, 101, size=(40, 1)).astype(np.float64)
    vals = np.clip(np.tile(base, (3, n)) + rng.integers(-4, 5, size=(T, n)), 0, 100)
    vals[rng.random(vals.shape) < 0.02] = np.nan
    v = torch.tensor(vals, device="cuda")
    eng.set_learning(True, True)
    got = np.stack([eng.step(v[k]).cpu().numpy() for k in range(T)])
    eng.status()
    sample = [0, 3, 64, 127, 200, 311, 448, n - 1]
    orcs = {s: oracle_mod.OracleModel(sp_seed=2045 + s, tm_seed=2045 + s) for s in sample}
    for s, o in orcs.items():
        want = np.array([o.step([vals[k, s]], True, True) for k in range(T)], np.float32)
        assert np.array_equal(got[:, s], want), f"stream {s}"
    for s in (sample[2], sample[-1]):
        sp_equal(eng, s, orcs[s])
        tm_equal(eng, s, orcs[s])


def test_config3_65536_streams_paged_vs_oracle(rt, oracle_mod, traces):
    """Config 3 at its stated size and horizon (65,536 fresh
    learning streams, T = 256; the reference trains through the whole file,
    ModelTraining.py:91-93): seed 2045 + s, one GPU, paged SP permanences, the
    bench's inputs (trace + jitter), 256 lockstep steps; 5 sampled streams
    equal independent oracle models at every step -- score, SP active columns
    and TM output cells -- and, after the last step, one in its whole SP state
    and one in its whole TM state (segments, synapses, permanences, RNG)."""
    import bench
    n, T = 65536, 256
    sampled = (0, 1, 31337, 40961, n - 1)
    trace = np.asarray(traces["test"], np.float64)
    vals = bench.make_inputs(n, 0, n, 0, T, trace)
    cfg = rt.default_config(seg_capacity=10240, upd_capacity=512, seed_stride=1, sp_perm_rows=800)
    eng = rt.HTMEngine(n, config=cfg)
    v = torch.tensor(vals, device="cuda")
    idx = torch.tensor(sampled, device="cuda")
    orcs = [oracle_mod.OracleModel(sp_seed=2045 + s, tm_seed=2045 + s) for s in sampled]
    for k in range(T):
        got = eng.step(v[k]).index_select(0, idx).cpu().numpy()
        act = eng.get_output("active_columns").index_select(0, idx).cpu().numpy()
        out = eng.bitmap_to_dense(eng.get_output("tm_output").index_select(0, idx))
        for i, (s, o) in enumerate(zip(sampled, orcs)):
            assert got[i] == o.step([vals[k, s]], True, True), f"step {k} stream {s}: score"
            ao = np.zeros(eng.n_columns, np.uint8)
            ao[o.active_columns()] = 1
            assert np.array_equal(act[i], ao), f"step {k} stream {s}: active columns"
            assert np.array_equal(out[i], o.tm_output()), f"step {k} stream {s}: TM output cells"
    eng.status()
    assert 0 < eng.sp_perm_rows_used() <= n * 800
    sp_equal(eng, n - 1, orcs[-1])
    tm_equal(eng, 31337, orcs[2])


# response times in ms next to cpu/mem percent: per-field encoder ranges
FIELDS = [("cpu", 0.0, 100.0), ("max", 0.0, 5000.0), ("mean", 0.0, 2000.0), ("mem", 0.0, 100.0)]


def aggregate_records(traces, T, seed=13):
    """cpu/mem from the reference's traces; mean/max response time (ms) a noisy
    function of load, the shape StreamAggregator emits."""
    rng = np.random.default_rng(seed)
    cpu = np.asarray(traces["train"][:T], np.float64)
    mem = np.clip(0.6 * cpu + 20 + rng.normal(0, 3, T), 0, 100)
    mean = np.clip(150 + 12 * cpu + rng.normal(0, 40, T), 0, None)
    mx = np.clip(mean * rng.uniform(1.5, 3.0, T), 0, None)
    return np.stack([cpu, mx, mean, mem], axis=1)


def test_config5_four_field_aggregate_4096_columns(rt, oracle_mod, traces):
    """cpu / max / mean / mem (sorted field order, per-field ranges) through
    the 4-field encoder into the 4096-column SP, learning on, then TM learning
    off; bit-exact against the oracle every step and in the final state."""
    rec = aggregate_records(traces, 200)
    rec[7, 1] = np.nan  # a missing aggregate field
    mins = tuple(f[1] for f in FIELDS)
    maxs = tuple(f[2] for f in FIELDS)
    eng = rt.HTMEngine(1, n_fields=4, sp_columns=4096, seg_capacity=1 << 13,
                       field_minval=mins, field_maxval=maxs)
    orc = oracle_mod.OracleModel(n_fields=4, sp_columns=4096)
    for f in range(4):
        orc.params.field_minval[f], orc.params.field_maxval[f] = mins[f], maxs[f]
    orc = oracle_mod.OracleModel(orc.params)
    # the per-field ranges reach the encoder: field 1 = max response time
    x = [50.0, 2500.0, 1000.0, 50.0]
    sdr = orc.encode(x)
    for f in range(4):
        res = (maxs[f] - mins[f]) / (500 - 21)  # ScalarEncoder resolution (Appendix A.1)
        assert np.nonzero(sdr[500 * f:500 * (f + 1)])[0][0] == int(((x[f] - mins[f]) + res / 2.0) / res)
    for part, (sp_l, tm_l) in ((rec[:150], (True, True)), (rec[150:], (True, False))):
        eng.set_learning(sp_l, tm_l)
        for k in range(part.shape[0]):
            g = eng.step(torch.tensor(part[k], device="cuda")).cpu().numpy()[0]
            o = orc.step(part[k], sp_l, tm_l)
            assert g == o, f"record {k}: gpu {g} oracle {o}"
    sp_equal(eng, 0, orc)
    tm_equal(eng, 0, orc)


def test_config5_1024_streams_test_phase_vs_oracle(rt, oracle_mod, traces):
    """Config 5 at one GPU's shard: 1,024 streams of the bench's four-field
    aggregate model (bench.FIELDS5 ranges, bench.config5_inputs records: the
    reference's TestingData cpu/max/mean/mem, StreamAggregator.py:100-115)
    into 4096 columns.  Fresh streams (seed 2045 + s) learn 48 records
    (lockstep, SP+TM on), then run the test phase the way bench.run_config5
    does (ModelTesting.py:66-72: SP learning on, TM off, each record fed 1 + 7
    times in htm_run chunks, AnomalyLikelihood and the SLO harness per
    record).  Five sampled streams equal independent oracle models at every
    step; their likelihoods equal the restatement within 1e-6 relative (parity
    unpinned w.r.t. NuPIC) and their SLO counts the literal harness exactly.
    (Fresh streams instead of the bench's trained state keep the oracle's
    share of the test to seconds.)"""
    import bench
    import likelihood_reference as lr
    from test_slo_harness import gpu_stats, ref_stats
    n, L, R, W = 1024, 48, 80, 8
    sampled = (0, 1, 333, 700, n - 1)
    mins = tuple(f[1] for f in bench.FIELDS5)
    maxs = tuple(f[2] for f in bench.FIELDS5)
    d = traces["raw"]
    rec, means, viol = bench.config5_inputs(d, n, 0, n, L + R)
    rec[5, 17, 1] = np.nan  # a missing aggregate field (learning phase)
    rec[L + 3, 333, 2] = np.nan  # ... and in a test record of a sampled stream
    eng = rt.HTMEngine(n, seed_stride=1, n_fields=4, sp_columns=4096, seg_capacity=1 << 13,
                       field_minval=mins, field_maxval=maxs)
    lkp = dict(learning_period=30, estimation_samples=20, historic_window=120, reestimation_period=25)
    lik = rt.AnomalyLikelihood(n, **lkp)
    slo = rt.SLOHarness(n, threshold=0.98)
    v = torch.tensor(rec, device="cuda")
    idx = torch.tensor(sampled, device="cuda")
    eng.set_learning(True, True)
    learn = np.stack([eng.step(v[k]).index_select(0, idx).cpu().numpy() for k in range(L)])
    eng.set_learning(True, False)
    eng.set_run_chunk(16 * W)
    vals = v[L:].repeat_interleave(W, dim=0)
    scores = torch.empty((R * W, n), dtype=torch.float32, device="cuda")
    liks = torch.empty((R, n), dtype=torch.float64, device="cuda")
    mt, vt = torch.tensor(means[L:], device="cuda"), torch.tensor(viol[L:], device="cuda")
    for a in range(0, R, 16):
        eng.run(vals[a * W:(a + 16) * W], out=scores[a * W:(a + 16) * W])
        for r in range(a, a + 16):
            lik.anomaly_probability(v[L + r], scores[r * W], out=liks[r])
            slo.record(scores[r * W:(r + 1) * W], vt[r], mt[r])
    eng.status()
    got = scores.index_select(1, idx).cpu().numpy().reshape(R, W, len(sampled))
    got_lik = liks.index_select(1, idx).cpu().numpy()
    stats = slo.stats()
    orcs = []
    for s in sampled:
        p = oracle_mod.default_params(sp_seed=2045 + s, tm_seed=2045 + s, n_fields=4, sp_columns=4096)
        for f in range(4):
            p.field_minval[f], p.field_maxval[f] = mins[f], maxs[f]
        orcs.append(oracle_mod.OracleModel(p))
    for k in range(L):
        for i, (s, o) in enumerate(zip(sampled, orcs)):
            assert learn[k, i] == o.step(rec[k, s], True, True), f"learning record {k} stream {s}"
    for i, (s, o) in enumerate(zip(sampled, orcs)):
        ref = lr.AnomalyLikelihood(lkp["learning_period"], lkp["estimation_samples"], lkp["historic_window"],
                                   lkp["reestimation_period"])
        windows = []
        for r in range(R):
            win = [o.step(rec[L + r, s], True, False) for _ in range(W)]
            assert np.array_equal(got[r, :, i], np.array(win, np.float32)), f"test record {r} stream {s}"
            want_lik = ref.anomaly_probability(rec[L + r, s, 0], float(win[0]))
            np.testing.assert_allclose(got_lik[r, i], want_lik, rtol=1e-6, atol=0, err_msg=f"record {r} stream {s}")
            windows.append(win)
        assert gpu_stats(stats[s]) == ref_stats(windows, means[L:, s], viol[L:, s], 0.98), f"SLO stream {s}"
    assert np.any(got_lik != 0.5)
