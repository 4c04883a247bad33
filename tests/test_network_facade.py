"""The batched Network facade (network.py): host-side logic on CPU, and the
reference's Model-1 call pattern driven through it on the GPU."""
import os

import numpy as np
import pytest

import reference_model1 as ref
from conftest import GOLDEN


def test_reference_params_translate_to_the_default_config(rt):
    enc = ref.create_encoder(rt)
    cfg = rt.network.engine_config(enc, dict(ref.SP_PARAMS, inputWidth=500), ref.TM_PARAMS)
    assert cfg.as_dict() == rt.default_config().as_dict()


def test_two_field_encoder_config(rt):
    enc = ref.create_encoder(rt, multilevel=True)
    assert enc.getWidth() == 1000 and [f.name for f in enc.fields()] == ["cpu", "mem"]
    cfg = rt.network.engine_config(enc, dict(ref.SP_PARAMS, inputWidth=1000), ref.TM_PARAMS)
    assert cfg.n_fields == 2


@pytest.mark.parametrize("region,key,val", [("sp", "globalInhibition", 0), ("tm", "globalDecay", 0.1),
                                            ("tm", "maxAge", 100000), ("tm", "outputType", "activeState1CellPerCol"),
                                            ("sp", "potentialRadius_x", 3), ("tm", "doPooling", True)])
def test_unsupported_parameters_raise(rt, region, key, val):
    enc = ref.create_encoder(rt)
    sp, tm = dict(ref.SP_PARAMS, inputWidth=500), dict(ref.TM_PARAMS)
    (sp if region == "sp" else tm)[key] = val
    with pytest.raises(ValueError):
        rt.network.engine_config(enc, sp, tm)


def test_input_width_mismatch_raises(rt):
    with pytest.raises(ValueError):
        rt.network.engine_config(ref.create_encoder(rt), dict(ref.SP_PARAMS, inputWidth=400), ref.TM_PARAMS)


def test_scalar_encoder_buckets_match_the_oracle(rt, oracle_mod):
    enc = ref.create_encoder(rt).fields()[0]
    m = oracle_mod.OracleModel()
    xs = np.concatenate([np.arange(-5, 106, 0.25), [np.nan, 33.3333, 0.104, 99.9]])
    b = enc.bucket_indices(xs)
    for x, bi in zip(xs, b):
        sdr = m.encode([x])
        on = np.nonzero(sdr)[0]
        if np.isnan(x):
            assert bi == -1 and len(on) == 0
        else:
            assert on[0] == bi and len(on) == 21 and enc.getBucketIndices(float(x)) == [bi]


def test_record_stream_batches_and_missing_values(rt):
    ds = rt.BatchRecordStream(["cpu"], n_streams=3)
    ds.setData([1.0, None, 3])
    v = ds.getNextRecord()
    assert v.shape == (3, 1) and np.isnan(v[1, 0]) and v[2, 0] == 3.0
    ds.setData(np.array([4, 5, 6]), np.array([7.0, 8.0, 9.0]))
    assert ds.getNextRecord().shape == (3, 2)
    ds.setData(42)  # scalar broadcast to every stream
    assert np.all(ds.getNextRecord() == 42)
    with pytest.raises(ValueError):
        ds.setData([1, 2])


def test_sensor_region_forwards_data_source(rt):
    # ModelTesting.initModels: network.regions[_RECORD_SENSOR].dataSource = ds (ModelTesting.py:178)
    net = rt.Network()
    s = net.addRegion("s", "py.RecordSensor", "{}")
    sp = net.addRegion("sp", "py.SPRegion", "{}")
    ds = rt.BatchRecordStream(["cpu"])
    net.regions["s"].dataSource = ds
    assert s.getSelf().dataSource is ds and net.regions["s"].dataSource is ds
    with pytest.raises(AttributeError):
        sp.dataSource = ds


def test_graph_errors_are_raised_before_any_gpu_work(rt):
    net = rt.Network()
    net.addRegion("s", "py.RecordSensor", "{}")
    with pytest.raises(ValueError):
        net.addRegion("s", "py.SPRegion", "{}")
    with pytest.raises(ValueError):
        net.addRegion("x", "py.KNNClassifierRegion", "{}")
    with pytest.raises(ValueError):
        net.link("s", "nope", "UniformLink", "")
    with pytest.raises(ValueError):
        net.regions["s"].setParameter("learningMode", True)
    with pytest.raises(RuntimeError):
        net.run(1)  # no SP/TM regions


def test_second_level_config_reads_the_l1_bottom_up_out(rt):
    # MultiLevelNetworkModel.py:92-93: l2 inputWidth = L1 TMRegion bottomUpOut count
    cfg = rt.network.engine_config(None, dict(ref.SP_PARAMS, inputWidth=24576), ref.TM_PARAMS, input_width=24576)
    d = cfg.as_dict()
    assert d["sdr_bits"] == 24576 and d["sp_columns"] == 2048 and d["tm_cells_per_col"] == 12
    with pytest.raises(ValueError):
        rt.network.engine_config(None, dict(ref.SP_PARAMS, inputWidth=2048), ref.TM_PARAMS, input_width=24576)


@pytest.mark.parametrize("anomaly", [False, True])
def test_multilevel_graph_resolves_to_two_levels(rt, anomaly):
    """The Model 2/3 graphs (feedback link included) resolve to a sensor and two
    SP -> TM levels; classifiers attach to the level that feeds them."""
    net = ref.create_multilevel_network(rt, rt.BatchRecordStream(["cpu", "mem"] if anomaly else ["cpu"]),
                                        anomaly=anomaly)
    sensor, levels, cls = net._chain()
    assert sensor.name == ref.SENSOR
    assert [(lv.sp.name, lv.tm.name) for lv in levels] == [(ref.SPR, ref.TMR), (ref.L2_SPR, ref.L2_TMR)]
    assert cls == ({ref.CLS: 0, ref.L2_CLS: 1} if anomaly else {ref.L2_CLS: 1})


def test_dangling_second_level_raises(rt):
    net = ref.create_one_level_network(rt, rt.BatchRecordStream(["cpu"]))
    net.addRegion("l2sp", "py.SPRegion", "{}")  # never linked
    with pytest.raises(RuntimeError, match="not on the"):
        net._chain()


@pytest.mark.gpu
def test_model1_through_the_facade_matches_golden(rt, traces, tmp_path):
    """ModelTraining/ModelTesting's call pattern through the drop-in surface:
    setData -> run(1) -> getOutputData('anomalyScore')[0], save before the
    2185th step, reload with Network(path), TM learning off."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    g = np.load(os.path.join(GOLDEN, "model1_golden.npz"))
    ds = rt.BatchRecordStream(["cpu"])
    net = ref.create_one_level_network(rt, ds, seg_capacity=72 * 1024)
    tmr = net.regions[ref.TMR]
    got = []
    for k, cpu in enumerate(traces["train"][:2184]):
        ds.setData(float(cpu))
        net.run(1)
        got.append(tmr.getOutputData("anomalyScore")[0])
        if k == 0:
            act = net.regions[ref.SPR].getOutputData("bottomUpOut")[0]
            assert np.array_equal(np.nonzero(act)[0], np.sort(g["train_active"][0]))
            assert net.regions[ref.SENSOR].getOutputData("actValueOut")[0] == cpu
    assert np.array_equal(np.array(got, np.float32), g["train_scores"])
    path = net.save(str(tmp_path / "network1.nta"))
    net2 = rt.Network(path)
    ds2 = rt.BatchRecordStream(["cpu"])
    net2.regions[ref.SENSOR].dataSource = ds2  # the reference's own line, ModelTesting.py:178
    assert net2.regions[ref.SENSOR].getSelf().dataSource is ds2
    tm2 = net2.regions[ref.TMR]
    for r, cpu in enumerate(traces["test"][:40]):
        win = []
        for j in range(8):
            ds2.setData(float(cpu))
            if j == 0:
                tm2.setParameter("learningMode", False)  # NetworkModel.py:40-44
            net2.run(1)
            win.append(tm2.getOutputData("anomalyScore")[0])
        assert np.array_equal(np.array(win, np.float32), g["test_windows"][r])
    # the classifier (restored from the saved network) ran alongside: one
    # distribution per step over the buckets it has seen
    p = net2.regions[ref.CLS].getOutputData("probabilities")
    assert p.shape == (7 * 1000,)
    assert np.allclose(p.reshape(7, 1000).sum(axis=1), 1.0)


@pytest.mark.gpu
def test_batched_facade_streams_are_independent(rt, traces):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    n = 4
    ds = rt.BatchRecordStream(["cpu"], n_streams=n)
    net = ref.create_one_level_network(rt, ds, n_streams=n, seg_capacity=1 << 13)
    ds1 = rt.BatchRecordStream(["cpu"])
    one = ref.create_one_level_network(rt, ds1, seg_capacity=1 << 13)
    rng = np.random.default_rng(11)
    for k in range(60):
        v = np.clip(traces["train"][k] + rng.integers(-3, 4, size=n), 0, 100).astype(np.float64)
        ds.setData(v)
        net.run(1)
        ds1.setData(float(v[2]))
        one.run(1)
        a = net.regions[ref.TMR].getOutputData("anomalyScore")
        assert a.shape == (n,)
        assert a[2] == one.regions[ref.TMR].getOutputData("anomalyScore")[0]


@pytest.mark.gpu
@pytest.mark.parametrize("anomaly", [False, True])
def test_multilevel_facade_matches_engine_pair_and_reloads(rt, traces, tmp_path, anomaly):
    """Models 2/3 through the drop-in surface: the l2 TMRegion anomalyScore
    (MultiLevelNetworkModel.py:150, MultiLevelNetworkAnomaly.py:171) equals two
    engines driven directly (L1 step -> tm_output -> L2 step_sdr, whose oracle
    parity tests/test_multilevel_gpu.py holds), and a saved bundle
    (network2/3.nta: engine.htm + engine_l2.htm + classifiers) resumes exactly."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    names = ["cpu", "mem"] if anomaly else ["cpu"]
    ds = rt.BatchRecordStream(names)
    net = ref.create_multilevel_network(rt, ds, anomaly=anomaly, seg_capacity=1 << 13)
    nf = len(names)
    l1 = rt.HTMEngine(1, n_fields=nf, seg_capacity=1 << 13)
    l2 = rt.HTMEngine(1, sdr_bits=24576, seg_capacity=1 << 13)
    cpu = np.asarray(traces["train"][:90], np.float64)
    mem = np.clip(100.0 - cpu, 0, 100)
    recs = np.stack([cpu, mem], axis=1)[:, :nf]
    tmr2 = net.regions[ref.L2_TMR]
    for k in range(60):
        ds.setData(*[float(x) for x in recs[k]])
        net.run(1)
        l1.step(torch.tensor(recs[k], device="cuda"))
        want = l2.step_sdr(l1.get_output("tm_output")).cpu().numpy()[0]
        assert tmr2.getOutputData("anomalyScore")[0] == want, f"step {k}"
    assert net.regions[ref.L2_SPR].getOutputData("bottomUpOut").shape == (1, 2048)
    p = net.regions[ref.L2_CLS].getOutputData("probabilities")
    assert p.shape == (7 * 1000,) and np.allclose(p.reshape(7, 1000).sum(axis=1), 1.0)
    path = net.save(str(tmp_path / ("network3.nta" if anomaly else "network2.nta")))
    assert os.path.exists(os.path.join(path, "engine_l2.htm"))
    net2 = rt.Network(path)
    ds2 = rt.BatchRecordStream(names)
    net2.regions[ref.SENSOR].dataSource = ds2
    for r in (net, net2):
        r.regions[ref.TMR].setParameter("learningMode", False)
        r.regions[ref.L2_TMR].setParameter("learningMode", False)
    for k in range(60, 90):
        for d in (ds, ds2):
            d.setData(*[float(x) for x in recs[k]])
        net.run(1)
        net2.run(1)
        a = net.regions[ref.L2_TMR].getOutputData("anomalyScore")[0]
        assert a == net2.regions[ref.L2_TMR].getOutputData("anomalyScore")[0], f"step {k}"
        assert np.array_equal(net.regions[ref.L2_CLS].getOutputData("probabilities"),
                              net2.regions[ref.L2_CLS].getOutputData("probabilities"))


def test_four_field_aggregate_encoder_with_per_field_ranges(rt):
    """north_star's cpu %, mem %, mean and max response time (StreamAggregator.py:101-115):
    fields share n/w/clipInput, each keeps its own [minval, maxval]."""
    enc = rt.MultiEncoder()
    spec = {k: {"fieldname": k, "type": "ScalarEncoder", "name": k, "minval": 0.0, "maxval": hi,
                "clipInput": True, "w": 21, "n": 500}
            for k, hi in (("cpu", 100.0), ("mem", 100.0), ("mean", 2000.0), ("max", 5000.0))}
    enc.addMultipleEncoders(spec)
    cfg = rt.network.engine_config(enc, dict(ref.SP_PARAMS, inputWidth=2000, columnCount=4096),
                                   dict(ref.TM_PARAMS, columnCount=4096, inputWidth=4096)).as_dict()
    names = [f.name for f in enc.fields()]
    assert cfg["n_fields"] == 4 and cfg["sp_columns"] == 4096
    assert cfg["field_maxval"] == [dict(cpu=100.0, mem=100.0, mean=2000.0, max=5000.0)[k] for k in names]
    spec["mem"]["w"] = 11
    bad = rt.MultiEncoder()
    bad.addMultipleEncoders(spec)
    with pytest.raises(ValueError):
        rt.network.engine_config(bad, dict(ref.SP_PARAMS, inputWidth=1990), ref.TM_PARAMS)
