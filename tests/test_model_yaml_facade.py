"""The reference's model.yaml parameter set through the drop-in facade.

ML/HTM/params/model.yaml lists the sensor's RandomDistributedScalarEncoder
(:15-21), spParams (:28-41) and tmParams (:45-63) of an OPF model; nothing in
the reference loads it.  Here those dicts go through the same surface the
reference's NetworkModel.py uses (MultiEncoder.addMultipleEncoders,
Network.addRegion with the region parameter JSON, link, setData, run(1),
getOutputData('anomalyScore')): the CPU test checks the translation to the
engine's config, the GPU test runs the network against the oracle.
"""
import json

import numpy as np
import pytest

YAML_ENCODER = {"cpu_metric": {"fieldname": "cpu_metric", "name": "cpu_metric", "resolution": 0.88, "seed": 1,
                               "type": "RandomDistributedScalarEncoder"}}
YAML_SP = {"inputWidth": 946, "columnCount": 2048, "spVerbosity": 0, "spatialImp": "cpp", "globalInhibition": 1,
           "localAreaDensity": -1.0, "numActiveColumnsPerInhArea": 40, "seed": 1956, "potentialPct": 0.85,
           "synPermConnected": 0.1, "synPermActiveInc": 0.04, "synPermInactiveDec": 0.005, "boostStrength": 3.0}
YAML_TM = {"verbosity": 0, "columnCount": 2048, "cellsPerColumn": 32, "inputWidth": 2048, "seed": 1960,
           "temporalImp": "cpp", "newSynapseCount": 20, "initialPerm": 0.21, "permanenceInc": 0.1,
           "permanenceDec": 0.1, "maxAge": 0, "globalDecay": 0.0, "maxSynapsesPerSegment": 32,
           "maxSegmentsPerCell": 128, "minThreshold": 12, "activationThreshold": 16, "outputType": "normal",
           "pamLength": 1}


def yaml_network(rt, ds, n_streams=1, **engine_opts):
    net = rt.Network(n_streams=n_streams, **engine_opts)
    net.addRegion("sensor", "py.RecordSensor", json.dumps({"verbosity": 0}))
    sensor = net.regions["sensor"].getSelf()
    enc = rt.MultiEncoder()
    enc.addMultipleEncoders(YAML_ENCODER)
    sensor.encoder = enc
    sensor.dataSource = ds
    # OPF sets the SP's inputWidth to the encoder's width (the yaml's 946 is overwritten)
    net.addRegion("sp", "py.SPRegion", json.dumps(dict(YAML_SP, inputWidth=enc.getWidth())))
    net.link("sensor", "sp", "UniformLink", "")
    net.addRegion("tm", "py.TMRegion", json.dumps(YAML_TM))
    net.regions["tm"].setParameter("anomalyMode", True)
    net.link("sp", "tm", "UniformLink", "")
    return net


def test_yaml_dicts_translate_to_the_model_yaml_config(rt):
    enc = rt.MultiEncoder()
    enc.addMultipleEncoders(YAML_ENCODER)
    assert enc.getWidth() == 400  # NuPIC's RDSE default n
    cfg = rt.network.engine_config(enc, dict(YAML_SP, inputWidth=400), YAML_TM)
    want = rt._lib.model_yaml_config()
    assert cfg.as_dict() == want.as_dict()
    with pytest.raises(ValueError):
        rt.network.engine_config(enc, YAML_SP, YAML_TM)  # 946 != the encoder's 400 bits
    with pytest.raises(ValueError):
        rt.network.RandomDistributedScalarEncoder(0.88, offset=50.0)  # fixed offsets are not supported


@pytest.mark.gpu
def test_yaml_network_through_the_facade_matches_the_oracle(rt, oracle_mod, traces):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    ds = rt.BatchRecordStream(["cpu_metric"])
    net = yaml_network(rt, ds, seg_capacity=1 << 14)
    orc = oracle_mod.OracleModel(oracle_mod.model_yaml_params())
    for k, cpu in enumerate(traces["train"][:160]):
        learn = k < 120
        if k == 120:
            net.regions["tm"].setParameter("learningMode", False)  # NetworkModel.py:40-44
        ds.setData(float(cpu))
        net.run(1)
        got = net.regions["tm"].getOutputData("anomalyScore")[0]
        assert got == orc.step([cpu], True, learn), f"record {k}"
        assert net.regions["sensor"].getOutputData("bucketIdxOut")[0] == orc.bucket()
