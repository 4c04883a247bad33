"""The reference's Model-1 graph construction (ML/HTM/NetworkModel.py:48-110,
ML/HTM/NetworkUtils.py:25-64,77-153), written against the batched facade
exactly as the reference writes it against nupic.engine -- the drop-in
check.  Parameter dicts restate NetworkUtils.py:26-64."""
import json

_SEED = 2045
SP_PARAMS = {"spVerbosity": 0, "spatialImp": "cpp", "seed": _SEED, "inputWidth": 0, "globalInhibition": 1,
             "columnCount": 2048, "numActiveColumnsPerInhArea": 40, "potentialPct": 0.8,
             "synPermConnected": 0.1, "synPermActiveInc": 0.0001, "synPermInactiveDec": 0.0005,
             "boostStrength": 0.0}
TM_PARAMS = {"verbosity": 0, "temporalImp": "cpp", "seed": _SEED, "columnCount": 2048, "cellsPerColumn": 12,
             "inputWidth": 2048, "newSynapseCount": 20, "maxSynapsesPerSegment": 32, "maxSegmentsPerCell": 128,
             "initialPerm": 0.21, "permanenceInc": 0.1, "permanenceDec": 0.1, "globalDecay": 0.0, "maxAge": 0,
             "minThreshold": 9, "activationThreshold": 12, "outputType": "normal", "pamLength": 3}
SENSOR, SPR, TMR, CLS = "sensorRegion", "l1SpatialPoolerRegion", "l1TemporalMemoryRegion", "l1Classifier"


def create_encoder(rt, multilevel=False):
    enc = rt.MultiEncoder()
    spec = {"cpu": {"fieldname": "cpu", "type": "ScalarEncoder", "name": "cpu", "minval": 0.0, "maxval": 100.0,
                    "clipInput": True, "w": 21, "n": 500}}
    if multilevel:
        spec["mem"] = dict(spec["cpu"], fieldname="mem", name="mem")
    enc.addMultipleEncoders(spec)
    return enc


def create_one_level_network(rt, data_source, n_streams=1, multilevel=False, **engine_opts):
    network = rt.Network(n_streams=n_streams, **engine_opts)
    network.addRegion(SENSOR, "py.RecordSensor", json.dumps({"verbosity": 0}))
    sensor = network.regions[SENSOR].getSelf()
    sensor.encoder = create_encoder(rt, multilevel)
    network.regions[SENSOR].setParameter("predictedField", "cpu")
    sensor.dataSource = data_source
    sp = dict(SP_PARAMS, inputWidth=sensor.encoder.getWidth())
    spr = network.addRegion(SPR, "py.SPRegion", json.dumps(sp))
    spr.setParameter("learningMode", True)
    spr.setParameter("anomalyMode", False)
    network.link(SENSOR, SPR, "UniformLink", "")
    tm = network.addRegion(TMR, "py.TMRegion", json.dumps(TM_PARAMS))
    tm.setParameter("topDownMode", True)
    tm.setParameter("learningMode", True)
    tm.setParameter("inferenceMode", True)
    tm.setParameter("anomalyMode", True)
    network.link(SPR, TMR, "UniformLink", "")
    cls = network.addRegion(CLS, "py.SDRClassifierRegion",
                            json.dumps({"alpha": 0.005, "steps": "1,2,3,4,5,6,7", "implementation": "py",
                                        "verbosity": 0}))
    cls.setParameter("inferenceMode", True)
    cls.setParameter("learningMode", True)
    network.link(TMR, CLS, "UniformLink", "", srcOutput="bottomUpOut", destInput="bottomUpIn")
    network.link(SENSOR, CLS, "UniformLink", "", srcOutput="categoryOut", destInput="categoryIn")
    return network


L2_SPR, L2_TMR, L2_CLS = "l2SpatialPoolerRegion", "l2TemporalMemoryRegion", "l2Classifier"
CLS_PARAMS = {"alpha": 0.005, "steps": "1,2,3,4,5,6,7", "implementation": "py", "verbosity": 0}


def _add_sp(network, name, width):
    spr = network.addRegion(name, "py.SPRegion", json.dumps(dict(SP_PARAMS, inputWidth=width)))
    spr.setParameter("learningMode", True)
    spr.setParameter("anomalyMode", False)
    return spr


def _add_tm(network, name):
    tm = network.addRegion(name, "py.TMRegion", json.dumps(TM_PARAMS))
    for k in ("topDownMode", "learningMode", "inferenceMode", "anomalyMode"):
        tm.setParameter(k, True)
    return tm


def _add_classifier(network, name, tm_name):
    cls = network.addRegion(name, "py.SDRClassifierRegion", json.dumps(CLS_PARAMS))
    cls.setParameter("inferenceMode", True)
    cls.setParameter("learningMode", True)
    network.link(tm_name, name, "UniformLink", "", srcOutput="bottomUpOut", destInput="bottomUpIn")
    for out, inp in (("categoryOut", "categoryIn"), ("bucketIdxOut", "bucketIdxIn"), ("actValueOut", "actValueIn")):
        network.link(SENSOR, name, "UniformLink", "", srcOutput=out, destInput=inp)


def create_multilevel_network(rt, data_source, n_streams=1, anomaly=False, **engine_opts):
    """Model 2 (ML/HTM/MultiLevelNetworkModel.py:53-127: cpu encoder, L2
    classifier, L2 TM topDownOut -> L1 SP topDownIn feedback) or, with
    anomaly=True, Model 3 (MultiLevelNetworkAnomaly.py:61-127: cpu+mem encoder,
    L1 and L2 classifiers)."""
    network = rt.Network(n_streams=n_streams, **engine_opts)
    network.addRegion(SENSOR, "py.RecordSensor", json.dumps({"verbosity": 0}))
    sensor = network.regions[SENSOR].getSelf()
    sensor.encoder = create_encoder(rt, anomaly)
    network.regions[SENSOR].setParameter("predictedField", "cpu")
    sensor.dataSource = data_source
    _add_sp(network, SPR, sensor.encoder.getWidth())
    network.link(SENSOR, SPR, "UniformLink", "")
    l1 = _add_tm(network, TMR)
    network.link(SPR, TMR, "UniformLink", "")
    if anomaly:
        _add_classifier(network, CLS, TMR)
    # second level: inputWidth = the L1 TMRegion's bottomUpOut element count
    width = TM_PARAMS["columnCount"] * TM_PARAMS["cellsPerColumn"]
    _add_sp(network, L2_SPR, width)
    network.link(TMR, L2_SPR, "UniformLink", "")
    _add_tm(network, L2_TMR)
    network.link(L2_SPR, L2_TMR, "UniformLink", "")
    _add_classifier(network, L2_CLS, L2_TMR)
    if not anomaly:
        network.link(L2_TMR, SPR, "UniformLink", "", srcOutput="topDownOut", destInput="topDownIn")
    assert l1 is network.regions[TMR]
    return network
