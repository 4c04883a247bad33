"""Drop-in batched counterpart of the NuPIC network surface the reference uses.

The reference builds one `nupic.engine.Network` per model and drives it one
record at a time (ML/HTM/NetworkModel.py:48-157, NetworkUtils.py:111-163):

    network = Network()
    network.addRegion("sensorRegion", "py.RecordSensor", json.dumps({...}))
    network.regions["sensorRegion"].getSelf().encoder = createEncoder()
    network.addRegion("l1SpatialPoolerRegion", "py.SPRegion", json.dumps(SP_PARAMS))
    network.link("sensorRegion", "l1SpatialPoolerRegion", "UniformLink", "")
    ...
    dataSource.setData(cpu)                          # StreamReader.py:157-161
    network.run(1)                                   # NetworkModel.py:127
    score = network.regions[TM].getOutputData("anomalyScore")[0]   # :133
    network.save("network1.nta"); Network("network1.nta")          # NetworkUtils.py:156-163

This module keeps exactly that call pattern, but one `Network` steps
`n_streams` independent copies of the graph in lockstep on one MI355X through
the HIP engine (`HTMEngine`, include/htm_amd.h).  Every output is batched
along a leading stream axis; element 0 is stream 0, so single-stream code
that indexes `[0]` keeps working unchanged.

Scope: RecordSensor (ScalarEncoder / MultiEncoder),
SPRegion and TMRegion are executed by the engine; an SDRClassifierRegion
(NetworkModel.py:70-97) runs on the GPU too (classifier.py, csrc/classifier.hip),
fed TM bottomUpOut and the sensor's bucket/actual value of the first encoder
field, its actualValues / probabilities outputs shaped like the region's
([maxCategoryCount], [steps * maxCategoryCount]; with a leading stream axis
when n_streams > 1).
Errors follow the NuPIC convention of raising (NTA_THROW -> RuntimeError /
ValueError); there is no CPU fallback -- creating the engine fails loudly if
the HIP library or a GPU is missing.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np

from . import _lib

SENSOR, SP, TM, CLASSIFIER = "py.RecordSensor", "py.SPRegion", "py.TMRegion", "py.SDRClassifierRegion"
_ENGINE_FILE = "engine.htm"
_CLS_FILE = "classifier.npz"
_META_FILE = "network.json"


# ---------------------------------------------------------------- encoders
class ScalarEncoder:
    """nupic.encoders.ScalarEncoder parameters (non-periodic, as the reference
    configures it: NetworkUtils.py:80-88).  Encoding itself runs on the GPU
    (sp.hip enc_first_on_bit); the host side only answers bucket queries for
    the sensor's bucketIdxOut output."""

    def __init__(self, w, minval, maxval, n=0, clipInput=False, name=None, fieldname=None, periodic=False,
                 radius=0, resolution=0, forced=False, verbosity=0):
        if periodic:
            raise ValueError("periodic ScalarEncoder is not supported")
        if radius or resolution:
            raise ValueError("ScalarEncoder: only the n/w form used by the reference is supported")
        if n <= w:
            raise ValueError("ScalarEncoder: n must be > w")
        if maxval <= minval:
            raise ValueError("ScalarEncoder: maxval must be > minval")
        self.w, self.n = int(w), int(n)
        self.minval, self.maxval = float(minval), float(maxval)
        self.clipInput = bool(clipInput)
        self.name = name if name is not None else "[%s:%s]" % (minval, maxval)
        self.fieldname = fieldname if fieldname is not None else self.name
        self.resolution = (self.maxval - self.minval) / float(self.n - self.w)
        self.halfwidth = (self.w - 1) // 2

    def getWidth(self):
        return self.n

    def getBucketIndices(self, x):
        """[minbin] or [None] for a missing value (ScalarEncoder._getFirstOnBit)."""
        if x is None or (isinstance(x, float) and math.isnan(x)):
            return [None]
        x = float(x)
        if x < self.minval:
            if not self.clipInput:
                raise ValueError("input %s less than minval %s" % (x, self.minval))
            x = self.minval
        if x > self.maxval:
            if not self.clipInput:
                raise ValueError("input %s greater than maxval %s" % (x, self.maxval))
            x = self.maxval
        centerbin = int((x - self.minval + self.resolution / 2.0) / self.resolution) + self.halfwidth
        return [centerbin - self.halfwidth]

    def bucket_indices(self, xs: np.ndarray) -> np.ndarray:
        """Vectorised getBucketIndices over a batch (missing -> -1)."""
        x = np.asarray(xs, dtype=np.float64)
        miss = np.isnan(x)
        if not self.clipInput and np.any(~miss & ((x < self.minval) | (x > self.maxval))):
            raise ValueError("input outside [minval, maxval] with clipInput False")
        xc = np.clip(np.where(miss, self.minval, x), self.minval, self.maxval)
        b = ((xc - self.minval + self.resolution / 2.0) / self.resolution).astype(np.int64)
        return np.where(miss, -1, b)


class RandomDistributedScalarEncoder:
    """nupic.encoders.RandomDistributedScalarEncoder parameters -- the encoder
    of the reference's model.yaml (ML/HTM/params/model.yaml:15-21).  Encoding
    runs on the GPU (sp.hip rdse_encode_kernel, per-stream bucket maps and
    offsets); bucket queries read the engine's HTM_OUT_BUCKETS output."""

    MAX_BUCKETS = _lib.RDSE_BUCKETS

    def __init__(self, resolution, w=21, n=400, name=None, offset=None, seed=42, verbosity=0, fieldname=None):
        if w <= 0 or w % 2 == 0:
            raise ValueError("w must be an odd positive integer")
        if resolution <= 0:
            raise ValueError("resolution must be a positive number")
        if n <= 6 * w:
            raise ValueError("n must be an int strictly greater than 6*w")
        if offset is not None:
            raise ValueError("RDSE offset: only None (the first value encoded) is supported")
        self.w, self.n, self.resolution, self.seed = int(w), int(n), float(resolution), int(seed)
        self.name = name if name is not None else "[%s]" % self.resolution
        self.fieldname = fieldname if fieldname is not None else self.name
        self.clipInput = True

    def getWidth(self):
        return self.n


class MultiEncoder:
    """nupic.encoders.MultiEncoder: sub-encoders concatenated in sorted field
    name order (NetworkUtils.py:77-108)."""

    def __init__(self, encoderDefinitions=None):
        self.encoders = {}
        if encoderDefinitions:
            self.addMultipleEncoders(encoderDefinitions)

    def addEncoder(self, name, encoder):
        self.encoders[name] = encoder

    def addMultipleEncoders(self, fieldEncodings):
        for key in sorted(fieldEncodings):
            spec = dict(fieldEncodings[key])
            kind = spec.pop("type", "ScalarEncoder")
            cls = {"ScalarEncoder": ScalarEncoder, "RandomDistributedScalarEncoder": RandomDistributedScalarEncoder}
            if kind not in cls:
                raise ValueError("encoder type %s is not supported (ScalarEncoder, RandomDistributedScalarEncoder)" % kind)
            fieldname = spec.pop("fieldname", key)
            name = spec.pop("name", key)
            self.addEncoder(key, cls[kind](name=name, fieldname=fieldname, **spec))

    def fields(self):
        return [self.encoders[k] for k in sorted(self.encoders)]

    def getWidth(self):
        return sum(e.getWidth() for e in self.fields())


# ----------------------------------------------------------- data source
class BatchRecordStream:
    """Batched stand-in for the reference's kafkaRecordStream
    (ML/HTM/StreamReader.py:64-230).  The reference hands one value per field
    to the sensor through module globals (setData :157-161, grabStreamData
    :179-188); here each network owns its stream object and `setData` takes
    one value (or an array of n_streams values) per field.  None / NaN are
    missing values (SENTINEL_VALUE_FOR_MISSING_DATA -> all-zero SDR)."""

    def __init__(self, names=("cpu",), n_streams=1):
        self.names = list(names)
        self.n_streams = int(n_streams)
        self._values = None
        self._recordCount = 0

    def setData(self, dataRec, memRec=None):
        fields = [dataRec] if memRec is None else [dataRec, memRec]
        cols = []
        for f in fields:
            if isinstance(f, np.ndarray) and f.dtype.kind in "fiu":
                a = f.astype(np.float64).ravel()
            else:
                a = np.asarray([np.nan if f is None else f] if np.ndim(f) == 0 else f, dtype=object)
                a = np.array([np.nan if v is None else float(v) for v in a.ravel()], dtype=np.float64)
            if a.size == 1 and self.n_streams > 1:
                a = np.full(self.n_streams, a[0])
            if a.size != self.n_streams:
                raise ValueError("setData: expected %d values per field, got %d" % (self.n_streams, a.size))
            cols.append(a)
        self._values = np.stack(cols, axis=1)  # [n_streams, fields]

    def getNextRecord(self):
        if self._values is None:
            raise RuntimeError("no data: call setData() before network.run()")
        self._recordCount += 1
        return self._values

    def rewind(self):
        self._recordCount = 0

    def getNextRecordIdx(self):
        return self._recordCount


# ------------------------------------------------------------------ regions
class _RegionImpl:
    """getSelf() object of a region (holds parameters and host attributes)."""

    def __init__(self, params):
        self.params = dict(params)


class _SensorImpl(_RegionImpl):
    def __init__(self, params):
        super().__init__(params)
        self.encoder = None
        self.dataSource = None
        self.predictedField = None
        self.values = None  # [n_streams, fields] of the last run


class _ClassifierImpl(_RegionImpl):
    def __init__(self, params):
        super().__init__(params)
        steps = str(params.get("steps", "1"))
        self.stepsList = [int(x) for x in steps.split(",") if x.strip()]
        self.maxCategoryCount = int(params.get("maxCategoryCount", 1000))  # SDRClassifierRegion default
        self.alpha = float(params.get("alpha", 0.001))
        if params.get("implementation", "py") not in ("py", "cpp"):
            raise ValueError("SDRClassifier implementation %r is not supported" % params.get("implementation"))
        self.classifier = None  # classifier.SDRClassifier, built with the engine
        self.recordNum = 0
        self.actualValues = None
        self.probabilities = None


class Region:
    """network.regions[name]: setParameter / getParameter / getOutputData /
    getSelf, as the reference calls them (NetworkUtils.py:116-152,
    NetworkModel.py:41-44,129-133)."""

    _MODES = {
        SENSOR: {"predictedField", "verbosity"},
        SP: {"learningMode", "inferenceMode", "anomalyMode", "topDownMode"},
        TM: {"learningMode", "inferenceMode", "anomalyMode", "topDownMode"},
        CLASSIFIER: {"learningMode", "inferenceMode"},
    }

    def __init__(self, network, name, node_type, params):
        self.network = network
        self.name = name
        self.type = node_type
        self.modes = {"learningMode": True, "inferenceMode": True, "anomalyMode": False, "topDownMode": False}
        self._impl = {SENSOR: _SensorImpl, CLASSIFIER: _ClassifierImpl}.get(node_type, _RegionImpl)(params)

    def getSelf(self):
        return self._impl

    @property
    def dataSource(self):
        """Sensor regions: the RecordSensor's data source.  ModelTesting.initModels
        re-attaches it on the loaded network with
        `network.regions[_RECORD_SENSOR].dataSource = ds` (ModelTesting.py:176-178)."""
        if self.type != SENSOR:
            raise AttributeError("region %s (%s) has no dataSource" % (self.name, self.type))
        return self._impl.dataSource

    @dataSource.setter
    def dataSource(self, ds):
        if self.type != SENSOR:
            raise AttributeError("region %s (%s) has no dataSource" % (self.name, self.type))
        self._impl.dataSource = ds

    def setParameter(self, name, value):
        if name not in self._MODES[self.type]:
            raise ValueError("region %s (%s) has no settable parameter %r" % (self.name, self.type, name))
        if self.type == SENSOR:
            setattr(self._impl, name, value)
            return
        if self.type == TM and name == "inferenceMode" and not value:
            raise ValueError("TMRegion inferenceMode False is not supported (the anomaly score needs inference)")
        self.modes[name] = bool(value)
        if name == "learningMode":
            self.network._learning_changed()

    def getParameter(self, name):
        if self.type == SENSOR:
            return getattr(self._impl, name)
        if name in self.modes:
            return self.modes[name]
        return self._impl.params[name]

    def getOutputData(self, name):
        return self.network._output(self, name)


# ------------------------------------------------------------------ network
# reference parameter names -> htm_config fields (NetworkUtils.py:26-64)
_SP_MAP = {"columnCount": "sp_columns", "numActiveColumnsPerInhArea": "sp_num_active",
           "potentialPct": "sp_potential_pct", "synPermConnected": "sp_perm_connected",
           "synPermActiveInc": "sp_perm_active_inc", "synPermInactiveDec": "sp_perm_inactive_dec",
           "minPctOverlapDutyCycle": "sp_min_pct_overlap_dc", "dutyCyclePeriod": "sp_duty_cycle_period",
           "boostStrength": "sp_boost_strength", "stimulusThreshold": "sp_stimulus_threshold", "seed": "sp_seed"}
_TM_MAP = {"cellsPerColumn": "tm_cells_per_col", "newSynapseCount": "tm_new_syn_count",
           "maxSynapsesPerSegment": "tm_max_syn_per_seg", "maxSegmentsPerCell": "tm_max_segs_per_cell",
           "initialPerm": "tm_initial_perm", "connectedPerm": "tm_connected_perm",
           "permanenceInc": "tm_perm_inc", "permanenceDec": "tm_perm_dec", "permanenceMax": "tm_perm_max",
           "minThreshold": "tm_min_threshold", "activationThreshold": "tm_activation_threshold",
           "pamLength": "tm_pam_length", "maxInfBacktrack": "tm_max_inf_backtrack",
           "maxLrnBacktrack": "tm_max_lrn_backtrack", "maxSeqLength": "tm_max_seq_length",
           "segUpdateValidDuration": "tm_seg_update_valid_duration", "seed": "tm_seed"}
# parameters accepted only at the value the engine implements
_SP_FIXED = {"globalInhibition": 1, "spatialImp": "cpp", "localAreaDensity": -1.0, "wrapAround": True}
_TM_FIXED = {"globalDecay": 0.0, "maxAge": 0, "outputType": "normal", "temporalImp": "cpp", "doPooling": False,
             "burnIn": 2, "collectStats": False}
_IGNORED = {"spVerbosity", "verbosity", "inputWidth", "columnCount", "potentialRadius", "spatialImp",
            "temporalImp"}


def engine_config(sensor_enc: MultiEncoder | None, sp_params: dict, tm_params: dict, input_width: int = 0,
                  **engine_opts):
    """Translate the reference's region parameter dicts into an htm_config
    (raises ValueError for anything the engine does not implement).  With
    sensor_enc None the SP reads an input SDR of input_width bits (a second
    level, fed the TMRegion bottomUpOut below it: MultiLevelNetworkModel.py:92-94)."""
    if sensor_enc is not None:
        fields = sensor_enc.fields()
        if not fields:
            raise ValueError("the sensor has no encoder (NetworkUtils.createEncoder)")
        e0 = fields[0]
        if len(fields) > 4:
            raise ValueError("at most 4 encoder fields (got %d)" % len(fields))
        for e in fields[1:]:
            if (type(e), e.n, e.w, e.clipInput) != (type(e0), e0.n, e0.w, e0.clipInput):
                raise ValueError("all encoder fields must share the encoder type and n/w/clipInput")
        if isinstance(e0, RandomDistributedScalarEncoder):
            if any((e.resolution, e.seed) != (e0.resolution, e0.seed) for e in fields[1:]):
                raise ValueError("all RDSE fields must share resolution and seed")
            over = dict(n_fields=len(fields), enc_n=e0.n, enc_w=e0.w, enc_type=_lib.ENC_RDSE,
                        rdse_resolution=e0.resolution, rdse_seed=e0.seed)
        else:
            over = dict(n_fields=len(fields), enc_n=e0.n, enc_w=e0.w, enc_minval=e0.minval, enc_maxval=e0.maxval,
                        enc_clip=int(e0.clipInput))
        if not isinstance(e0, RandomDistributedScalarEncoder) and \
                any((e.minval, e.maxval) != (e0.minval, e0.maxval) for e in fields[1:]):
            # per-field ranges (e.g. cpu/mem % next to response times in ms)
            pad = [0.0] * (4 - len(fields))
            over["field_minval"] = tuple([float(e.minval) for e in fields] + pad)
            over["field_maxval"] = tuple([float(e.maxval) for e in fields] + pad)
        width = sensor_enc.getWidth()
    else:
        over = dict(sdr_bits=int(input_width))
        width = int(input_width)
    for params, mapping, fixed, region in ((sp_params, _SP_MAP, _SP_FIXED, "SPRegion"),
                                           (tm_params, _TM_MAP, _TM_FIXED, "TMRegion")):
        for k, v in params.items():
            if k in mapping:
                over[mapping[k]] = v
            elif k in fixed:
                if v != fixed[k] and not (isinstance(v, (int, float)) and float(v) == float(fixed[k])):
                    raise ValueError("%s %s=%r is not supported (only %r)" % (region, k, v, fixed[k]))
            elif k not in _IGNORED:
                raise ValueError("%s parameter %r is not supported" % (region, k))
    if int(sp_params.get("inputWidth", 0) or width) != width:
        raise ValueError("SPRegion inputWidth %s != the width of its input (%d)" % (sp_params.get("inputWidth"), width))
    cols = int(sp_params.get("columnCount", 2048))
    if int(tm_params.get("columnCount", cols)) != cols or int(tm_params.get("inputWidth", cols)) != cols:
        raise ValueError("TMRegion columnCount/inputWidth must equal the SP columnCount")
    over.update(engine_opts)
    return _lib.default_config(**over)


class _Level:
    """One SPRegion -> TMRegion level of the graph and the engine that runs it
    for every stream (level 0 reads the sensor, level k > 0 the bottomUpOut of
    level k - 1)."""

    def __init__(self, sp: Region, tm: Region):
        self.sp, self.tm = sp, tm
        self.engine = None
        self.scores = None


class Network:
    """Batched nupic.engine.Network: `Network()` builds an empty graph,
    `Network(path)` loads a saved one (ModelTesting.py:176).

    Graphs: RecordSensor -> SPRegion -> TMRegion, optionally followed by more
    SPRegion -> TMRegion levels each fed the TMRegion bottomUpOut below it (the
    two-level Models 2/3, MultiLevelNetworkModel.py:53-127,
    MultiLevelNetworkAnomaly.py:61-127), and SDRClassifierRegions fed any
    level's TMRegion bottomUpOut.  The Model-2 feedback link (L2 TMRegion
    topDownOut -> L1 SPRegion topDownIn, MultiLevelNetworkModel.py:113-114) is
    accepted and has no effect: an SPRegion reads topDownIn only in topDownMode,
    which NetworkUtils never enables for an SPRegion (NetworkUtils.py:126-136),
    so the reference's bottom-up results do not depend on it either."""

    def __init__(self, path: str | None = None, n_streams: int = 1, device: int | None = None, **engine_opts):
        self.regions = {}
        self.links = []
        self.n_streams = int(n_streams)
        self.device = device
        self.engine_opts = dict(engine_opts)
        self.levels: list[_Level] = []
        self._cls_level = {}  # classifier region name -> level index
        self._learn_dirty = False
        if path is not None:
            self._load(path)

    @property
    def engine(self):
        """The first level's engine (the only one of a Model-1 graph)."""
        return self.levels[0].engine if self.levels else None

    # ------------------------------------------------------------ building
    def addRegion(self, name, nodeType, nodeParams="{}"):
        if self.levels:
            raise RuntimeError("cannot add regions after the network is initialized")
        if name in self.regions:
            raise ValueError("region %r already exists" % name)
        if nodeType not in (SENSOR, SP, TM, CLASSIFIER):
            raise ValueError("region type %r is not supported by the MI355X engine" % nodeType)
        params = json.loads(nodeParams) if isinstance(nodeParams, str) else dict(nodeParams or {})
        r = Region(self, name, nodeType, params)
        self.regions[name] = r
        return r

    def link(self, srcName, destName, linkType="UniformLink", linkParams="", srcOutput=None, destInput=None):
        for n in (srcName, destName):
            if n not in self.regions:
                raise ValueError("unknown region %r" % n)
        if linkType != "UniformLink":
            raise ValueError("link type %r is not supported" % linkType)
        self.links.append((srcName, destName, srcOutput or "bottomUpOut", destInput or "bottomUpIn"))

    def _find(self, kind):
        rs = [r for r in self.regions.values() if r.type == kind]
        if len(rs) != 1:
            raise RuntimeError("the engine runs exactly one %s per network (found %d)" % (kind, len(rs)))
        return rs[0]

    def _feed(self):
        """bottom-up links (src, dest): bottomUpOut/dataOut -> bottomUpIn"""
        return {(s, d) for s, d, so, di in self.links if di == "bottomUpIn" or so in ("bottomUpOut", "dataOut")}

    def _chain(self):
        """The sensor and its SPRegion -> TMRegion levels in bottom-up order."""
        sensor = self._find(SENSOR)
        feed = self._feed()
        levels, src = [], sensor.name
        while True:
            sps = [r for r in self.regions.values() if r.type == SP and (src, r.name) in feed]
            if not sps:
                break
            if len(sps) > 1:
                raise RuntimeError("%s feeds %d SPRegions; the engine runs one chain" % (src, len(sps)))
            tms = [r for r in self.regions.values() if r.type == TM and (sps[0].name, r.name) in feed]
            if len(tms) != 1:
                raise RuntimeError("SPRegion %s must feed exactly one TMRegion (NetworkModel.py:67)" % sps[0].name)
            if any(lv.sp is sps[0] for lv in levels):
                raise RuntimeError("the SPRegion -> TMRegion chain has a cycle")
            levels.append(_Level(sps[0], tms[0]))
            src = tms[0].name
        if not levels:
            raise RuntimeError("the graph must link sensor -> SPRegion -> TMRegion (NetworkModel.py:61,67)")
        on_chain = {lv.sp.name for lv in levels} | {lv.tm.name for lv in levels}
        for r in self.regions.values():
            if r.type in (SP, TM) and r.name not in on_chain:
                raise RuntimeError("region %s is not on the sensor -> SPRegion -> TMRegion chain" % r.name)
        cls_level = {}
        for r in self.regions.values():
            if r.type == CLASSIFIER:
                src_lv = [k for k, lv in enumerate(levels) if (lv.tm.name, r.name) in feed]
                if len(src_lv) != 1:
                    raise RuntimeError("SDRClassifierRegion %s must be fed one TMRegion bottomUpOut" % r.name)
                cls_level[r.name] = src_lv[0]
        return sensor, levels, cls_level

    def _sensor_encoder(self, sensor):
        enc = sensor.getSelf().encoder
        if enc is None:
            raise RuntimeError("sensor %r has no encoder" % sensor.name)
        if isinstance(enc, (ScalarEncoder, RandomDistributedScalarEncoder)):
            m = MultiEncoder()
            m.addEncoder(enc.name, enc)
            enc = m
        return enc

    def initialize(self):
        if self.levels:
            return
        from .engine import HTMEngine
        sensor, levels, cls_level = self._chain()
        enc = self._sensor_encoder(sensor)
        try:
            for k, lv in enumerate(levels):
                if k == 0:
                    cfg = engine_config(enc, lv.sp.getSelf().params, lv.tm.getSelf().params, **self.engine_opts)
                else:
                    width = levels[k - 1].engine.n_cells  # TMRegion bottomUpOut element count
                    cfg = engine_config(None, lv.sp.getSelf().params, lv.tm.getSelf().params, input_width=width,
                                        **self.engine_opts)
                lv.engine = HTMEngine(self.n_streams, config=cfg, device=self.device)
        except Exception:
            for lv in levels:
                if lv.engine is not None:
                    lv.engine.close()
            raise
        self.levels, self._cls_level = levels, cls_level
        for name in cls_level:
            self._init_classifier(self.regions[name])
        self._learning_changed()

    def _level_of(self, region):
        for lv in self.levels:
            if region is lv.sp or region is lv.tm:
                return lv
        raise RuntimeError("region %s is not on the engine's chain" % region.name)

    def _first_field(self):
        enc = self._find(SENSOR).getSelf().encoder
        return enc.fields()[0] if isinstance(enc, MultiEncoder) else enc

    def _init_classifier(self, r, cls_obj=None):
        from .classifier import SDRClassifier
        impl = r.getSelf()
        f0 = self._first_field()
        # ScalarEncoder buckets (clipped, non-periodic); the RDSE's maxBuckets
        nb = f0.MAX_BUCKETS if isinstance(f0, RandomDistributedScalarEncoder) else f0.n - f0.w + 1
        if impl.maxCategoryCount < nb:
            raise ValueError("maxCategoryCount %d < %d encoder buckets" % (impl.maxCategoryCount, nb))
        eng = self.levels[self._cls_level[r.name]].engine
        impl.classifier = cls_obj if cls_obj is not None else SDRClassifier(
            self.n_streams, eng.n_cells, nb, steps=impl.stepsList, alpha=impl.alpha, device=eng.device)
        impl.actualValues = np.zeros((self.n_streams, impl.maxCategoryCount))
        impl.probabilities = np.zeros((self.n_streams, len(impl.stepsList) * impl.maxCategoryCount))

    def _run_classifiers(self, vals):
        """SDRClassifierRegion.compute of every stream after the TM steps: its
        level's TM bottomUpOut, bucketIdxOut / actValueOut of the first encoder
        field (a missing value does not learn)."""
        f0 = None
        for name, k in self._cls_level.items():
            r = self.regions[name]
            impl = r.getSelf()
            learn, infer = r.modes["learningMode"], r.modes["inferenceMode"]
            f0 = f0 or self._first_field()
            pat = self.levels[k].engine.get_output("tm_output")
            if not learn:
                bucket = None
            elif isinstance(f0, RandomDistributedScalarEncoder):  # the GPU encoder's bucketIdxOut
                bucket = self.levels[0].engine.get_output("buckets")[:, 0].cpu().numpy().astype(np.int64)
            else:
                bucket = f0.bucket_indices(vals[:, 0])
            prob, act = impl.classifier.compute(pat, bucket, vals[:, 0] if learn else None, learn=learn, infer=infer)
            impl.classifier.status()  # raises like NuPIC on an empty pattern (this record only)
            impl.recordNum += 1
            if infer:
                nb, n = impl.classifier.n_buckets, impl.maxCategoryCount
                impl.actualValues[:, :nb] = act.cpu().numpy()
                p = prob.cpu().numpy()
                for i in range(len(impl.stepsList)):
                    impl.probabilities[:, i * n:i * n + nb] = p[:, i]

    def _learning_changed(self):
        self._learn_dirty = True

    def _apply_learning(self):
        if self._learn_dirty and self.levels:
            for lv in self.levels:
                lv.engine.set_learning(lv.sp.modes["learningMode"], lv.tm.modes["learningMode"])
            self._learn_dirty = False

    # ------------------------------------------------------------- running
    def run(self, n):
        """network.run(n): n lockstep steps of every stream (NetworkModel.py:127).
        Each step pulls one record (a value per stream and field) from the
        sensor's data source, like RecordSensor.compute does, and runs the
        levels bottom-up (the links carry no delay)."""
        self.initialize()
        self._apply_learning()
        import torch
        sensor = self._find(SENSOR).getSelf()
        if sensor.dataSource is None:
            raise RuntimeError("sensor has no dataSource")
        l0 = self.levels[0]
        for _ in range(int(n)):
            vals = np.asarray(sensor.dataSource.getNextRecord(), dtype=np.float64)
            if vals.shape != (self.n_streams, l0.engine.n_fields):
                raise ValueError("record shape %s != (%d streams, %d fields)" %
                                 (vals.shape, self.n_streams, l0.engine.n_fields))
            sensor.values = vals
            l0.scores = l0.engine.step(torch.from_numpy(np.ascontiguousarray(vals).ravel()))
            for below, lv in zip(self.levels, self.levels[1:]):
                lv.scores = lv.engine.step_sdr(below.engine.get_output("tm_output"))
            self._run_classifiers(vals)
        # NuPIC raises (NTA_THROW) when a Cells4 pool limit is hit; the engine
        # records the overflow per stream -- surface it the same way
        for lv in self.levels:
            lv.engine.status()

    def _output(self, region, name):
        if not self.levels:
            raise RuntimeError("network has not run yet")
        if region.type == SENSOR:
            vals = region.getSelf().values
            if vals is None:
                raise RuntimeError("network has not run yet")
            if name == "actValueOut":
                return vals[:, 0].astype(np.float64)
            if name == "bucketIdxOut":
                f0 = self._first_field()
                if isinstance(f0, RandomDistributedScalarEncoder):  # the GPU encoder's state
                    return self.levels[0].engine.get_output("buckets")[:, 0].cpu().numpy().astype(np.float64)
                return f0.bucket_indices(vals[:, 0]).astype(np.float64)
            if name == "sourceOut":
                return vals.copy()
        elif region.type == SP:
            eng = self._level_of(region).engine
            if name == "bottomUpOut":
                return eng.get_output("active_columns").cpu().numpy().astype(np.float32)
        elif region.type == TM:
            lv = self._level_of(region)
            eng = lv.engine
            if name == "anomalyScore":
                if not region.modes["anomalyMode"]:
                    raise RuntimeError("anomalyScore needs anomalyMode True (NetworkUtils.py:152)")
                if lv.scores is None:
                    raise RuntimeError("network has not run yet")
                return lv.scores.cpu().numpy()
            if name == "bottomUpOut":
                return eng.bitmap_to_dense(eng.get_output("tm_output")).astype(np.float32)
            if name == "topDownOut":
                return eng.get_output("col_confidence").cpu().numpy()
            if name in ("activeCells", "lrnActiveStateT"):
                return eng.bitmap_to_dense(eng.get_output("inf_active" if name == "activeCells" else "lrn_active"))
            if name == "predictedActiveCells":
                a = eng.bitmap_to_dense(eng.get_output("inf_active"))
                return a & eng.bitmap_to_dense(eng.get_output("inf_predicted"))
        elif region.type == CLASSIFIER:
            impl = region.getSelf()
            one = (lambda a: a[0]) if self.n_streams == 1 else (lambda a: a)
            if name == "actualValues":
                return one(impl.actualValues.copy())
            if name == "probabilities":
                return one(impl.probabilities.copy())
            if name == "categoriesOut":
                n = impl.maxCategoryCount
                out = np.stack([impl.actualValues[np.arange(self.n_streams),
                                                  impl.probabilities[:, i * n:(i + 1) * n].argmax(axis=1)]
                                for i in range(len(impl.stepsList))], axis=1)
                return one(out)
        raise ValueError("region %s (%s) has no output %r" % (region.name, region.type, name))

    def scores_tensor(self, level: int = -1):
        """Device tensor of the last step's anomaly scores of a level (default:
        the top one, whose TMRegion anomalyScore the two-level models report,
        MultiLevelNetworkModel.py:150) -- no host copy."""
        return self.levels[level].scores if self.levels else None

    # ----------------------------------------------------------- save/load
    @staticmethod
    def _engine_file(k):
        return _ENGINE_FILE if k == 0 else "engine_l%d.htm" % (k + 1)

    @staticmethod
    def _cls_file(name, first):
        return _CLS_FILE if first else "classifier_%s.npz" % name

    def save(self, path):
        """network.save(path) (NetworkUtils.py:156-159): a bundle directory like
        NuPIC's .nta -- network.json (regions, parameters, links, modes) plus
        one engine file per level (every stream's SP/TM state, htm_save:
        engine.htm, engine_l2.htm, ...) and the classifiers' state."""
        self.initialize()
        self._apply_learning()
        for lv in self.levels:
            lv.engine.status()  # never save a state whose pools overflowed
        os.makedirs(path, exist_ok=True)
        meta = {"n_streams": self.n_streams, "links": self.links, "regions": []}
        for r in self.regions.values():
            ent = {"name": r.name, "type": r.type, "params": r.getSelf().params, "modes": r.modes}
            if r.type == SENSOR:
                enc = r.getSelf().encoder
                fields = enc.fields() if isinstance(enc, MultiEncoder) else [enc]
                ent["encoder"] = [dict(key=f.name, fieldname=f.fieldname, n=f.n, w=f.w, minval=f.minval,
                                       maxval=f.maxval, clipInput=f.clipInput) for f in fields]
                ent["predictedField"] = r.getSelf().predictedField
            meta["regions"].append(ent)
        with open(os.path.join(path, _META_FILE), "w") as f:
            json.dump(meta, f, indent=1)
        for k, lv in enumerate(self.levels):
            lv.engine.save(os.path.join(path, self._engine_file(k)))
        for i, name in enumerate(self._cls_level):
            self.regions[name].getSelf().classifier.save(os.path.join(path, self._cls_file(name, i == 0)))
        return path

    def _load(self, path):
        from .engine import HTMEngine
        with open(os.path.join(path, _META_FILE)) as f:
            meta = json.load(f)
        self.n_streams = int(meta["n_streams"])
        for ent in meta["regions"]:
            r = self.addRegion(ent["name"], ent["type"], ent["params"])
            r.modes.update(ent["modes"])
            if ent["type"] == SENSOR:
                enc = MultiEncoder()
                for e in ent["encoder"]:
                    enc.addEncoder(e["key"], ScalarEncoder(w=e["w"], minval=e["minval"], maxval=e["maxval"],
                                                           n=e["n"], clipInput=e["clipInput"], name=e["key"],
                                                           fieldname=e["fieldname"]))
                r.getSelf().encoder = enc
                r.getSelf().predictedField = ent.get("predictedField")
        self.links = [tuple(x) for x in meta["links"]]
        _, levels, cls_level = self._chain()
        try:
            for k, lv in enumerate(levels):
                lv.engine = HTMEngine.load(os.path.join(path, self._engine_file(k)), device=self.device)
                if lv.engine.n_streams != self.n_streams:
                    raise RuntimeError("engine file holds %d streams, network.json says %d" %
                                       (lv.engine.n_streams, self.n_streams))
        except Exception:
            for lv in levels:
                if lv.engine is not None:
                    lv.engine.close()
            raise
        self.levels, self._cls_level = levels, cls_level
        self._learn_dirty = True
        from .classifier import SDRClassifier
        for i, name in enumerate(cls_level):
            cp = os.path.join(path, self._cls_file(name, i == 0))
            eng = self.levels[cls_level[name]].engine
            self._init_classifier(self.regions[name],
                                  SDRClassifier.load(cp, device=eng.device) if os.path.exists(cp) else None)
