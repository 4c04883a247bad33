"""CPU restatement of NuPIC 1.0.x's SDRClassifier (nupic/algorithms/
sdr_classifier.py, implementation 'py') behind SDRClassifierRegion.compute,
plus the reference's getPredictionResults.  TEST INFRASTRUCTURE ONLY: the
checker of the MI355X classifier kernels (csrc/classifier.hip).

Reference call sites: the region is built with alpha 0.005 and steps
'1,2,3,4,5,6,7' (ML/HTM/NetworkModel.py:70-97), fed TM bottomUpOut plus the
sensor's bucketIdxOut / actValueOut (:88-95), learns during training and is
switched to learningMode False on the first test record together with the TM
(NetworkModel.py:40-44); its output is read by NetworkUtils.getPredictionResults
(ML/HTM/NetworkUtils.py:166-184), whose per-step results give the
7-step lookahead count (ModelTesting.py:66-72).

PARITY UNPINNED: NuPIC is not installable here and the
reference holds no classifier fixtures, so this restates the published
algorithm:

* history: deque of (recordNum, patternNZ), maxlen max(steps) + 1;
* weights per step: float64 [maxInputIdx + 1, maxBucketIdx + 1], grown with
  zero rows / columns as larger input / bucket indices arrive (rows before
  inference, columns during learning);
* inferSingleStep: activation = weights[patternNZ].sum(axis=0) (rows added
  in patternNZ order), softmax = exp(a - max(a)) / sum(exp(...)), the sum in
  numpy's pairwise order (numpy_pairwise_sum below; numpy 1.x and 2.x agree);
* learn: actualValues[bucket] EMA with actValueAlpha 0.3 (first value taken
  as is); for every history entry whose age nSteps is in steps,
  weights[nSteps][bit, :] += alpha * (target - inferSingleStep(entry)), the
  error taken before any of this record's updates (each age appears once);
* infer runs before learn, with the default value for buckets that never had
  an actual value = actValueList[0] (the region's dummy 0 when not learning).
The GPU uses the device exp (ocml) where numpy uses its own; probabilities are
compared within 1e-12 relative, argmax-derived predictions exactly.
"""
from collections import deque

import numpy as np

MAX_CATEGORY_COUNT = 1000  # SDRClassifierRegion default


def numpy_pairwise_sum(a):
    """numpy's float64 add.reduce over a contiguous vector (pairwise, blocks of 8)."""
    n = len(a)
    if n < 8:
        r = 0.0
        for x in a:
            r += float(x)
        return r
    if n <= 128:
        r = [float(x) for x in a[:8]]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += float(a[i + j])
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += float(a[i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return numpy_pairwise_sum(a[:n2]) + numpy_pairwise_sum(a[n2:])


def infer_single_step(pattern_nz, weights):
    act = np.zeros(weights.shape[1])
    for i, bit in enumerate(pattern_nz):  # rows in patternNZ order
        act = weights[bit].copy() if i == 0 else act + weights[bit]
    act = act - np.max(act)
    e = np.exp(act)
    return e / numpy_pairwise_sum(e)


class SDRClassifier:
    def __init__(self, steps=(1,), alpha=0.001, act_value_alpha=0.3):
        self.steps = list(steps)
        self.alpha = alpha
        self.act_value_alpha = act_value_alpha
        self.history = deque(maxlen=max(self.steps) + 1)
        self.max_input = 0
        self.max_bucket = 0
        self.weights = {k: np.zeros((1, 1)) for k in self.steps}
        self.actual_values = [None]

    def compute(self, record_num, pattern_nz, bucket_idx, act_value, learn, infer):
        if len(self.history) == 0 or record_num > self.history[-1][0]:
            self.history.append((record_num, list(pattern_nz)))
        if len(pattern_nz) == 0:
            raise ValueError("max() arg is an empty sequence")  # NuPIC's max(patternNZ)
        m = int(max(pattern_nz))
        if m > self.max_input:
            for k in self.steps:
                self.weights[k] = np.concatenate(
                    (self.weights[k], np.zeros((m - self.max_input, self.max_bucket + 1))), axis=0)
            self.max_input = m
        retval = None
        if infer:
            default = 0 if self.steps[0] == 0 else act_value
            retval = {"actualValues": [x if x is not None else default for x in self.actual_values]}
            for k in self.steps:
                retval[k] = infer_single_step(pattern_nz, self.weights[k])
        if learn and bucket_idx is not None:
            if bucket_idx > self.max_bucket:
                for k in self.steps:
                    self.weights[k] = np.concatenate(
                        (self.weights[k], np.zeros((self.max_input + 1, bucket_idx - self.max_bucket))), axis=1)
                self.max_bucket = int(bucket_idx)
            while self.max_bucket > len(self.actual_values) - 1:
                self.actual_values.append(None)
            if self.actual_values[bucket_idx] is None:
                self.actual_values[bucket_idx] = act_value
            else:
                self.actual_values[bucket_idx] = ((1.0 - self.act_value_alpha) * self.actual_values[bucket_idx]
                                                  + self.act_value_alpha * act_value)
            target = np.zeros(self.max_bucket + 1)
            target[bucket_idx] = 1.0
            err = {}
            for rec, pnz in self.history:
                k = record_num - rec
                if k in self.steps:
                    err[k] = target - infer_single_step(pnz, self.weights[k])
            for rec, pnz in self.history:
                k = record_num - rec
                if k in self.steps:
                    for bit in pnz:
                        self.weights[k][bit, :] += self.alpha * err[k]
        return retval


class SDRClassifierRegion:
    """SDRClassifierRegion.compute over one stream: outputs actualValues
    [maxCategoryCount] and probabilities [len(steps) * maxCategoryCount]."""

    def __init__(self, steps="1", alpha=0.001, max_category_count=MAX_CATEGORY_COUNT):
        self.stepsList = [int(x) for x in str(steps).split(",")]
        self.maxCategoryCount = max_category_count
        self.cl = SDRClassifier(self.stepsList, alpha)
        self.learningMode = True
        self.inferenceMode = True
        self.recordNum = 0
        self.actualValues = np.zeros(max_category_count)
        self.probabilities = np.zeros(len(self.stepsList) * max_category_count)

    def compute(self, bottom_up_in, bucket_idx, act_value):
        pnz = np.nonzero(bottom_up_in)[0]
        if self.learningMode:
            b, v = (int(bucket_idx), float(act_value)) if bucket_idx is not None else (None, float(act_value))
        else:
            b, v = 0, 0  # the region's dummy classification
        r = self.cl.compute(self.recordNum, pnz, b, v, self.learningMode, self.inferenceMode)
        if r:
            av = r["actualValues"]
            self.actualValues[:len(av)] = av
            n = self.maxCategoryCount
            for i, k in enumerate(self.stepsList):
                p = r[k]
                self.probabilities[i * n:(i + 1) * n] = 0.0
                self.probabilities[i * n:i * n + min(n, len(p))] = p[:n]
        self.recordNum += 1


def prediction_results(actual_values, probabilities, steps, n=MAX_CATEGORY_COUNT):
    """NetworkUtils.getPredictionResults (ML/HTM/NetworkUtils.py:166-184),
    including its [i*N:(i+1)*N - 1] slice."""
    results, conf = [], []
    for i in range(len(steps)):
        sp = probabilities[i * n:(i + 1) * n - 1]
        j = int(np.argmax(sp))
        results.append(actual_values[j])
        conf.append(sp[j])
    return results, conf
