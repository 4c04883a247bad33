"""CPU restatement of NuPIC 1.0.x AnomalyLikelihood (nupic/algorithms/
anomaly_likelihood.py) for one stream.  TEST INFRASTRUCTURE ONLY: the checker
of the MI355X likelihood kernel (csrc/likelihood.hip).

PARITY UNPINNED: the reference never computes an anomaly likelihood (SURVEY.md
§0.2, §8(a) row a13 -- only BASELINE.json's north star asks for it) and NuPIC
is not available here, so this restates the published algorithm from its
description, not from code or fixtures:

* probation: the first learningPeriod + estimationSamples (288 + 100) records
  return 0.5;
* the distribution is (re)estimated when missing and every
  reestimationPeriod (100) records, BEFORE the record joins the history, from
  the history deque (<= historicWindowSize = 8640 records): moving averages
  (window 10) of the raw scores, the first `skip` of them dropped
  (skip = min(n, max(0, learningPeriod - max(0, n - historicWindowSize)))),
  mean/variance of the rest with lower bounds 0.03 / 0.0003 -- or the null
  distribution (mean 0.5, stdev 1e3) when no sample is left or the metric
  values' variance is below 1.5e-5;
* every record: moving average of the raw score continues from the
  estimate's window, tail probability Q((avg - mean) / stdev) (mirrored
  below the mean), the "red" filter (a value <= 1e-5 right after another one
  becomes 1e-3), and the returned likelihood is 1 - that.
"""
import math
from collections import deque

LEARNING_PERIOD = 288
ESTIMATION_SAMPLES = 100
HISTORIC_WINDOW = 8640
REESTIMATION_PERIOD = 100
AVERAGING_WINDOW = 10
RED, YELLOW = 1.0 - 0.99999, 1.0 - 0.999


def null_distribution():
    return {"mean": 0.5, "variance": 1e6, "stdev": 1e3}


def estimate_normal(xs, lower_bound=True):
    n = len(xs)
    mean = sum(xs) / n
    var = sum((x - mean) ** 2 for x in xs) / n
    if lower_bound:
        mean = max(mean, 0.03)
        var = max(var, 0.0003)
    return {"mean": mean, "variance": var, "stdev": math.sqrt(var)}


def tail_probability(x, d):
    if x < d["mean"]:
        x = 2 * d["mean"] - x
    z = (x - d["mean"]) / d["stdev"]
    return 0.5 * math.erfc(z / 1.4142)


class MovingAverage:
    def __init__(self, window=AVERAGING_WINDOW):
        self.window, self.values, self.total = window, [], 0.0

    def next(self, v):
        if len(self.values) == self.window:
            self.total -= self.values.pop(0)
        self.values.append(v)
        self.total += v
        return float(self.total) / len(self.values)


class AnomalyLikelihood:
    def __init__(self, learning_period=LEARNING_PERIOD, estimation_samples=ESTIMATION_SAMPLES,
                 historic_window=HISTORIC_WINDOW, reestimation_period=REESTIMATION_PERIOD):
        self.lp, self.es, self.hw, self.rp = learning_period, estimation_samples, historic_window, reestimation_period
        self.iteration = 0
        self.history = deque(maxlen=historic_window)  # (value, raw score)
        self.dist = None
        self.ma = None
        self.hist_lik = []

    def _estimate(self):
        n = self.iteration
        skip = min(n, max(0, self.lp - max(0, n - self.hw)))
        ma = MovingAverage()
        avgs = [ma.next(s) for _, s in self.history]
        if len(avgs) <= skip:
            dist = null_distribution()
        else:
            dist = estimate_normal(avgs[skip:])
            metric = estimate_normal([v for v, _ in self.history][skip:], lower_bound=False)
            if metric["variance"] < 1.5e-5:
                dist = null_distribution()
        self.dist = dist
        self.ma = ma
        self.hist_lik = [tail_probability(a, dist) for a in avgs[-min(AVERAGING_WINDOW, len(avgs)):]]

    def anomaly_probability(self, value, score):
        if self.iteration < self.lp + self.es:
            lik = 0.5
        else:
            if self.dist is None or self.iteration % self.rp == 0:
                self._estimate()
            avg = self.ma.next(score)
            p = tail_probability(avg, self.dist)
            prev = self.hist_lik[-1] if self.hist_lik else None
            filt = (p if (prev is not None and prev > RED) else YELLOW) if (p <= RED and prev is not None) else p
            self.hist_lik = (self.hist_lik + [p])[-AVERAGING_WINDOW:]
            lik = 1.0 - filt
        self.history.append((float(value), float(score)))
        self.iteration += 1
        return lik
