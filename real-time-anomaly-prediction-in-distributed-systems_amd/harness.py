"""Batched counterparts of the reference's drivers.

* `SLOHarness` -- ModelTesting.py's SLO-violation prediction (runModel
  :36-107, processpredictionList :113-146, getModelStats :148-171) for N
  streams at once, on the GPU (csrc/slo.hip through the C ABI).
* `model_training` / `model_testing` -- the record loops of ModelTraining.py
  (:21-56, :80-97) and ModelTesting.py (:36-107, :194-213) for Model 1, over
  [records, streams] value arrays: record skipping on missing metrics, the
  save of network1 BEFORE the 2185th record's step (NetworkModel.py:123-127),
  TM learning switched off on the first test record while the SP keeps
  learning (NetworkModel.py:40-44), and 1 + 7 network steps per test record
  fed the same value (ModelTesting.py:66-72).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check

ANOMALY_SCORE = 0.85      # ModelTesting.py:30 (the README's sweep uses 0.98 / 0.99)
MAX_LEAD_TIME = 50        # ModelTesting.py:31
SLO_RESPONSE_TIME = 70    # ModelTesting.py:32
SAVE_FREQUENCY = 2185     # NetworkUtils.py:67
LOOKAHEAD = 7             # len(results[0]) of NetworkModel.py:19-20


class SLOHarness:
    """Per-stream SLO prediction state machine on the GPU."""

    def __init__(self, n_streams: int, threshold: float = ANOMALY_SCORE, max_lead: int = MAX_LEAD_TIME,
                 slo_response: int = SLO_RESPONSE_TIME, device: int | None = None):
        import torch
        self._L = _lib.lib()
        self.n_streams = int(n_streams)
        self.device = torch.cuda.current_device() if device is None else int(device)
        h = ctypes.c_void_p()
        check(self._L.htm_slo_create(self.n_streams, float(threshold), int(max_lead), int(slo_response),
                                     self.device, ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._L.htm_slo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, x, dtype):
        import torch
        t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
        t = t.to(device=f"cuda:{self.device}", dtype=dtype).contiguous()
        if t.numel() != self.n_streams:
            raise ValueError("expected one value per stream")
        return t

    def record(self, window_scores, violations, means, valid=None):
        """One runModel record of every stream: window_scores [w, n_streams]
        float32 device tensor (the engine's scores of the record's 1 + 7
        steps), violations / int(mean) per stream, valid = False skips the
        stream's record (a null cpu/mem, :51-53)."""
        import torch
        w = window_scores
        if not isinstance(w, torch.Tensor) or w.dtype != torch.float32 or w.dim() != 2 or \
                w.shape[1] != self.n_streams:
            raise ValueError("window_scores must be a float32 [window, n_streams] tensor")
        w = w.to(f"cuda:{self.device}").contiguous()
        v = self._dev(violations, torch.int32)
        m = self._dev(means, torch.int32)
        ok = self._dev(valid, torch.uint8) if valid is not None else None
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check(self._L.htm_slo_record(self.h, ctypes.c_void_p(w.data_ptr()), int(w.shape[0]),
                                     ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(m.data_ptr()),
                                     ctypes.c_void_p(ok.data_ptr()) if ok is not None else None, st))
        self._keep = (w, v, m, ok)  # alive until the kernel has read them

    def stats(self) -> np.ndarray:
        """getModelStats per stream: int64 [n_streams, 5] = TP, FP, TN, FN, lead-time sum."""
        import torch
        out = np.zeros((self.n_streams, 5), np.int64)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check(self._L.htm_slo_stats(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), st))
        return out


class AnomalyLikelihood:
    """NuPIC's AnomalyLikelihood.anomalyProbability for N streams at once on
    the GPU (csrc/likelihood.hip; parity unpinned -- the reference has no
    likelihood).  Defaults are NuPIC's."""

    def __init__(self, n_streams: int, learning_period: int = 288, estimation_samples: int = 100,
                 historic_window: int = 8640, reestimation_period: int = 100, device: int | None = None):
        import torch
        self._L = _lib.lib()
        self.n_streams = int(n_streams)
        self.device = torch.cuda.current_device() if device is None else int(device)
        h = ctypes.c_void_p()
        check(self._L.htm_likelihood_create(self.n_streams, int(learning_period), int(estimation_samples),
                                            int(historic_window), int(reestimation_period), self.device,
                                            ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._L.htm_likelihood_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def anomaly_probability(self, values, scores, out=None):
        """values: device float64 [n_streams] or [n_streams, fields] (field 0 is
        the metric); scores: device float32 [n_streams].  Returns float64 [n]."""
        import torch
        v = values.contiguous()
        stride = 1 if v.dim() == 1 else v.shape[1]
        if v.dtype != torch.float64 or v.shape[0] != self.n_streams:
            raise ValueError("values must be float64 [n_streams(, fields)]")
        sc = scores.contiguous()
        if sc.dtype != torch.float32 or sc.numel() != self.n_streams:
            raise ValueError("scores must be float32 [n_streams]")
        if out is None:
            out = torch.empty(self.n_streams, dtype=torch.float64, device=sc.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check(self._L.htm_likelihood_step(self.h, ctypes.c_void_p(v.data_ptr()), int(stride),
                                          ctypes.c_void_p(sc.data_ptr()), ctypes.c_void_p(out.data_ptr()), st))
        return out


def valid_records(cpu, mem):
    """ModelTraining.py:29-32 / ModelTesting.py:51-53: a record with a null cpu
    or mem is skipped."""
    return ~(np.isnan(np.asarray(cpu, np.float64)) | np.isnan(np.asarray(mem, np.float64)))


def model_training(engine, cpu, save_path=None):
    """ModelTraining.runModel over cpu[records] (one stream: [records]; N
    streams sharing the record sequence: [records, N]).  Every stream sees
    every valid record once with SP and TM learning on; when the record
    counter reaches SAVE_FREQUENCY the engine is saved BEFORE that record's
    step (NetworkModel.py:123-127).  Returns the scores [steps, N]."""
    import torch
    v = np.asarray(cpu, np.float64)
    v = v.reshape(v.shape[0], -1)
    engine.set_learning(True, True)
    dev = f"cuda:{engine.device}"
    vals = torch.tensor(v, device=dev)
    n = v.shape[0]
    out = torch.empty((n, engine.n_streams), dtype=torch.float32, device=dev)
    k_save = SAVE_FREQUENCY - 1 if (save_path and n >= SAVE_FREQUENCY) else n
    engine.run(vals[:k_save], out=out[:k_save])
    engine.status()  # raise on pool / queue overflow (NuPIC's NTA_THROW)
    if k_save < n:
        engine.save(save_path)
        engine.run(vals[k_save:], out=out[k_save:])
        engine.status()
    return out


def model_testing(engine, cpu, violations, means, threshold=ANOMALY_SCORE, lookahead=LOOKAHEAD, slo=None,
                  chunk_records=256):
    """ModelTesting.runModel over test records for every stream: TM learning
    off (SP learning on), 1 + lookahead steps per record fed the record's
    value, the scores judged by the SLO harness on the GPU.  cpu / violations
    / means: [records] or [records, N].  Returns (windows [records, 1 +
    lookahead, N] float32 on the host, stats int64 [N, 5])."""
    import torch
    v = np.asarray(cpu, np.float64)
    v = v.reshape(v.shape[0], -1)
    n_rec, n = v.shape
    if n != engine.n_streams:
        v = np.broadcast_to(v, (n_rec, engine.n_streams))
        n = engine.n_streams
    viol = np.broadcast_to(np.asarray(violations, np.int64).reshape(n_rec, -1), (n_rec, n)).astype(np.int32)
    mean = np.broadcast_to(np.asarray(means).reshape(n_rec, -1), (n_rec, n)).astype(np.float64).astype(np.int32)
    w = 1 + lookahead
    slo = slo if slo is not None else SLOHarness(n, threshold=threshold, device=engine.device)
    engine.set_learning(True, False)  # NetworkModel.py:40-44 on the first test record
    dev = f"cuda:{engine.device}"
    windows = np.zeros((n_rec, w, n), np.float32)
    for r0 in range(0, n_rec, chunk_records):
        m = min(chunk_records, n_rec - r0)
        steps = torch.tensor(np.repeat(v[r0:r0 + m], w, axis=0), device=dev)  # [m * w, n]
        sc = engine.run(steps)
        vv = torch.tensor(viol[r0:r0 + m], device=dev)
        mm = torch.tensor(mean[r0:r0 + m], device=dev)
        for j in range(m):
            slo.record(sc[j * w:(j + 1) * w], vv[j], mm[j])
        windows[r0:r0 + m] = sc.reshape(m, w, n).cpu().numpy()
        engine.status()  # raise on pool / queue overflow (NuPIC's NTA_THROW)
    return windows, slo.stats()
