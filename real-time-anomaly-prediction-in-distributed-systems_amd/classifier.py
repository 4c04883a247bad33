"""Batched SDRClassifier on the GPU.

Replaces the "py.SDRClassifierRegion" of the reference's Model 1
(ML/HTM/NetworkModel.py:70-97: alpha 0.005, steps 1..7, fed TM bottomUpOut,
bucketIdxOut and actValueOut), whose outputs NetworkUtils.getPredictionResults
reads (ML/HTM/NetworkUtils.py:166-184).  The arithmetic runs in
csrc/classifier.hip through the C ABI (htm_cls_*); NuPIC 1.0.x semantics as
restated in oracle/sdr_classifier_reference.py (parity unpinned w.r.t.
NuPIC).  The classifier never feeds the anomaly score.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check

CLS_ST = {"scalars": 1, "actual": 2, "actual_ok": 3, "hist_rec": 4, "hist_len": 5, "hist_idx": 6, "weights": 7}
_ST_DTYPE = {"scalars": np.int32, "actual": np.float64, "actual_ok": np.int32, "hist_rec": np.int32,
             "hist_len": np.int32, "hist_idx": np.uint16, "weights": np.float64}


class SDRClassifier:
    """NuPIC SDRClassifier for n_streams streams.  `compute` is one
    SDRClassifierRegion.compute of every stream; outputs stay on the device."""

    def __init__(self, n_streams: int, n_inputs: int, n_buckets: int, steps=(1,), alpha: float = 0.001,
                 act_value_alpha: float = 0.3, device: int | None = None):
        import torch
        self._L = _lib.lib()
        self.n_streams, self.n_inputs, self.n_buckets = int(n_streams), int(n_inputs), int(n_buckets)
        self.steps = [int(k) for k in steps]
        self.alpha, self.act_value_alpha = float(alpha), float(act_value_alpha)
        self.device = torch.cuda.current_device() if device is None else int(device)
        st = (ctypes.c_int32 * len(self.steps))(*self.steps)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self._L.htm_cls_create(self.n_streams, self.n_inputs, self.n_buckets, st, len(self.steps),
                                         self.alpha, self.act_value_alpha, self.device, ctypes.byref(h)))
        self.h = h
        dev = f"cuda:{self.device}"
        self.probabilities = torch.zeros((self.n_streams, len(self.steps), self.n_buckets), dtype=torch.float64,
                                         device=dev)
        self.actual_values = torch.zeros((self.n_streams, self.n_buckets), dtype=torch.float64, device=dev)

    def close(self):
        if getattr(self, "h", None):
            self._L.htm_cls_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def compute(self, pattern_words, bucket=None, act_value=None, learn: bool = True, infer: bool = True):
        """pattern_words: device int32/uint32 bitmap [n_streams, n_inputs/32]
        (the engine's "tm_output"); bucket: int per stream (< 0: no learning
        for that stream); act_value: float per stream.  Returns
        (probabilities [n, steps, buckets], actual_values [n, buckets]) device
        float64 views, valid until the next compute."""
        import torch
        dev = f"cuda:{self.device}"
        p = pattern_words.to(dev).contiguous()
        if p.numel() * p.element_size() != self.n_streams * self.n_inputs // 8:
            raise ValueError("pattern must be a [n_streams, n_inputs/32] word bitmap")
        b = v = None
        if learn:
            if bucket is None or act_value is None:
                raise ValueError("learning needs bucket and act_value")
            b = torch.as_tensor(np.asarray(bucket) if not isinstance(bucket, torch.Tensor) else bucket)
            b = b.to(device=dev, dtype=torch.int32).reshape(-1).contiguous()
            v = torch.as_tensor(np.asarray(act_value, np.float64) if not isinstance(act_value, torch.Tensor)
                                else act_value)
            v = v.to(device=dev, dtype=torch.float64).reshape(-1).contiguous()
            if b.numel() != self.n_streams or v.numel() != self.n_streams:
                raise ValueError("expected one bucket and one value per stream")
        check(self._L.htm_cls_compute(self.h, ctypes.c_void_p(p.data_ptr()),
                                      ctypes.c_void_p(b.data_ptr()) if b is not None else None,
                                      ctypes.c_void_p(v.data_ptr()) if v is not None else None,
                                      1 if learn else 0, 1 if infer else 0,
                                      ctypes.c_void_p(self.probabilities.data_ptr()),
                                      ctypes.c_void_p(self.actual_values.data_ptr()), self._stream()))
        self._keep = (p, b, v)
        return self.probabilities, self.actual_values

    def status(self) -> int:
        f = ctypes.c_int32()
        check(self._L.htm_cls_status(self.h, ctypes.byref(f)))
        if f.value & 1:
            raise ValueError("SDRClassifier: empty input pattern (NuPIC max() of an empty sequence)")
        if f.value & 2:
            raise ValueError("SDRClassifier: bucket index >= n_buckets")
        return f.value

    # -------------------------------------------------------------- state
    def export_state(self, region: str, s0: int = 0, n: int | None = None) -> np.ndarray:
        n = self.n_streams - s0 if n is None else n
        per = self._L.htm_cls_state_bytes(self.h, CLS_ST[region])
        out = np.empty(per * n, np.uint8)
        check(self._L.htm_cls_export_state(self.h, CLS_ST[region], s0, n, out.ctypes.data_as(ctypes.c_void_p),
                                           out.nbytes))
        return out.view(_ST_DTYPE[region]).reshape(n, -1)

    def import_state(self, region: str, data: np.ndarray, s0: int = 0):
        a = np.ascontiguousarray(data, dtype=_ST_DTYPE[region])
        per = self._L.htm_cls_state_bytes(self.h, CLS_ST[region])
        n = a.nbytes // per
        check(self._L.htm_cls_import_state(self.h, CLS_ST[region], s0, n, a.ctypes.data_as(ctypes.c_void_p),
                                           a.nbytes))

    def state_summary(self, s: int) -> dict:
        sc = self.export_state("scalars", s, 1)[0]
        return {"record_num": int(sc[0]), "max_input": int(sc[1]), "max_bucket": int(sc[2])}

    def weights(self, s: int, step: int) -> np.ndarray:
        """Stream s's weight matrix for `step`, cut to NuPIC's live shape
        [maxInputIdx + 1, maxBucketIdx + 1]."""
        w = self.export_state("weights", s, 1).reshape(len(self.steps), self.n_inputs, self.n_buckets)
        sm = self.state_summary(s)
        return w[self.steps.index(step), :sm["max_input"] + 1, :sm["max_bucket"] + 1]

    def save(self, path: str):
        """State of every stream to one .npz; weights cut to the largest live
        [maxInputIdx + 1, maxBucketIdx + 1] over streams (the rest is zero)."""
        st = {k: self.export_state(k) for k in CLS_ST if k != "weights"}
        mi, mb = int(st["scalars"][:, 1].max()) + 1, int(st["scalars"][:, 2].max()) + 1
        w = self.export_state("weights").reshape(self.n_streams, len(self.steps), self.n_inputs, self.n_buckets)
        st["weights"] = np.ascontiguousarray(w[:, :, :mi, :mb])
        np.savez(path, meta=np.array([self.n_streams, self.n_inputs, self.n_buckets] + self.steps, np.int64),
                 rates=np.array([self.alpha, self.act_value_alpha]), **st)

    @classmethod
    def load(cls, path: str, device: int | None = None) -> "SDRClassifier":
        d = np.load(path, allow_pickle=False)
        m = [int(x) for x in d["meta"]]
        c = cls(m[0], m[1], m[2], steps=m[3:], alpha=float(d["rates"][0]), act_value_alpha=float(d["rates"][1]),
                device=device)
        for k in CLS_ST:
            if k == "weights":
                w = np.zeros((m[0], len(c.steps), m[1], m[2]), np.float64)
                lw = d[k]
                w[:, :, :lw.shape[2], :lw.shape[3]] = lw
                c.import_state(k, w.reshape(m[0], -1))
            else:
                c.import_state(k, d[k])
        return c


def prediction_results(actual_values: np.ndarray, probabilities: np.ndarray, steps, n: int):
    """NetworkUtils.getPredictionResults (ML/HTM/NetworkUtils.py:166-184) over
    one stream's region outputs, including its [i*N:(i+1)*N - 1] slice."""
    results, confidence = [], []
    for i in range(len(steps)):
        sp = probabilities[i * n:(i + 1) * n - 1]
        j = int(np.argmax(sp))
        results.append(actual_values[j])
        confidence.append(sp[j])
    return results, confidence
