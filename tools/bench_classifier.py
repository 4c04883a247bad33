"""Microbenchmark of the SDRClassifier kernels (csrc/classifier.hip): S
Model-1-shape streams (24,576 TM cells, 480 buckets, steps 1..7, alpha
0.005), ~250-bit patterns (40 active columns x ~6 cells), learning on.
Reports records/s and the algorithmic HBM rate of cls_step_kernel:
per stream-record, for each step k: inference reads |p| rows x B live
buckets x 8 B, the error pass reads |p_k| x B x 8 B (the pattern of age k),
the update reads and writes the same -> sum_k (|p| + 3 |p_k|) x B x 8 B."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

rt = _pkg.load()
S = int(os.environ.get("CLS_STREAMS", "64"))
R = int(os.environ.get("CLS_RECORDS", "200"))
cells, nb, steps = 2048 * 12, 480, [1, 2, 3, 4, 5, 6, 7]
cl = rt.classifier.SDRClassifier(S, cells, nb, steps=steps, alpha=0.005)
rng = np.random.default_rng(0)
pats = []
for r in range(R):
    w = np.zeros((S, cells // 32), np.uint32)
    for s in range(S):
        cols = rng.choice(2048, size=40, replace=False)
        idx = (cols[:, None] * 12 + rng.integers(0, 12, size=(40, 6))).ravel()
        np.bitwise_or.at(w[s], idx // 32, (1 << (idx % 32)).astype(np.uint32))
    pats.append(torch.tensor(w.view(np.int32), device="cuda"))
buckets = torch.tensor(rng.integers(0, nb, size=(R, S)), dtype=torch.int32, device="cuda")
vals = torch.tensor(rng.random((R, S)) * 100, device="cuda")
plen = np.array([[int(np.unpackbits(p.cpu().numpy()[s].view(np.uint8)).sum()) for s in range(S)] for p in pats])
for r in range(16):  # warm-up: buckets grow to the full range quickly
    cl.compute(pats[r], buckets[r], vals[r])
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(16, R):
    cl.compute(pats[r], buckets[r], vals[r])
torch.cuda.synchronize()
dt = time.perf_counter() - t0
cl.status()
n = R - 16
B = nb  # live buckets after warm-up (random buckets over the full range)
byts = sum(int((plen[r] + 3 * plen[r - k]).sum()) for r in range(16, R) for k in steps) * B * 8
print(json.dumps({"streams": S, "records": n, "records_per_s": round(S * n / dt, 1), "ms_per_record": round(dt / n * 1e3, 4),
                  "algorithmic_GBps": round(byts / dt / 1e9, 1), "avg_pattern_bits": float(plen.mean())}))
