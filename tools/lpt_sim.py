"""Offline: would dispatching the previous step's slowest streams first shorten
a lockstep launch?  Reads tools/wg_timeline.py's WG_DUMP ([launch][stream]
workgroup durations, us), list-schedules every launch on SLOTS resident slots
in stream order, and in the order of the previous launch's durations (longest
first; coarse: by duration class), and prints the makespans.
usage: python tools/lpt_sim.py durs.npy [slots]"""
import sys

import numpy as np


def makespan(d, order, slots):
    free = np.zeros(slots)
    for s in order:
        i = int(np.argmin(free))
        free[i] += d[s]
    return free.max()


A = np.load(sys.argv[1])
D = A[:, 0] if A.ndim == 3 else A
if A.ndim == 3:
    for j, name in ((1, "step bytes"), (2, "active cells (end of step)")):
        cj = [np.corrcoef(A[t, 0], A[t, j])[0, 1] for t in range(A.shape[0])]
        print(f"corr(duration, {name}): median {np.median(cj):.3f}")
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 768
ident, lpt, cls2, cls4, oracle, by_cells, by_bytes = [], [], [], [], [], [], []
for t in range(1, D.shape[0]):
    d, prev = D[t], D[t - 1]
    n = len(d)
    ident.append(makespan(d, range(n), slots))
    lpt.append(makespan(d, np.argsort(-prev, kind="stable"), slots))
    med = np.median(prev)
    cls2.append(makespan(d, np.concatenate([np.nonzero(prev > med)[0], np.nonzero(prev <= med)[0]]), slots))
    q = np.quantile(prev, [0.5, 0.75, 0.9])
    c = np.digitize(prev, q)
    cls4.append(makespan(d, np.concatenate([np.nonzero(c == k)[0] for k in (3, 2, 1, 0)]), slots))
    oracle.append(makespan(d, np.argsort(-d, kind="stable"), slots))
    if A.ndim == 3:
        by_cells.append(makespan(d, np.argsort(-A[t, 2], kind="stable"), slots))
        by_bytes.append(makespan(d, np.argsort(-A[t, 1], kind="stable"), slots))
cc = [np.corrcoef(D[t], D[t - 1])[0, 1] for t in range(1, D.shape[0])]
print(f"launches {D.shape[0] - 1}, streams {D.shape[1]}, slots {slots}")
print(f"duration corr(t, t-1): median {np.median(cc):.3f}")
for name, v in (("stream order", ident), ("prev-LPT", lpt), ("prev 2 classes", cls2), ("prev 4 classes", cls4),
                ("clairvoyant LPT", oracle), ("LPT by cells", by_cells), ("LPT by bytes", by_bytes)):
    if not v:
        continue
    print(f"{name:16s} makespan median {np.median(v):7.1f} us")
