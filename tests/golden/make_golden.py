"""Generate oracle golden fixtures (run here, committed; the GPU box has no
reference checkout and does not need to run the slow CPU oracle).

model1_golden.npz: the reference's Model-1 experiment replayed through the
oracle (ModelTraining.py then ModelTesting.py):
  train_scores[2184]           anomaly scores of the 2184 training steps the
                               saved network has seen (the save at record
                               2185 happens before its step, NetworkModel.py:123)
  train_active[300, 40]        active columns of the first 300 training steps
  test_windows[2324, 8]        1 + 7 scores per test record (SP learn on, TM
                               learn off; ModelTesting.py:66-72)
  digests                      sha256 of the canonical oracle state after
                               training (SP perms, TM segments)
These pin the oracle against regressions and are the GPU end-to-end check.
Parity against NuPIC itself is UNPINNED (see oracle/htm_oracle.h).
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402


def state_digest(m):
    h = hashlib.sha256()
    st = m.sp_state()
    for k in ["perm", "potential", "connected", "overlap_dc", "active_dc"]:
        h.update(np.ascontiguousarray(st[k]).tobytes())
    sp = h.hexdigest()
    h = hashlib.sha256()
    seg = m.tm_segments(32)
    for k in ["cell", "is_seq", "pos_act", "last_dc_iter", "nsyn", "last_dc", "src", "perm"]:
        h.update(np.ascontiguousarray(seg[k]).tobytes())
    return sp, h.hexdigest()


def main():
    d = np.load(os.path.join(HERE, "model1_traces.npz"))
    train = [c for c, mm in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(mm))]
    assert len(train) == 2185
    m = oracle.OracleModel()
    t0 = time.time()
    scores, active = [], []
    for k, v in enumerate(train[:2184]):
        scores.append(m.step(v, True, True))
        if k < 300:
            active.append(m.active_columns())
    print("train done %.1fs" % (time.time() - t0), flush=True)
    sp_dig, tm_dig = state_digest(m)
    sc = m.tm_scalars()
    te = d["test_cpu"]
    wins = np.zeros((len(te), 8), np.float32)
    for r, v in enumerate(te):
        for j in range(8):
            wins[r, j] = m.step(v, True, False)
    print("test done %.1fs" % (time.time() - t0), flush=True)
    np.savez_compressed(os.path.join(HERE, "model1_golden.npz"),
                        train_scores=np.array(scores, np.float32), train_active=np.array(active, np.int16),
                        test_windows=wins, sp_digest=np.array(sp_dig), tm_digest=np.array(tm_dig),
                        n_segments=np.int64(sc["n_segments"]), n_synapses=np.int64(sc["n_synapses"]))
    print("wrote model1_golden.npz", sc)


if __name__ == "__main__":
    main()
