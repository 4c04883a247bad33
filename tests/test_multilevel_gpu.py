"""GPU parity of the two-level networks (Models 2 and 3) against the oracle.

Reference: ML/HTM/MultiLevelNetworkModel.py:53-127 (Model 2: cpu encoder,
L1 SP -> L1 TM -> L2 SP -> L2 TM, l2 anomalyScore returned at :150) and
ML/HTM/MultiLevelNetworkAnomaly.py:61-127 (Model 3: the cpu+mem encoder).  The
L2 SPRegion's input is the L1 TMRegion bottomUpOut (inputWidth = 2048 x 12 =
24,576, MultiLevelNetworkModel.py:92-94); both levels use the same
NetworkUtils SP/TM parameters and seed.  The engine side is two HTMEngines:
L1 reads encoder values, L2 (sdr_bits=24576) reads L1's "tm_output" bitmap
through htm_step_sdr.  The oracle's L2 (orc_step_sdr) is a restatement of the
same NuPIC code on a 0/1 input vector: parity with NuPIC itself is unpinned
for the two-level models (no reference outputs exist for them).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from test_gpu_parity import sp_equal, tm_equal  # noqa: E402

L2_BITS = 2048 * 12


def traces():
    return np.load(os.path.join(GOLDEN, "model1_traces.npz"))


def two_level(rt, oracle_mod, n, n_fields, stride):
    l1 = rt.HTMEngine(n, n_fields=n_fields, seed_stride=stride, seg_capacity=1 << 13)
    l2 = rt.HTMEngine(n, sdr_bits=L2_BITS, seed_stride=stride, seg_capacity=1 << 13)
    o1 = [oracle_mod.OracleModel(n_fields=n_fields, sp_seed=2045 + stride * s, tm_seed=2045 + stride * s)
          for s in range(n)]
    o2 = [oracle_mod.OracleModel(sdr_bits=L2_BITS, sp_seed=2045 + stride * s, tm_seed=2045 + stride * s)
          for s in range(n)]
    return l1, l2, o1, o2


def run_two_level(l1, l2, o1, o2, values, sp_learn, tm_learn):
    """network.run(1) per record: L1 then L2 in the same step (the links carry
    no delay).  Checks L1 score, the bottomUpOut handed to L2, L2 score and the
    L2 active columns at every step."""
    n = len(o1)
    for eng in (l1, l2):
        eng.set_learning(sp_learn, tm_learn)
    for k in range(values.shape[0]):
        v = values[k].reshape(n, -1)
        g1 = l1.step(torch.tensor(v.ravel(), device="cuda")).cpu().numpy()
        sdr = l1.get_output("tm_output")
        g2 = l2.step_sdr(sdr).cpu().numpy()
        bits = l1.bitmap_to_dense(sdr)
        act2 = l2.get_output("active_columns").cpu().numpy()
        for s in range(n):
            r1 = o1[s].step(v[s], sp_learn, tm_learn)
            assert g1[s] == r1, f"L1 step {k} stream {s}: gpu {g1[s]} oracle {r1}"
            ob = o1[s].tm_output()
            assert np.array_equal(bits[s], ob), f"L1 bottomUpOut differs at step {k} stream {s}"
            r2 = o2[s].step_sdr(ob, sp_learn, tm_learn)
            assert g2[s] == r2, f"L2 step {k} stream {s}: gpu {g2[s]} oracle {r2}"
            ao = np.zeros(l2.n_columns, np.uint8)
            ao[o2[s].active_columns()] = 1
            assert np.array_equal(act2[s], ao), f"L2 active columns differ at step {k} stream {s}"


def test_model2_two_level_cpu(rt, oracle_mod):
    """Model 2: cpu-only encoder; training (both levels learning) then TM
    learning off on the test records (runNetwork disableTraining,
    MultiLevelNetworkModel.py:40-51: SP keeps learning)."""
    tr = traces()
    train = np.asarray(tr["train_cpu"], np.float64)
    train = train[~np.isnan(train)][:160]
    test = np.asarray(tr["test_cpu"], np.float64)[:60]
    n = 2
    l1, l2, o1, o2 = two_level(rt, oracle_mod, n, 1, 5)
    sp_equal(l2, 1, o2[1])  # L2 SP initialisation over 24,576 inputs
    vals = np.stack([train, np.roll(train, 7)], axis=1)
    run_two_level(l1, l2, o1, o2, vals, True, True)
    tm_equal(l2, 0, o2[0])
    te = np.stack([test, np.roll(test, 3)], axis=1)
    run_two_level(l1, l2, o1, o2, te, True, False)
    for s in range(n):
        sp_equal(l2, s, o2[s])
        tm_equal(l2, s, o2[s])
        tm_equal(l1, s, o1[s])


def test_model3_two_level_cpu_mem(rt, oracle_mod):
    """Model 3: the cpu+mem MultiEncoder (NetworkUtils.py:77-107,
    multilevelAnomaly=True) under the same two-level network."""
    tr = traces()
    a = np.stack([tr["train_cpu"], tr["train_mem"]], axis=1).astype(np.float64)
    a = a[~np.isnan(a).any(axis=1)][:140]
    b = np.stack([tr["test_cpu"], tr["test_mem"]], axis=1).astype(np.float64)[:40]
    l1, l2, o1, o2 = two_level(rt, oracle_mod, 1, 2, 0)
    run_two_level(l1, l2, o1, o2, a, True, True)
    run_two_level(l1, l2, o1, o2, b, True, False)
    sp_equal(l2, 0, o2[0])
    tm_equal(l2, 0, o2[0])


def test_sdr_engine_rejects_encoder_calls(rt):
    l2 = rt.HTMEngine(1, sdr_bits=L2_BITS, seg_capacity=1 << 12)
    with pytest.raises(Exception, match="input SDR"):
        l2.step(torch.zeros(1, dtype=torch.float64, device="cuda"))
    l1 = rt.HTMEngine(1, seg_capacity=1 << 12)
    with pytest.raises(ValueError):
        l1.step_sdr(torch.zeros((1, L2_BITS // 32), dtype=torch.int32, device="cuda"))


def test_run_sdr_equals_steps(rt):
    """htm_run_sdr over [T, N, words] == T htm_step_sdr calls (random sparse SDRs)."""
    rng = np.random.default_rng(3)
    T, n = 12, 3
    dense = (rng.random((T, n, L2_BITS)) < 0.02).astype(np.uint8)
    words = np.packbits(dense, axis=2, bitorder="little").view(np.uint32).view(np.int32)
    x = torch.tensor(words, device="cuda")
    a = rt.HTMEngine(n, sdr_bits=L2_BITS, seed_stride=1, seg_capacity=1 << 12)
    b = rt.HTMEngine(n, sdr_bits=L2_BITS, seed_stride=1, seg_capacity=1 << 12)
    ra = a.run_sdr(x).cpu().numpy()
    rb = np.stack([b.step_sdr(x[t]).cpu().numpy() for t in range(T)])
    assert np.array_equal(ra, rb)
