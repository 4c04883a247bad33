"""SDRClassifier kernels (csrc/classifier.hip) against the CPU restatement
(oracle/sdr_classifier_reference.py), fed the same TM output patterns.

Parity w.r.t. NuPIC is unpinned.  Tolerance: probabilities within 1e-9
relative (the device exp and numpy's exp may differ in the last ulp, and the
difference feeds back through learning); actual values, bucket bounds and
history are exact, and so are the getPredictionResults argmax predictions."""
import numpy as np
import pytest

import sdr_classifier_reference as scr

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

STEPS = [1, 2, 3, 4, 5, 6, 7]  # NetworkModel.py:79
ALPHA = 0.005                  # NetworkModel.py:73
NB = 480                       # ScalarEncoder n=500 w=21 buckets


def compare(rt, cl, regs, pat_words, vals, learn, n_cells, k):
    enc = rt.ScalarEncoder(w=21, minval=0.0, maxval=100.0, n=500, clipInput=True)
    b = enc.bucket_indices(vals)
    prob, act = cl.compute(pat_words, b if learn else None, vals if learn else None, learn=learn, infer=True)
    prob, act = prob.cpu().numpy(), act.cpu().numpy()
    dense = np.unpackbits(pat_words.cpu().numpy().astype(np.uint32).view(np.uint8).reshape(len(regs), -1),
                          axis=1, bitorder="little")[:, :n_cells]
    for s, reg in enumerate(regs):
        reg.learningMode = learn
        reg.compute(dense[s], int(b[s]), float(vals[s]))
        n = reg.maxCategoryCount
        assert np.array_equal(act[s], reg.actualValues[:NB]), f"actual values differ at record {k} stream {s}"
        for i in range(len(STEPS)):
            ref = reg.probabilities[i * n:i * n + NB]
            np.testing.assert_allclose(prob[s, i], ref, rtol=1e-9, atol=1e-15,
                                       err_msg=f"step {STEPS[i]} record {k} stream {s}")
        full = np.zeros_like(reg.probabilities)
        for i in range(len(STEPS)):
            full[i * n:i * n + NB] = prob[s, i]
        av = np.zeros_like(reg.actualValues)
        av[:NB] = act[s]
        assert scr.prediction_results(av, full, STEPS)[0] == scr.prediction_results(
            reg.actualValues, reg.probabilities, STEPS)[0]


def test_classifier_matches_restatement_on_model1_patterns(rt, traces):
    n = 3
    eng = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 13)
    cl = rt.classifier.SDRClassifier(n, eng.n_cells, NB, steps=STEPS, alpha=ALPHA)
    regs = [scr.SDRClassifierRegion(steps=",".join(map(str, STEPS)), alpha=ALPHA) for _ in range(n)]
    tr = traces["train"]
    for k in range(160):
        v = np.array([tr[(k + 37 * s) % len(tr)] for s in range(n)], np.float64)
        eng.step(torch.tensor(v, device="cuda"))
        compare(rt, cl, regs, eng.get_output("tm_output"), v, True, eng.n_cells, k)
    eng.set_learning(True, False)
    for k in range(160, 200):  # ModelTesting: classifier learning off (NetworkModel.py:40-44)
        v = np.array([tr[(k + 37 * s) % len(tr)] for s in range(n)], np.float64)
        eng.step(torch.tensor(v, device="cuda"))
        compare(rt, cl, regs, eng.get_output("tm_output"), v, False, eng.n_cells, k)
    assert cl.status() == 0
    for s in range(n):
        sm = cl.state_summary(s)
        c = regs[s].cl
        assert (sm["max_input"], sm["max_bucket"], sm["record_num"]) == (c.max_input, c.max_bucket, 200)
        np.testing.assert_allclose(cl.weights(s, 3), c.weights[3], rtol=1e-9, atol=1e-15)


def test_classifier_save_load_roundtrip(rt, tmp_path):
    n, cells = 2, 2048 * 12
    rng = np.random.default_rng(3)
    cl = rt.classifier.SDRClassifier(n, cells, NB, steps=[1, 2], alpha=0.05)
    words = lambda: torch.tensor(rng.integers(0, 2**31, size=(n, cells // 32)) & rng.integers(0, 2**31, size=(n, cells // 32)) & rng.integers(0, 2**31, size=(n, cells // 32)),
                                 dtype=torch.int32, device="cuda")
    for _ in range(12):
        cl.compute(words(), rng.integers(0, NB, size=n), rng.random(n) * 100)
    p = str(tmp_path / "cls.npz")
    cl.save(p)
    c2 = rt.classifier.SDRClassifier.load(p)
    w = words()
    a = [x.cpu().numpy().copy() for x in cl.compute(w, [5, 6], [1.0, 2.0])]
    b = [x.cpu().numpy().copy() for x in c2.compute(w, [5, 6], [1.0, 2.0])]
    assert all(np.array_equal(x, y) for x, y in zip(a, b))


def test_empty_pattern_and_bad_bucket_are_reported(rt):
    cl = rt.classifier.SDRClassifier(1, 64, 8, steps=[1])
    cl.compute(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), [1], [1.0])
    with pytest.raises(ValueError):
        cl.status()
    cl2 = rt.classifier.SDRClassifier(1, 64, 8, steps=[1])
    cl2.compute(torch.ones((1, 2), dtype=torch.int32, device="cuda"), [9], [1.0])
    with pytest.raises(ValueError):
        cl2.status()


def test_facade_classifier_prediction_results(rt, traces):
    """The reference's createOneLevelNetwork + getPredictionResults through the facade."""
    import reference_model1 as ref
    src = rt.BatchRecordStream(names=("cpu",), n_streams=1)
    net = ref.create_one_level_network(rt, src)
    cls = net.regions[ref.CLS]
    reg = scr.SDRClassifierRegion(steps="1,2,3,4,5,6,7", alpha=0.005)
    tr = traces["train"][:80]
    for k, v in enumerate(tr):
        src.setData(float(v))
        net.run(1)
        res, conf = scr.prediction_results(cls.getOutputData("actualValues"), cls.getOutputData("probabilities"),
                                           cls.getSelf().stepsList)
        dense = net.regions[ref.TMR].getOutputData("bottomUpOut")[0]
        reg.compute(dense, int(rt.ScalarEncoder(w=21, minval=0.0, maxval=100.0, n=500, clipInput=True)
                               .getBucketIndices(float(v))[0]), float(v))
        assert res == scr.prediction_results(reg.actualValues, reg.probabilities, reg.stepsList)[0], k
    assert cls.getOutputData("probabilities").shape == (7 * 1000,)
