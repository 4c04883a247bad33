"""Paged SP permanences (htm_config.sp_perm_rows > 0, the config-3 layout).

A paged engine keeps a pool row only for the columns whose permanences have
changed; the other columns' initial values are replayed on the GPU from
nupic::Random checkpoints of the SP initialisation.  It must be
indistinguishable from the dense engine: same scores, same exported SP/TM
state (HTM_ST_SP_PERM is dense in both), through learning, TM-frozen steps
with SP learning on (the reference's test phase, NetworkModel.py:40-44),
export/import, replicate and save/load.  Config 3's per-stream budget
(BASELINE.json configs[2]) is what makes it necessary: dense float32
permanences are 3.2 MiB per stream, 210 GB at 65,536 streams.
"""
import numpy as np
import pytest

from test_gpu_parity import sp_equal, tm_equal

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

N = 16


def inputs(T, n, seed=5):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 101, size=(30, 1)).astype(np.float64)
    v = np.clip(np.tile(base, (T // 30 + 1, n))[:T] + rng.integers(-3, 4, size=(T, n)), 0, 100)
    v[rng.random(v.shape) < 0.02] = np.nan
    return v


def engines(rt, n=N, rows=1536, **kw):
    dense = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 13, **kw)
    paged = rt.HTMEngine(n, seed_stride=1, seg_capacity=1 << 13, sp_perm_rows=rows, **kw)
    return dense, paged


def same_state(a, b, n):
    for region in ("sp_perm", "sp_connT", "sp_potmask", "sp_duty", "sp_scalars", "tm_bitmaps", "tm_colconf",
                   "tm_seg_meta", "tm_seg_src", "tm_seg_perm", "tm_seg_duty"):
        assert np.array_equal(a.export_state(region, 0, n), b.export_state(region, 0, n)), region


def test_initial_permanences_replayed_exactly(rt):
    """Every column's replayed initial permanences (no column has a row yet)
    equal the dense initialisation, for streams with different seeds."""
    dense, paged = engines(rt)
    assert np.array_equal(dense.export_state("sp_perm", 0, N), paged.export_state("sp_perm", 0, N))
    assert np.array_equal(dense.export_state("sp_potmask", 0, N), paged.export_state("sp_potmask", 0, N))
    assert paged.state_bytes("sp_perm_ckpt") == 2048 // 8 * 64 * 4
    assert dense.state_bytes("sp_perm_ckpt") == 0
    assert paged.device_bytes() < dense.device_bytes()


def test_learning_matches_dense_and_oracle(rt, oracle_mod):
    """SP+TM learning (fused run chunks and single steps), then TM frozen with
    SP learning on, then both off: scores and all state identical to the dense
    engine; two streams against independent oracle models."""
    dense, paged = engines(rt)
    T = 150
    vals = inputs(T, N)
    v = torch.tensor(vals, device="cuda")
    got_d = [dense.run(v[:100]).cpu().numpy()]
    got_p = [paged.run(v[:100]).cpu().numpy()]
    for k in range(100, 120):
        got_d.append(dense.step(v[k]).cpu().numpy()[None])
        got_p.append(paged.step(v[k]).cpu().numpy()[None])
    for e in (dense, paged):
        e.set_learning(True, False)
    got_d.append(dense.run(v[120:140]).cpu().numpy())
    got_p.append(paged.run(v[120:140]).cpu().numpy())
    for e in (dense, paged):
        e.set_learning(False, False)
    got_d.append(dense.run(v[140:]).cpu().numpy())
    got_p.append(paged.run(v[140:]).cpu().numpy())
    dense.status()
    paged.status()
    gd, gp = np.concatenate(got_d), np.concatenate(got_p)
    assert np.array_equal(gd, gp)
    same_state(dense, paged, N)
    for s in (0, 11):
        o = oracle_mod.OracleModel(sp_seed=2045 + s, tm_seed=2045 + s)
        flags = [(True, True)] * 120 + [(True, False)] * 20 + [(False, False)] * 10
        want = np.array([o.step([vals[k, s]], *flags[k]) for k in range(T)], np.float32)
        assert np.array_equal(gp[:, s], want), f"stream {s}"
        sp_equal(paged, s, o)
        tm_equal(paged, s, o)


def test_exhausted_row_pool_is_reported(rt):
    """Two rows per stream cannot hold one step's 40 adapted columns: the
    engine flags it (NuPIC would not lose updates, so results are invalid)."""
    eng = rt.HTMEngine(4, seed_stride=1, seg_capacity=1 << 12, sp_perm_rows=2)
    eng.step(torch.tensor([10.0, 20.0, 30.0, 40.0], device="cuda"))
    with pytest.raises(rt.HtmError, match="SP permanence row pool"):
        eng.status()


def test_export_import_between_layouts(rt):
    """A trained paged stream exported region by region and imported into a
    paged engine of other seeds and into a dense engine: identical state and
    identical scores afterwards (the import re-bases onto the source's
    checkpoints, so no permanence changes value)."""
    _, src = engines(rt, n=2)
    v = torch.tensor(inputs(80, 2), device="cuda")
    src.run(v)
    dst_p = rt.HTMEngine(3, seed_stride=1, sp_seed=9000, tm_seed=9000, seg_capacity=1 << 13, sp_perm_rows=1536)
    dst_d = rt.HTMEngine(3, seed_stride=1, sp_seed=9000, tm_seed=9000, seg_capacity=1 << 13)
    for dst in (dst_p, dst_d):
        for region in rt._lib.ST:
            dst.import_state(region, src.export_state(region, 1, 1), s0=2)
        for region in ("sp_perm", "sp_potmask", "tm_seg_src", "tm_seg_perm"):
            assert np.array_equal(dst.export_state(region, 2, 1), src.export_state(region, 1, 1)), region
    w = torch.tensor(inputs(40, 3, seed=8), device="cuda")
    ref = src.run(torch.stack([w[:, 2], w[:, 2]], 1)).cpu().numpy()[:, 1]
    for dst in (dst_p, dst_d):
        got = dst.run(w).cpu().numpy()[:, 2]
        assert np.array_equal(got, ref)
    assert np.array_equal(dst_p.export_state("sp_perm", 0, 3), dst_d.export_state("sp_perm", 0, 3))


def test_replicate_and_save_load(rt, tmp_path):
    """replicate(0) on a paged engine equals replicate(0) on a dense one; a
    saved and reloaded paged engine continues with the same scores."""
    dense, paged = engines(rt, n=6)
    v = torch.tensor(inputs(60, 6), device="cuda")
    dense.run(v)
    paged.run(v)
    dense.replicate(0)
    paged.replicate(0)
    same_state(dense, paged, 6)
    p = str(tmp_path / "paged.htm")
    paged.save(p)
    back = rt.HTMEngine.load(p)
    assert back.config.sp_perm_rows == 1536
    same_state(paged, back, 6)
    w = torch.tensor(np.repeat(inputs(30, 1, seed=2), 6, axis=1), device="cuda")  # one input trace
    a = dense.run(w).cpu().numpy()
    b = paged.run(w).cpu().numpy()
    c = back.run(w).cpu().numpy()
    assert np.array_equal(a, b) and np.array_equal(a, c)
    assert np.array_equal(a, np.repeat(a[:, :1], 6, axis=1))  # replicas of one stream


def test_paged_sdr_input_level(rt):
    """The level-2 SP of Models 2/3 (SDR input) paged vs dense."""
    rng = np.random.default_rng(3)
    kw = dict(sdr_bits=4096, seg_capacity=1 << 12)
    dense = rt.HTMEngine(3, seed_stride=1, **kw)
    paged = rt.HTMEngine(3, seed_stride=1, sp_perm_rows=1024, **kw)
    for k in range(25):
        sdr = np.zeros((3, 4096 // 32), np.uint32)
        bits = rng.choice(4096, size=(3, 80), replace=True)
        for s in range(3):
            for b in bits[s]:
                sdr[s, b // 32] |= np.uint32(1 << (b % 32))
        t = torch.tensor(sdr.view(np.int32), device="cuda")
        assert np.array_equal(dense.step_sdr(t).cpu().numpy(), paged.step_sdr(t).cpu().numpy())
    same_state(dense, paged, 3)
