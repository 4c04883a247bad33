"""Oracle unit tests: encoder, nupic::Random, SpatialPooler and TM invariants.

The oracle restates NuPIC 1.0.x as wired by the reference (parity UNPINNED
against NuPIC itself, see oracle/htm_oracle.h); these tests pin its rules.
"""
import math

import numpy as np
import pytest


def test_encoder_known_answers(oracle_mod):
    # ScalarEncoder(n=500, w=21, minval=0, maxval=100, clipInput=True):
    # resolution = 100/479, first on-bit = int((x + r/2) / r)  (NetworkUtils.py:77-88)
    m = oracle_mod.OracleModel()
    r = 100.0 / 479
    for x in [0.0, 0.1, 1.0, 13.0, 50.0, 70.0, 99.9, 100.0, 150.0, -5.0]:
        xc = min(max(x, 0.0), 100.0)
        b = int((xc + r / 2) / r)
        enc = m.encode([x])
        assert enc.sum() == 21
        assert np.nonzero(enc)[0][0] == b
        assert np.nonzero(enc)[0][-1] == b + 20
    assert m.encode([float("nan")]).sum() == 0
    assert np.nonzero(m.encode([100.0]))[0][-1] == 499


def test_multi_field_encoder(oracle_mod):
    m = oracle_mod.OracleModel(n_fields=2)
    e = m.encode([10.0, 90.0])
    assert e.shape == (1000,) and e.sum() == 42
    assert np.array_equal(e[:500], m.encode([10.0, 0.0])[:500])


def test_rng_deterministic_and_31bit(oracle_mod):
    a = oracle_mod.rng_stream(2045, 1000)
    b = oracle_mod.rng_stream(2045, 1000)
    c = oracle_mod.rng_stream(2046, 1000)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a.max() < 2 ** 31
    r = oracle_mod.rng_real64(2045, 20000)
    assert 0.0 <= r.min() and r.max() < 1.0
    assert abs(r.mean() - 0.5) < 0.01
    # 48 mantissa bits: every value is a multiple of 2^-48
    assert np.all(np.ldexp(r, 48) == np.floor(np.ldexp(r, 48)))


def test_sp_init_invariants(oracle_mod):
    m = oracle_mod.OracleModel()
    st = m.sp_state()
    pot, perm, conn = st["potential"], st["perm"], st["connected"]
    assert np.all(pot.sum(1) == 400)            # round(500 * 0.8)
    assert np.all(perm[pot == 0] == 0)
    assert perm.min() >= 0 and perm.max() <= 1
    assert np.array_equal(conn, (perm >= np.float32(0.1) - np.float32(1e-6)).astype(np.uint8))
    # initPermanence_ truncation to 5 decimals
    nz = perm[perm > 0].astype(np.float64)
    assert np.allclose(np.round(nz * 1e5), nz * 1e5, atol=1e-2)
    # about half the potential synapses start connected
    assert 0.45 < conn.sum() / pot.sum() < 0.55


def test_sp_inhibition_tie_break_highest_index(oracle_mod):
    # all-zero input: every overlap is 0 (stimulusThreshold 0 keeps them
    # eligible) and ties go to the highest column indices
    m = oracle_mod.OracleModel()
    m.step([float("nan")], False, False)
    assert np.array_equal(m.active_columns(), np.arange(2008, 2048))


def test_sp_always_40_and_learning_touches_active_only(oracle_mod):
    m = oracle_mod.OracleModel()
    before = m.sp_state()["perm"].copy()
    m.step([42.0], True, False)
    act = m.active_columns()
    assert len(act) == 40
    after = m.sp_state()["perm"]
    changed = np.nonzero((after != before).any(1))[0]
    assert set(changed.tolist()) <= set(act.tolist())
    ov = m.sp_overlaps()
    # winners have the 40 largest overlaps
    assert ov[act].min() >= np.sort(ov)[-40]


def test_sp_duty_cycles_formula(oracle_mod):
    m = oracle_mod.OracleModel()
    odc = np.zeros(2048, np.float32)
    adc = np.zeros(2048, np.float32)
    for it, x in enumerate([10.0, 20.0, 30.0, 20.0, 10.0], start=1):
        m.step([x], True, False)
        ov = (m.sp_overlaps() > 0).astype(np.float32)
        ac = np.zeros(2048, np.float32)
        ac[m.active_columns()] = 1
        p = np.float32(min(1000, it))
        odc = (odc * (p - np.float32(1)) + ov) / p
        adc = (adc * (p - np.float32(1)) + ac) / p
        st = m.sp_state()
        assert np.array_equal(st["overlap_dc"], odc)
        assert np.array_equal(st["active_dc"], adc)


def test_raw_anomaly_is_k_over_40(oracle_mod):
    m = oracle_mod.OracleModel()
    for x in [5.0, 10.0, 15.0, 10.0, 5.0, 10.0, 15.0, 10.0, 5.0] * 3:
        s = m.step([x], True, True)
        k = round(float(s) * 40)
        assert s == np.float32((40 - (40 - k)) / 40.0) or s == np.float32(k / 40.0)


def test_tm_learns_a_repeating_sequence(oracle_mod):
    m = oracle_mod.OracleModel()
    seq = [10.0, 30.0, 50.0, 70.0, 90.0]
    scores = [float(m.step([x], True, True)) for x in seq * 40]
    assert scores[0] == 1.0
    assert max(scores[-10:]) <= 0.1    # (nearly) fully predicted after learning
    segs = m.tm_segments(32)
    assert np.all(segs["nsyn"] <= 32)
    assert segs["perm"].max() <= 1.0 and segs["perm"].min() >= 0.0
    sc = m.tm_scalars()
    assert sc["lrn_iter"] == 200 and sc["n_prev_inf"] <= 11 and sc["n_prev_lrn"] <= 6


def test_tm_learning_off_keeps_segments(oracle_mod):
    m = oracle_mod.OracleModel()
    for x in [10.0, 30.0, 50.0] * 10:
        m.step([x], True, True)
    before = m.tm_segments(32)
    for x in [10.0, 30.0, 50.0, 70.0] * 3:
        m.step([x], True, False)
    after = m.tm_segments(32)
    for k in ["cell", "nsyn", "src", "perm", "pos_act"]:
        assert np.array_equal(before[k], after[k])


def test_tm_reset_clears_states(oracle_mod):
    m = oracle_mod.OracleModel()
    for x in [10.0, 30.0, 50.0] * 5:
        m.step([x], True, True)
    m.tm_reset()
    st = m.tm_states()
    assert all(v.sum() == 0 for v in st.values())
    assert m.tm_scalars()["n_prev_inf"] == 0
    m.step([10.0], True, True)
    # after a reset only start cells (cell 0) of the active columns fire
    ia = m.tm_states()["inf_active"].reshape(2048, 12)
    assert ia[:, 1:].sum() == 0 and ia[:, 0].sum() == 40


def test_clone_is_independent(oracle_mod):
    m = oracle_mod.OracleModel()
    for x in [10.0, 30.0, 50.0] * 5:
        m.step([x], True, True)
    c = m.clone()
    a = [float(m.step([x], True, True)) for x in [10.0, 30.0, 50.0, 11.0]]
    b = [float(c.step([x], True, True)) for x in [10.0, 30.0, 50.0, 11.0]]
    assert a == b
