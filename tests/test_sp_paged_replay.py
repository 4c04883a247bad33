"""CPU check of the draw accounting the paged SP permanences rely on
(csrc/sp_dev.h sp_replay_init): a column's initial permanences
are recomputable from the nupic::Random stream alone once the draws before it
are counted -- 2 per column for the tieBreaker, then per column (wrap position
of its last potential input + 1) sampling draws, read off the potential mask,
and 4 per potential synapse.  Restated here in numpy against the oracle's
SpatialPooler initialisation (oracle/htm_oracle.c sp_init) for every column of
two seeds; the GPU replay itself is held to the dense engine by
tests/test_sp_paged.py."""
import numpy as np
import pytest

F32 = np.float32


def real64(lo, hi):
    return ((lo.astype(np.uint64) | (hi.astype(np.uint64) << np.uint64(32))) & np.uint64((1 << 48) - 1)).astype(
        np.float64) * (1.0 / 281474976710656.0)


def init_values(raw4):
    """sp_init_value for an [m, 4] array of raw draws (float32 arithmetic)."""
    conn, span, trim = F32(0.1), F32(1.0) - F32(0.1), F32(np.float64(F32(0.0001)) / 2.0)
    u1, u2 = real64(raw4[:, 0], raw4[:, 1]), real64(raw4[:, 2], raw4[:, 3])
    p = np.where(u1 <= 0.5, conn + (np.float64(span) * u2).astype(F32), conn * u2.astype(F32)).astype(F32)
    p = ((np.trunc(p * F32(100000.0)).astype(np.int32)).astype(np.float64) / 100000.0).astype(F32)
    p = np.where(p < trim, F32(0), p)
    return np.clip(p, F32(0), F32(1)).astype(F32)


@pytest.mark.parametrize("seed", [2045, 2045 + 65535])
def test_initial_permanences_from_counted_draws(oracle_mod, seed):
    m = oracle_mod.OracleModel(sp_seed=seed, tm_seed=seed)
    st = m.sp_state()
    pot, perm = st["potential"].astype(bool), st["perm"]
    ncol, nin = pot.shape
    raw = oracle_mod.rng_stream(seed, 2 * ncol + ncol * (nin + 4 * nin))
    pos = 2 * ncol  # tieBreaker_: one getReal64 (2 draws) per column
    for col in range(ncol):
        center = int(np.floor(F32((col + 0.5) * np.float64(F32(nin) / F32(ncol)))))
        wrap = (center % nin + np.arange(nin)) % nin  # WrappingNeighborhood order
        last = np.nonzero(pot[col][wrap])[0][-1]
        pos += last + 1  # sampling draws (the selection stops at the last chosen input)
        idx = np.nonzero(pot[col])[0]  # potential order = ascending input
        vals = init_values(raw[pos:pos + 4 * len(idx)].reshape(-1, 4))
        pos += 4 * len(idx)
        assert np.array_equal(vals, perm[col, idx]), f"column {col}"
