"""Batched HTM engine: N Model-1 streams stepped in lockstep on one MI355X.

Thin Python owner of a `htm_engine*` (include/htm_amd.h).  Device buffers for
inputs/scores are torch tensors (PyTorch-ROCm is the plumbing); every
computation runs in the HIP kernels of libhtm_amd.so.

Reference: one NuPIC `Network` per stream, driven by
ML/HTM/NetworkModel.py:35-157 (runNetwork/run) from ModelTraining.py /
ModelTesting.py; this engine replaces that per-stream loop.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import OUT, ST, HtmConfig, TmHeader, TmUpdate, check


class HTMEngine:
    """N independent encoder->SP->TM->anomaly streams on one GPU.

    >>> eng = HTMEngine(1024)                       # reference Model-1 params
    >>> scores = eng.step(torch.full((1024,), 42.0, device="cuda", dtype=torch.float64))
    """

    def __init__(self, n_streams: int, config: HtmConfig | None = None, device: int | None = None,
                 _handle=None, **overrides):
        self._L = _lib.lib()
        self.device = torch.cuda.current_device() if device is None else int(device)
        if _handle is not None:
            self.h = _handle
        else:
            cfg = config if config is not None else _lib.default_config(**overrides)
            h = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                check(self._L.htm_create(ctypes.byref(cfg), int(n_streams), self.device, ctypes.byref(h)))
            self.h = h
        cfg = HtmConfig()
        check(self._L.htm_get_config(self.h, ctypes.byref(cfg)))
        self.config = cfg
        self.n_streams = self._L.htm_n_streams(self.h)
        self.n_fields = cfg.n_fields
        self.n_columns = cfg.sp_columns
        self.cells_per_column = cfg.tm_cells_per_col
        self.n_cells = cfg.sp_columns * cfg.tm_cells_per_col
        self.sdr_bits = cfg.sdr_bits        # > 0: the SP reads an input SDR (step_sdr / run_sdr)
        self.sdr_words = (cfg.sdr_bits + 31) // 32
        self.sp_learn = True
        self.tm_learn = True
        # the engine's default (HTM_OPT_FUSED on); SDR-input engines always run unfused
        self.fused = not self.sdr_bits
        self.is_fleet = bool(self._L.htm_is_fleet(self.h))
        if self.is_fleet:
            self.sp_learn = self.tm_learn = False

    @classmethod
    def fleet(cls, model: "HTMEngine", n_streams: int, model_stream: int = 0, q_capacity: int = 8192,
              device: int | None = None) -> "HTMEngine":
        """Fleet mode (config 4): n_streams streams sharing the frozen SP+TM model
        of `model`'s stream `model_stream`, each with its own TM state."""
        L = _lib.lib()
        dev = model.device if device is None else int(device)
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(L.htm_create_fleet(model.h, int(model_stream), int(n_streams), int(q_capacity), dev,
                                     ctypes.byref(h)))
        return cls(0, device=dev, _handle=h)

    def _model_index(self, s: int) -> int:
        """instance of the model regions stream s reads (fleet: the shared one)"""
        return 0 if self.is_fleet else s

    # ------------------------------------------------------------------ life
    def close(self):
        if getattr(self, "h", None):
            self._L.htm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------- controls
    def set_learning(self, sp: bool, tm: bool):
        """SPRegion / TMRegion setParameter('learningMode', ...) (independent)."""
        check(self._L.htm_set_learning(self.h, int(bool(sp)), int(bool(tm))))
        self.sp_learn, self.tm_learn = bool(sp), bool(tm)

    def set_option(self, opt: int, value: int):
        check(self._L.htm_set_option(self.h, int(opt), int(value)))

    def use_frozen_index(self, on: bool):
        self.set_option(_lib.OPT_FROZEN_INDEX, int(on))

    def keep_prev_predicted(self, on: bool):
        self.set_option(_lib.OPT_KEEP_PREV, int(on))

    def tm_reset(self):
        check(self._L.htm_reset_tm(self.h, self._stream()))

    def status(self):
        """Synchronise and raise on any per-stream capacity overflow."""
        check(self._L.htm_status(self.h))

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ----------------------------------------------------------------- steps
    def _values(self, values) -> torch.Tensor:
        if not isinstance(values, torch.Tensor):
            values = torch.as_tensor(np.asarray(values, dtype=np.float64))
        v = values.to(device=f"cuda:{self.device}", dtype=torch.float64).contiguous()
        return v

    def step(self, values, out: torch.Tensor | None = None) -> torch.Tensor:
        """One network.run(1) for every stream; returns float32 anomaly scores [N]."""
        v = self._values(values)
        if v.numel() != self.n_streams * self.n_fields:
            raise ValueError(f"expected {self.n_streams * self.n_fields} values, got {v.numel()}")
        if out is None:
            out = torch.empty(self.n_streams, dtype=torch.float32, device=v.device)
        check(self._L.htm_step(self.h, ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                               self._stream()))
        return out

    def run(self, values, out: torch.Tensor | None = None) -> torch.Tensor:
        """values [T, N(, F)] -> scores [T, N]."""
        v = self._values(values)
        T = v.shape[0]
        if v.numel() != T * self.n_streams * self.n_fields:
            raise ValueError("values must be [T, n_streams(, n_fields)]")
        if out is None:
            out = torch.empty((T, self.n_streams), dtype=torch.float32, device=v.device)
        check(self._L.htm_run(self.h, T, ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                              self._stream()))
        return out

    def _sdr(self, sdr) -> torch.Tensor:
        if not isinstance(sdr, torch.Tensor):
            sdr = torch.as_tensor(np.ascontiguousarray(np.asarray(sdr, dtype=np.uint32)).view(np.int32))
        if sdr.dtype not in (torch.int32, torch.uint32):
            raise TypeError("input SDRs are uint32/int32 word bitmaps [..., n_streams, ceil(sdr_bits/32)]")
        return sdr.to(device=f"cuda:{self.device}").contiguous()

    def step_sdr(self, sdr, out: torch.Tensor | None = None) -> torch.Tensor:
        """One network.run(1) of an SDR-fed level (the L2 SPRegion + TMRegion of
        Models 2/3): sdr is the [N, ceil(sdr_bits/32)] word bitmap the level below
        produced, e.g. ``l1.get_output("tm_output")`` (bit i of word w = element
        32*w + i of the L1 TMRegion bottomUpOut).  Returns anomaly scores [N]."""
        if not self.sdr_bits:
            raise ValueError("this engine reads encoder values: use step()")
        x = self._sdr(sdr)
        if x.numel() != self.n_streams * self.sdr_words:
            raise ValueError(f"expected {self.n_streams} x {self.sdr_words} words, got {tuple(x.shape)}")
        if out is None:
            out = torch.empty(self.n_streams, dtype=torch.float32, device=x.device)
        check(self._L.htm_step_sdr(self.h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                   self._stream()))
        return out

    def run_sdr(self, sdr, out: torch.Tensor | None = None) -> torch.Tensor:
        """sdr [T, N, words] -> scores [T, N]."""
        if not self.sdr_bits:
            raise ValueError("this engine reads encoder values: use run()")
        x = self._sdr(sdr)
        T = x.shape[0]
        if x.numel() != T * self.n_streams * self.sdr_words:
            raise ValueError("sdr must be [T, n_streams, ceil(sdr_bits/32)]")
        if out is None:
            out = torch.empty((T, self.n_streams), dtype=torch.float32, device=x.device)
        check(self._L.htm_run_sdr(self.h, T, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                  self._stream()))
        return out

    # --------------------------------------------------------------- outputs
    def get_output(self, name: str) -> torch.Tensor:
        """region.getOutputData(...) for every stream (device tensor)."""
        which = OUT[name]
        per = self._L.htm_output_bytes(self.h, which)
        dtype = {"active_columns": torch.uint8, "prev_pred_columns": torch.uint8, "pred_columns": torch.uint8,
                 "col_confidence": torch.float32, "sp_overlaps": torch.int32}.get(name, torch.int32)
        esz = torch.tensor([], dtype=dtype).element_size()
        out = torch.empty((self.n_streams, per // esz), dtype=dtype, device=f"cuda:{self.device}")
        check(self._L.htm_get_output(self.h, which, ctypes.c_void_p(out.data_ptr()), per * self.n_streams,
                                     self._stream()))
        return out

    def bitmap_to_dense(self, words: torch.Tensor) -> np.ndarray:
        """uint32 cell bitmaps [N, cells/32] -> uint8 [N, cells]."""
        w = words.detach().cpu().numpy().astype(np.uint32).view(np.uint8)
        bits = np.unpackbits(w.reshape(w.shape[0], -1), axis=1, bitorder="little")
        return bits[:, : self.n_cells]

    # ----------------------------------------------------------------- state
    def state_bytes(self, region: str) -> int:
        return self._L.htm_state_bytes(self.h, ST[region])

    def export_state(self, region: str, s0: int = 0, n: int | None = None) -> np.ndarray:
        n = self.n_streams - s0 if n is None else n
        per = self.state_bytes(region)
        buf = np.zeros(per * n, np.uint8)
        check(self._L.htm_export_state(self.h, ST[region], s0, n, buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes))
        return buf.reshape(n, per)

    def import_state(self, region: str, data: np.ndarray, s0: int = 0):
        data = np.ascontiguousarray(data)
        per = self.state_bytes(region)
        if region == "sp_perm_ckpt" and (per == 0 or data.nbytes == 0):
            return  # SP checkpoints exist only in paged engines: none given or none held, keep the stream's own
        if per == 0:
            return  # a region this engine does not hold (e.g. RDSE state of a ScalarEncoder engine)
        n = data.nbytes // per
        check(self._L.htm_import_state(self.h, ST[region], s0, n, data.ctypes.data_as(ctypes.c_void_p), data.nbytes))

    def tm_header(self, s: int) -> TmHeader:
        raw = self.export_state("tm_header", s, 1)[0]
        return TmHeader.from_buffer_copy(raw.tobytes())

    def replicate(self, src: int = 0):
        """Copy stream `src` into every stream (config-2 setup)."""
        check(self._L.htm_replicate_stream(self.h, int(src), self._stream()))

    def device_bytes(self) -> int:
        return self._L.htm_device_bytes(self.h)

    def flush(self):
        """Complete the deferred dutyCycle() writes of lockstep steps
        (HTM_OPT_DEFER_DUTY) on the current stream (asynchronous)."""
        check(self._L.htm_flush(self.h, self._stream()))

    def defer_duty(self, on: bool):
        check(self._L.htm_set_option(self.h, _lib.OPT_DEFER_DUTY, int(on)))

    def flush_mode(self, mode: int):
        """Where the deferred-write flush runs: 0 beside the next steps on the
        engine's own HIP stream, 1 on the step stream; results identical."""
        check(self._L.htm_set_option(self.h, _lib.OPT_FLUSH_MODE, int(mode)))

    def flush_every(self, steps: int):
        """Lockstep steps between periodic flushes of the deferred dutyCycle()
        writes (HTM_OPT_FLUSH_EVERY; 0 = default)."""
        check(self._L.htm_set_option(self.h, _lib.OPT_FLUSH_EVERY, int(steps)))

    def split_learning(self, on: bool):
        """Learning lockstep steps run the SP kernel, then the TM-only learning
        kernel (HTM_OPT_SPLIT_LEARN, default on); results are identical."""
        check(self._L.htm_set_option(self.h, _lib.OPT_SPLIT_LEARN, int(on)))

    def ordered_steps(self, on: bool):
        """Frozen lockstep steps run their TM steps heaviest first
        (HTM_OPT_ORDERED, default on); results are identical either way."""
        check(self._L.htm_set_option(self.h, _lib.OPT_ORDERED, int(on)))

    def sp_perm_rows_used(self) -> int:
        """Paged SP permanences: pool rows handed out (0 for a dense engine)."""
        return int(self._L.htm_sp_perm_rows_used(self.h))

    def profile(self, on, every: int = 1):
        """Bracket the SP and TM kernels of every `every`-th launch with HIP
        events (profile_read averages the sampled launches)."""
        self.set_option(_lib.OPT_PROFILE, int(every) if on else 0)

    def profile_read(self) -> dict:
        """{sp_ms, tm_ms (fused launches: SP+TM), steps covered, launches}."""
        out = (ctypes.c_double * 4)()
        check(self._L.htm_profile_read(self.h, out))
        return dict(sp_ms=out[0], tm_ms=out[1], steps=int(out[2]), launches=int(out[3]))

    def use_fused(self, on: bool):
        """One fused SP+TM kernel per step / per htm_run chunk (default on)."""
        self.set_option(_lib.OPT_FUSED, int(on))
        self.fused = bool(on)

    def set_run_chunk(self, steps: int):
        """Steps per fused htm_run launch."""
        self.set_option(_lib.OPT_RUN_CHUNK, int(steps))

    def set_run_unit(self, steps: int):
        """Steps per work-queue unit of a fused htm_run launch (a stream's TM
        state stays in LDS across a unit)."""
        self.set_option(_lib.OPT_RUN_UNIT, int(steps))

    def counters(self) -> dict:
        out = (ctypes.c_uint64 * 8)()
        check(self._L.htm_counters(self.h, out))
        keys = ["tm_bytes", "inf_phase2", "inf_backtracks", "lrn_phase2", "lrn_backtracks", "seg_live",
                "seg_hwm", "error"]
        return {k: int(v) for k, v in zip(keys, out)}

    def debug_stamps(self) -> dict:
        """Per-phase TM cycle stamps + event counts (diagnostic stamps build only);
        "tail": the same over stream-steps whose TM part took >= 2^18 cycles."""
        N = 32
        out = (ctypes.c_uint64 * (4 * N))()
        check(self._L.htm_debug_stamps(self.h, out))
        names = ["load", "phase1", "list", "win_pre", "stream", "qscan", "fin1", "fin2", "backtrack", "learn", "wb",
                 "scan", "sort", "sums", "owner", "sload", "count", "fclr", "pred_cols", "defer", "sp", "norm",
                 "learn_scan", "learn_updates", "learn_wave0", "learn_bt_copy", "compact", "sp_learn",
                 "lw_build", "lw_draws", "lw_writes", "norm_compact"]
        cnames = {0: "phase2", 1: "windows", 2: "blocks", 3: "qualifying", 4: "active_cells", 5: "nonzero_cols",
                  6: "steps", 16: "pool_scans", 17: "pool_scan_slots", 18: "sp_row_replays",
                  19: "sp_row_replay_cycles", 20: "sp_row_replay_sample_cycles", 21: "sp_row_replay_skip_cycles",
                  22: "lp1_columns", 23: "lp2_columns", 24: "lw_samples", 25: "lw_sample_draws",
                  26: "lw_sample_cycles", 27: "lw_blocks_approx"}

        def part(o):
            return dict(cycles={k: int(out[o + i]) for i, k in enumerate(names)},
                        counts={k: int(out[o + N + i]) for i, k in cnames.items()},
                        step_cycle_hist={f"<2^{16 + b}" if b < 8 else ">=2^23": int(out[o + N + 7 + b])
                                         for b in range(9)})
        r = part(0)
        r["tail"] = part(2 * N)
        return r

    def frozen_index_valid(self) -> bool:
        return bool(self._L.htm_frozen_index_valid(self.h))

    # -------------------------------------------------------------- save/load
    def save(self, path: str):
        check(self._L.htm_save(self.h, path.encode()))

    @classmethod
    def load(cls, path: str, device: int | None = None) -> "HTMEngine":
        L = _lib.lib()
        dev = torch.cuda.current_device() if device is None else int(device)
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(L.htm_load(path.encode(), dev, ctypes.byref(h)))
        return cls(0, device=dev, _handle=h)

    # ------------------------------------------------- canonical state views
    def sp_state(self, s: int) -> dict:
        """SP state of stream s in the oracle's dense layout."""
        c = self.config
        nin = c.sdr_bits if c.sdr_bits else c.n_fields * c.enc_n
        nin_pad = (nin + 31) // 32 * 32
        nw = c.sp_columns // 32
        pot_words = self.export_state("sp_potmask", self._model_index(s), 1)[0].view(np.uint32).reshape(c.sp_columns, nin_pad // 32)
        pot = np.unpackbits(pot_words.view(np.uint8).reshape(c.sp_columns, -1), axis=1, bitorder="little")[:, :nin]
        packed = self.export_state("sp_perm", self._model_index(s), 1)[0].view(np.float32).reshape(c.sp_columns, -1)
        perm = np.zeros((c.sp_columns, nin), np.float32)
        for col in range(c.sp_columns):
            idx = np.nonzero(pot[col])[0]
            perm[col, idx] = packed[col, : len(idx)]
        connT = self.export_state("sp_connT", self._model_index(s), 1)[0].view(np.uint32).reshape(nin_pad, nw)
        conn = np.unpackbits(connT.view(np.uint8).reshape(nin_pad, -1), axis=1, bitorder="little")[:nin, :c.sp_columns]
        duty = self.export_state("sp_duty", self._model_index(s), 1)[0].view(np.float32).reshape(2, c.sp_columns)
        sc = self.export_state("sp_scalars", s, 1)[0].view(np.uint32)
        boost = self.export_state("sp_boost", self._model_index(s), 1)[0].view(np.float32).copy()
        return dict(perm=perm, potential=pot.astype(np.uint8), connected=conn.T.copy().astype(np.uint8),
                    overlap_dc=duty[0].copy(), active_dc=duty[1].copy(), boost=boost,
                    min_overlap_dc=np.float32(sc[2:3].view(np.float32)[0]), iter=int(sc[0]), iter_learn=int(sc[1]))

    def rdse_state(self, s: int, f: int = 0) -> dict:
        """RDSE encoder state of field f of stream s in the layout of
        oracle.OracleModel.rdse_state (bucket map rows outside the index range
        zero)."""
        c = self.config
        if c.enc_type != _lib.ENC_RDSE:
            raise ValueError("not an RDSE engine")
        raw = self.export_state("enc_rdse", s, 1)[0]
        blk = len(raw) // c.n_fields
        b = raw[f * blk:(f + 1) * blk]
        h = b[:256].view(np.int32)
        m = b[256:256 + _lib.RDSE_BUCKETS * c.enc_w * 2].view(np.int16).reshape(_lib.RDSE_BUCKETS, c.enc_w)
        lo, hi = int(h[0]), int(h[1])
        rows = np.zeros((_lib.RDSE_BUCKETS, c.enc_w), np.int32)
        rows[lo:hi + 1] = m[lo:hi + 1]
        return dict(min_idx=lo, max_idx=hi, has_offset=int(h[2]), num_tries=int(h[3]),
                    offset=float(h[4:6].view(np.float64)[0]), map=rows)

    def tm_segments(self, s: int) -> dict:
        """Live segments of stream s in canonical (cell, creation) order, the
        layout of oracle.OracleModel.tm_segments(32)."""
        meta = self.export_state("tm_seg_meta", self._model_index(s), 1)[0].view(np.uint32)
        hdr = self.tm_header(s)
        hwm = hdr.seg_hwm
        meta = meta[:hwm]
        live = ((meta >> 23) & 1).astype(bool)
        slots = np.nonzero(live)[0]
        cell = (meta[slots] & 0xFFFF).astype(np.int64)
        order = np.lexsort((slots, cell))
        slots = slots[order]
        m = meta[slots]
        src = self.export_state("tm_seg_src", self._model_index(s), 1)[0].view(np.uint16).reshape(-1, 32)[slots].astype(np.int32)
        perm = self.export_state("tm_seg_perm", self._model_index(s), 1)[0].view(np.float32).reshape(-1, 32)[slots]
        duty = self.export_state("tm_seg_duty", self._model_index(s), 1)[0].view(np.uint32).reshape(-1, 3)[slots]
        nsyn = ((m >> 16) & 0x3F).astype(np.int32)
        mask = np.arange(32)[None, :] < nsyn[:, None]
        return dict(cell=(m & 0xFFFF).astype(np.int32), is_seq=((m >> 22) & 1).astype(np.int32),
                    pos_act=duty[:, 0].astype(np.int32), last_dc_iter=duty[:, 2].astype(np.int32), nsyn=nsyn,
                    last_dc=duty[:, 1].copy().view(np.float32), src=np.where(mask, src, 0),
                    perm=np.where(mask, perm, np.float32(0)), slots=slots)

    def tm_states(self, s: int) -> dict:
        c = self.config
        cw = self.n_cells // 32
        bm = self.export_state("tm_bitmaps", s, 1)[0].view(np.uint32).reshape(4, cw)
        dense = np.unpackbits(bm.view(np.uint8).reshape(4, -1), axis=1, bitorder="little")[:, : self.n_cells]
        return dict(inf_active=dense[0], inf_pred=dense[1], lrn_active=dense[2], lrn_pred=dense[3])

    def col_confidence(self, s: int) -> np.ndarray:
        return self.export_state("tm_colconf", s, 1)[0].view(np.float32).copy()

    def tm_patterns(self, s: int) -> tuple[list, list]:
        hdr = self.tm_header(s)
        pat = self.export_state("tm_patterns", s, 1)[0].view(np.uint16).reshape(2, 16, 64)
        inf = [pat[0][(hdr.inf_pat_head + k) % 16][: hdr.inf_pat_len[(hdr.inf_pat_head + k) % 16]].tolist()
               for k in range(hdr.n_inf_pat)]
        lrn = [pat[1][(hdr.lrn_pat_head + k) % 16][: hdr.lrn_pat_len[(hdr.lrn_pat_head + k) % 16]].tolist()
               for k in range(hdr.n_lrn_pat)]
        return inf, lrn

    def tm_updates(self, s: int) -> list:
        hdr = self.tm_header(s)
        raw = self.export_state("tm_updates", s, 1)[0]
        n = hdr.n_upd
        arr = (TmUpdate * (len(raw) // ctypes.sizeof(TmUpdate))).from_buffer_copy(raw.tobytes())
        return [arr[k] for k in range(n)]
