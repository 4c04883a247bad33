"""ctypes binding of libhtm_amd.so (the C ABI declared in include/htm_amd.h).

The shared library holds the HIP kernels for gfx950 and the host engine.
Loading fails loudly if it has not been built: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libhtm_amd.so")
# diagnostic build with per-phase cycle stamps (tools/ only): HTM_AMD_STAMPS=1
if os.environ.get("HTM_AMD_STAMPS") == "1":
    LIB_PATH = os.path.join(PKG_DIR, "libhtm_amd_stamps.so")
# A/B of two builds on one box (tools/ab_libs.py only): libhtm_amd_<variant>.so
if os.environ.get("HTM_AMD_LIB_VARIANT"):
    LIB_PATH = os.path.join(PKG_DIR, "libhtm_amd_%s.so" % os.environ["HTM_AMD_LIB_VARIANT"])
# experiment builds (make variant ...; tools/ only)
if os.environ.get("HTM_AMD_LIB"):
    LIB_PATH = os.path.join(PKG_DIR, os.environ["HTM_AMD_LIB"])
CSRC = os.path.join(PKG_DIR, "csrc")

HTM_OK = 0
HTM_E_INVALID = -1
HTM_E_HIP = -2
HTM_E_CAPACITY = -3
HTM_E_IO = -4
HTM_E_STATE = -5

OUT = dict(active_columns=1, prev_pred_columns=2, inf_active=3, inf_predicted=4, lrn_active=5,
           lrn_predicted=6, col_confidence=7, tm_output=8, sp_overlaps=9, buckets=10, pred_columns=11)
# sp_perm_ckpt first: a paged engine imports its permanences against the
# initial values of the checkpoints they came with (HTM_ST_SP_PERM_CKPT)
ST = dict(sp_perm_ckpt=17, sp_connT=1, sp_potmask=2, sp_perm=3, sp_duty=4, sp_scalars=5, tm_header=6, tm_bitmaps=7,
          tm_colconf=8, tm_seg_meta=9, tm_seg_src=10, tm_seg_perm=11, tm_seg_conn=12, tm_seg_duty=13,
          tm_cell_nseg=14, tm_patterns=15, tm_updates=16, sp_boost=18, enc_rdse=19)
ENC_SCALAR, ENC_RDSE = 0, 1
RDSE_BUCKETS = 1000
OPT_FROZEN_INDEX = 1
OPT_KEEP_PREV = 2
OPT_KEEP_OVERLAPS = 3
OPT_PROFILE = 4
OPT_FUSED = 5
OPT_RUN_CHUNK = 6
OPT_RUN_UNIT = 7
OPT_DEFER_DUTY = 10
OPT_FLUSH_MODE = 11
OPT_ORDERED = 12
OPT_FLUSH_EVERY = 13
OPT_SPLIT_LEARN = 14


class HtmConfig(ctypes.Structure):
    """Mirror of htm_config (include/htm_amd.h)."""
    _fields_ = [
        ("n_fields", ctypes.c_int32), ("enc_n", ctypes.c_int32), ("enc_w", ctypes.c_int32),
        ("enc_minval", ctypes.c_double), ("enc_maxval", ctypes.c_double), ("enc_clip", ctypes.c_int32),
        ("sp_columns", ctypes.c_int32), ("sp_num_active", ctypes.c_int32),
        ("sp_potential_pct", ctypes.c_float), ("sp_perm_connected", ctypes.c_float),
        ("sp_perm_active_inc", ctypes.c_float), ("sp_perm_inactive_dec", ctypes.c_float),
        ("sp_min_pct_overlap_dc", ctypes.c_float), ("sp_duty_cycle_period", ctypes.c_int32),
        ("sp_boost_strength", ctypes.c_float), ("sp_stimulus_threshold", ctypes.c_int32),
        ("sp_update_period", ctypes.c_int32), ("sp_seed", ctypes.c_uint64),
        ("tm_cells_per_col", ctypes.c_int32), ("tm_new_syn_count", ctypes.c_int32),
        ("tm_max_syn_per_seg", ctypes.c_int32), ("tm_max_segs_per_cell", ctypes.c_int32),
        ("tm_initial_perm", ctypes.c_float), ("tm_connected_perm", ctypes.c_float),
        ("tm_perm_inc", ctypes.c_float), ("tm_perm_dec", ctypes.c_float), ("tm_perm_max", ctypes.c_float),
        ("tm_min_threshold", ctypes.c_int32), ("tm_activation_threshold", ctypes.c_int32),
        ("tm_pam_length", ctypes.c_int32), ("tm_max_inf_backtrack", ctypes.c_int32),
        ("tm_max_lrn_backtrack", ctypes.c_int32), ("tm_max_seq_length", ctypes.c_int32),
        ("tm_seg_update_valid_duration", ctypes.c_int32), ("tm_seed", ctypes.c_uint64),
        ("seg_capacity", ctypes.c_int32), ("upd_capacity", ctypes.c_int32), ("seed_stride", ctypes.c_int32),
        ("sdr_bits", ctypes.c_int32),
        ("field_minval", ctypes.c_double * 4), ("field_maxval", ctypes.c_double * 4),
        ("sp_perm_rows", ctypes.c_int32), ("reserved0", ctypes.c_int32),
        ("enc_type", ctypes.c_int32), ("reserved1", ctypes.c_int32), ("rdse_resolution", ctypes.c_double),
        ("rdse_seed", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: (list(v) if isinstance(v, ctypes.Array) else v)
                for k, v in ((k, getattr(self, k)) for k, _ in self._fields_)}


class TmHeader(ctypes.Structure):
    """Mirror of htm_tm_header."""
    _fields_ = [
        ("lrn_iter", ctypes.c_uint32), ("iter", ctypes.c_uint32),
        ("pam_counter", ctypes.c_int32), ("learned_seq_length", ctypes.c_int32),
        ("reset_called", ctypes.c_int32), ("have_avg_density", ctypes.c_int32),
        ("avg_input_density", ctypes.c_double), ("avg_learned_seq_length", ctypes.c_double),
        ("rng_state", ctypes.c_uint32 * 31), ("rng_f", ctypes.c_int32), ("rng_r", ctypes.c_int32),
        ("seg_hwm", ctypes.c_uint32), ("seg_live", ctypes.c_uint32),
        ("n_inf_pat", ctypes.c_int32), ("n_lrn_pat", ctypes.c_int32),
        ("inf_pat_len", ctypes.c_uint16 * 16), ("lrn_pat_len", ctypes.c_uint16 * 16),
        ("n_upd", ctypes.c_int32), ("error", ctypes.c_uint32),
        ("stat_inf_phase2", ctypes.c_uint32), ("stat_inf_backtrack", ctypes.c_uint32),
        ("stat_lrn_phase2", ctypes.c_uint32), ("stat_lrn_backtrack", ctypes.c_uint32),
        ("inf_pat_head", ctypes.c_uint16), ("lrn_pat_head", ctypes.c_uint16), ("lp2_pending", ctypes.c_uint32),
        ("stat_bytes", ctypes.c_uint64),
    ]


class TmUpdate(ctypes.Structure):
    """Mirror of htm_tm_update."""
    _fields_ = [("slot", ctypes.c_uint32), ("col", ctypes.c_uint16), ("cell", ctypes.c_uint8),
                ("n_new", ctypes.c_uint8), ("active_mask", ctypes.c_uint32), ("date", ctypes.c_uint32),
                ("new_src", ctypes.c_uint16 * 32)]


EXPORTED = [
    "htm_default_config", "htm_create", "htm_destroy", "htm_set_learning", "htm_set_option", "htm_status",
    "htm_step", "htm_run", "htm_step_sdr", "htm_run_sdr", "htm_get_output", "htm_output_bytes", "htm_state_bytes", "htm_export_state",
    "htm_import_state", "htm_reset_tm", "htm_save", "htm_load", "htm_replicate_stream", "htm_n_streams",
    "htm_get_config", "htm_device_bytes", "htm_sp_perm_rows_used", "htm_frozen_index_valid", "htm_last_error", "htm_abi_version",
    "htm_profile_read", "htm_counters", "htm_debug_stamps", "htm_build_info",
    "htm_slo_create", "htm_slo_destroy", "htm_slo_record", "htm_slo_stats", "htm_create_fleet", "htm_is_fleet", "htm_flush",
    "htm_likelihood_create", "htm_likelihood_destroy", "htm_likelihood_step",
    "htm_cls_create", "htm_cls_destroy", "htm_cls_compute", "htm_cls_status", "htm_cls_state_bytes",
    "htm_cls_export_state", "htm_cls_import_state",
]

_lib = None


def build(force: bool = False) -> str:
    """Compile libhtm_amd.so for gfx950 with hipcc (works without a GPU)."""
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h"))]
    newest = max(os.path.getmtime(s) for s in srcs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        jobs = str(min(8, os.cpu_count() or 1))
        subprocess.run(["make", "-C", CSRC, "-j", jobs], check=True)
    return LIB_PATH


class HtmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"htm error {code}: {msg}")
        self.code = code


def lib():
    """Load the HIP engine.  Raises if the library is missing: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    # torch's HIP runtime must be the one the engine binds to (same soname):
    # import torch first so a single libamdhip64 serves both.
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t
    P = ctypes.POINTER
    L.htm_default_config.argtypes = [P(HtmConfig)]
    L.htm_create.argtypes = [P(HtmConfig), i32, i32, P(vp)]
    L.htm_destroy.argtypes = [vp]
    L.htm_set_learning.argtypes = [vp, i32, i32]
    L.htm_set_option.argtypes = [vp, i32, i32]
    L.htm_status.argtypes = [vp]
    L.htm_step.argtypes = [vp, vp, vp, vp]
    L.htm_run.argtypes = [vp, i32, vp, vp, vp]
    L.htm_step_sdr.argtypes = [vp, vp, vp, vp]
    L.htm_run_sdr.argtypes = [vp, i32, vp, vp, vp]
    L.htm_get_output.argtypes = [vp, i32, vp, sz, vp]
    L.htm_output_bytes.argtypes = [vp, i32]
    L.htm_output_bytes.restype = sz
    L.htm_state_bytes.argtypes = [vp, i32]
    L.htm_state_bytes.restype = sz
    L.htm_export_state.argtypes = [vp, i32, i32, i32, vp, sz]
    L.htm_import_state.argtypes = [vp, i32, i32, i32, vp, sz]
    L.htm_reset_tm.argtypes = [vp, vp]
    L.htm_save.argtypes = [vp, ctypes.c_char_p]
    L.htm_load.argtypes = [ctypes.c_char_p, i32, P(vp)]
    L.htm_replicate_stream.argtypes = [vp, i32, vp]
    L.htm_n_streams.argtypes = [vp]
    L.htm_n_streams.restype = i32
    L.htm_get_config.argtypes = [vp, P(HtmConfig)]
    L.htm_device_bytes.argtypes = [vp]
    L.htm_device_bytes.restype = sz
    L.htm_sp_perm_rows_used.argtypes = [vp]
    L.htm_sp_perm_rows_used.restype = ctypes.c_uint64
    L.htm_frozen_index_valid.argtypes = [vp]
    L.htm_frozen_index_valid.restype = i32
    L.htm_last_error.restype = ctypes.c_char_p
    L.htm_abi_version.restype = i32
    L.htm_build_info.restype = ctypes.c_char_p
    L.htm_profile_read.argtypes = [vp, P(ctypes.c_double)]
    L.htm_counters.argtypes = [vp, P(ctypes.c_uint64)]
    L.htm_debug_stamps.argtypes = [vp, P(ctypes.c_uint64)]
    L.htm_create_fleet.argtypes = [vp, i32, i32, i32, i32, P(vp)]
    L.htm_flush.argtypes = [vp, vp]
    L.htm_is_fleet.argtypes = [vp]
    L.htm_is_fleet.restype = i32
    L.htm_likelihood_create.argtypes = [i32, i32, i32, i32, i32, i32, P(vp)]
    L.htm_likelihood_destroy.argtypes = [vp]
    L.htm_likelihood_step.argtypes = [vp, vp, i32, vp, vp, vp]
    L.htm_cls_create.argtypes = [i32, i32, i32, P(i32), i32, ctypes.c_double, ctypes.c_double, i32, P(vp)]
    L.htm_cls_destroy.argtypes = [vp]
    L.htm_cls_compute.argtypes = [vp, vp, vp, vp, i32, i32, vp, vp, vp]
    L.htm_cls_status.argtypes = [vp, P(i32)]
    L.htm_cls_state_bytes.argtypes = [vp, i32]
    L.htm_cls_state_bytes.restype = ctypes.c_size_t
    L.htm_cls_export_state.argtypes = [vp, i32, i32, i32, vp, ctypes.c_size_t]
    L.htm_cls_import_state.argtypes = [vp, i32, i32, i32, vp, ctypes.c_size_t]
    L.htm_slo_create.argtypes = [i32, ctypes.c_double, i32, i32, i32, P(vp)]
    L.htm_slo_destroy.argtypes = [vp]
    L.htm_slo_record.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    L.htm_slo_stats.argtypes = [vp, P(ctypes.c_int64), vp]
    _lib = L
    return L


def build_info() -> dict:
    """{translation unit: optimisation level} of the loaded library, plus
    "compiler" / "arch" (htm_build_info; csrc/cc.sh records the levels)."""
    raw = lib().htm_build_info().decode()
    out = {}
    for part in raw.split(";"):
        part = part.strip()
        if not part:
            continue
        if part.startswith("HIP version") or part.startswith("hipcc"):
            out["compiler"] = part
        elif part.startswith("arch "):
            out["arch"] = part[5:]
        else:
            unit, _, lvl = part.rpartition(" ")
            out[unit] = lvl
    return out


def check(code: int):
    if code != HTM_OK:
        raise HtmError(code, lib().htm_last_error().decode(errors="replace"))


# The reference's unused OPF parameter set, ML/HTM/params/model.yaml: the
# RandomDistributedScalarEncoder (:15-21; NuPIC defaults w 21, n 400 -- OPF
# sets the SP inputWidth to the encoder's width), SP (:28-41) with
# boostStrength 3.0, and the 32-cell BacktrackingTM (:45-63)
MODEL_YAML = dict(enc_type=ENC_RDSE, enc_n=400, enc_w=21, rdse_resolution=0.88, rdse_seed=1,
                  sp_seed=1956, sp_potential_pct=0.85, sp_perm_active_inc=0.04, sp_perm_inactive_dec=0.005,
                  sp_boost_strength=3.0, tm_cells_per_col=32, tm_seed=1960, tm_activation_threshold=16,
                  tm_min_threshold=12, tm_pam_length=1)


def model_yaml_config(**overrides) -> HtmConfig:
    kw = dict(MODEL_YAML)
    kw.update(overrides)
    return default_config(**kw)


def default_config(**overrides) -> HtmConfig:
    cfg = HtmConfig()
    lib().htm_default_config(ctypes.byref(cfg))
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise KeyError(f"unknown config field {k}")
        setattr(cfg, k, v)
    return cfg
