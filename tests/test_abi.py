"""The C-ABI library loads on a CPU-only host and exports every entry point
include/htm_amd.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "htm_amd.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(htm_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ["htm_create", "htm_destroy", "htm_step", "htm_set_learning", "htm_get_output",
                 "htm_save", "htm_load", "htm_last_error"]:
        assert must in fns


def test_library_exports_every_declared_symbol(rt):
    lib = ctypes.CDLL(rt._lib.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(rt._lib.EXPORTED) <= set(declared_functions())


def test_struct_layouts_match_the_header(rt, tmp_path):
    # compile a tiny C probe of the header's struct sizes/offsets with gcc
    src = tmp_path / "probe.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
        'int main(){printf("%%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(htm_config), sizeof(htm_tm_header),'
        ' sizeof(htm_tm_update), offsetof(htm_config, tm_seed), offsetof(htm_tm_header, inf_pat_head),'
        ' offsetof(htm_config, sdr_bits), offsetof(htm_config, sp_perm_rows));'
        'printf("%%zu %%zu\\n", offsetof(htm_config, enc_type), offsetof(htm_config, rdse_seed));}\n' % HEADER)
    exe = tmp_path / "probe"
    assert os.system(f"gcc {src} -o {exe}") == 0
    vals = [int(x) for x in os.popen(str(exe)).read().split()]
    L = rt._lib
    assert vals == [ctypes.sizeof(L.HtmConfig), ctypes.sizeof(L.TmHeader), ctypes.sizeof(L.TmUpdate),
                    L.HtmConfig.tm_seed.offset, L.TmHeader.inf_pat_head.offset, L.HtmConfig.sdr_bits.offset,
                    L.HtmConfig.sp_perm_rows.offset, L.HtmConfig.enc_type.offset, L.HtmConfig.rdse_seed.offset]


def test_default_config_is_the_reference_model1(rt):
    c = rt.default_config().as_dict()
    # NetworkUtils.py:26-64 and :77-88
    assert (c["enc_n"], c["enc_w"], c["enc_minval"], c["enc_maxval"], c["enc_clip"]) == (500, 21, 0.0, 100.0, 1)
    assert (c["sp_columns"], c["sp_num_active"], c["sp_seed"]) == (2048, 40, 2045)
    assert abs(c["sp_potential_pct"] - 0.8) < 1e-7 and abs(c["sp_perm_connected"] - 0.1) < 1e-7
    assert abs(c["sp_perm_active_inc"] - 0.0001) < 1e-9 and abs(c["sp_perm_inactive_dec"] - 0.0005) < 1e-9
    assert c["sp_boost_strength"] == 0.0
    assert (c["tm_cells_per_col"], c["tm_new_syn_count"], c["tm_max_syn_per_seg"], c["tm_max_segs_per_cell"]) == (12, 20, 32, 128)
    assert (c["tm_min_threshold"], c["tm_activation_threshold"], c["tm_pam_length"], c["tm_seed"]) == (9, 12, 3, 2045)
    assert abs(c["tm_initial_perm"] - 0.21) < 1e-7


def test_abi_version_and_error_string(rt):
    L = rt._lib.lib()
    assert L.htm_abi_version() == 6
    assert isinstance(L.htm_last_error(), bytes)


def test_invalid_config_rejected_without_gpu(rt):
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    L = rt._lib.lib()
    for bad in (dict(sp_boost_strength=-1.0), dict(enc_type=1, enc_w=20), dict(enc_type=1, enc_n=100),
                dict(enc_type=1, rdse_resolution=0.0), dict(enc_type=7)):
        cfg = rt.default_config(**bad)
        h = ctypes.c_void_p()
        code = L.htm_create(ctypes.byref(cfg), 4, 0, ctypes.byref(h))
        assert code != 0 and not h.value, bad


def test_model_yaml_config_is_the_reference_parameter_set(rt):
    """ML/HTM/params/model.yaml:15-63 (RDSE resolution 0.88 / seed 1, SP seed
    1956, potentialPct 0.85, inc 0.04, dec 0.005, boostStrength 3.0; TM 32 cells,
    seed 1960, thresholds 16 / 12, pamLength 1)."""
    c = rt._lib.model_yaml_config().as_dict()
    assert (c["enc_type"], c["enc_n"], c["enc_w"], c["rdse_resolution"], c["rdse_seed"]) == (1, 400, 21, 0.88, 1)
    assert (c["sp_seed"], c["sp_boost_strength"], c["tm_cells_per_col"], c["tm_seed"]) == (1956, 3.0, 32, 1960)
    assert abs(c["sp_potential_pct"] - 0.85) < 1e-7 and abs(c["sp_perm_active_inc"] - 0.04) < 1e-8
    assert (c["tm_activation_threshold"], c["tm_min_threshold"], c["tm_pam_length"]) == (16, 12, 1)
