"""CPU: the C-ABI library loads and exports every entry point include/vaevar.h declares; the parameter
enumeration equals the reference state_dict key set (pinned by the oracle); bad configs fail cleanly."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def header_symbols():
    h = open(os.path.join(ROOT, "include", "vaevar.h")).read()
    return sorted(set(re.findall(r"^int\s+(vv_\w+)\s*\(", h, flags=re.M)))


def test_library_exports_header():
    from vaevar import _lib

    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(_lib.lib, s), s
    assert set(syms) == set(_lib.EXPORTED), set(syms) ^ set(_lib.EXPORTED)
    assert _lib.lib.vv_version() >= 100


@pytest.mark.parametrize("name", ["TINY", "TINY_FLOW", "DECODER", "FLOW"])
def test_param_enumeration_matches_oracle(name):
    from oracle.lgunet_ref import param_shapes
    from vaevar import _lib, config as C

    cfg = getattr(C, name)
    pl = _lib.param_list(cfg)
    ps = param_shapes(cfg)
    assert [n for n, _ in pl] == list(dict.fromkeys(n for n, _ in pl))  # unique
    assert set(n for n, _ in pl) == set(ps)
    assert all(ps[n] == s for n, s in pl)


def test_decoder_param_count():
    from vaevar import _lib, config as C
    import numpy as np

    n = sum(int(np.prod(s)) for _, s in _lib.param_list(C.DECODER))
    assert n == 215_880_165  # VAE_lr.dec parameters (buffers excluded)


def test_bad_config_rejected():
    from vaevar import _lib, config as C

    cfg = dict(C.TINY)
    cfg["window_size"] = 6
    with pytest.raises(_lib.VVError, match="window_size"):
        _lib.param_list(cfg)
    cfg = dict(C.TINY)
    cfg["enc_depths"] = [2, 2, 2]
    cfg["enc_heads"] = [2, 4, 4]
    with pytest.raises(_lib.VVError, match="encoder levels"):
        _lib.param_list(cfg)


def test_problem_construction():
    import numpy as np
    from vaevar.problem import make_problem, obs_variance
    from vaevar import config as C

    p = make_problem(nch=69, Hs=32, Ws=64, T=2, seed=1, obs_frac=0.05)
    assert p["yo"].shape == (2, 69, 32, 64) and p["xb"].shape == (69, 32, 64)
    assert np.array_equal(p["H"][0], p["H"][1]) and np.all(p["H"][:, 0] == p["H"][:, 68])  # column mask
    std = np.asarray(C.MODEL_STD, np.float32)
    v = obs_variance(69, 0.005, 2, std)
    # da_4dvar.py:106-127, modify_tp == 2
    assert np.isclose(v[0], 0.005 ** 2 * std[0] ** 2, rtol=1e-6)
    assert np.isclose(v[2], 0.005 ** 2 * std[2] ** 2 / 16, rtol=1e-6)
    assert np.isclose(v[60], 0.005 ** 2 * std[60] ** 2 / 16, rtol=1e-6)
    assert np.allclose(p["R"][1], p["R"][0])  # q_type -1: R[t] = obs_var


def test_no_gpu_ctx_fails_cleanly():
    import torch
    from vaevar import _lib

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = _lib.lib.vv_ctx_create(0, ctypes.byref(h))
    assert rc != 0 and _lib.last_error()


def test_fcst_param_enumeration_matches_reference_keys():
    """vv_lgunet_param_info for LGUnet_all_1 (arch lgunet1) == the state_dict key set / shapes of the reference
    (the oracle's param_shapes is pinned to the real module by oracle/make_golden.py::g7)."""
    from oracle.lgunet1_ref import param_shapes
    from vaevar import _lib
    from vaevar import config as C

    for cfg in (C.TINY_FCST, C.MID_FCST, C.FCST):
        got = dict(_lib.param_list(cfg))
        want = param_shapes(cfg)
        assert set(got) == set(want)
        for k, v in want.items():
            assert tuple(got[k]) == tuple(v), k


def test_new_entry_points_reject_bad_arguments():
    """The observation-operator, metrics and two-loop entry points validate their arguments before any device
    work: a null context or null buffers return VV_E_ARG (1001) with a message, never a crash (no GPU needed)."""
    import ctypes

    from vaevar import _lib

    lib = _lib.lib
    assert lib.vv_set_obs_operator(None, 40, 13, None) == 1001
    assert lib.vv_obs_augment(None, None, 40, 13, None, None, 1, 8, 8, None) == 1001
    assert lib.vv_metrics(None, None, None, None, None, None, 1, 69, 8, 8, None, None, None) == 1001
    ro = (ctypes.c_float * 1)(1.0)
    assert lib.vv_lbfgs_two_loop(None, None, None, None, ro, 1, 1.0, 16, None) == 1001
    out = (ctypes.c_double * 4)()
    ops = (ctypes.c_int * 1)(0)
    ptrs = (ctypes.c_void_p * 1)(None)
    assert lib.vv_reduce_batch(None, 1, ops, ptrs, ptrs, 16, None, 0, out, None) == 1001
    assert lib.vv_closure_async(None, None, None, None, None) == 1001
    buf = ctypes.create_string_buffer(256)
    lib.vv_last_error(buf, 256)
    assert buf.value  # a message describes the failure


def test_tuning_api_keys_and_rejection():
    """The per-context dispatch knobs (vv_set_tuning / vv_get_tuning) replace the environment reads the library
    once did: every key the Python Context knows is documented in include/vaevar.h, a null context or an unknown
    key returns VV_E_ARG, and the library binary names no VAEVAR_ environment variable any more."""
    import ctypes

    from vaevar import _lib
    from vaevar.engine import Context

    lib = _lib.lib
    hdr = open(os.path.join(ROOT, "include", "vaevar.h")).read()
    for k in Context.TUNING_KEYS:
        assert f'"{k}"' in hdr, k
    v = ctypes.c_int()
    assert lib.vv_set_tuning(None, b"h3_mink", 384) == 1001
    assert lib.vv_get_tuning(None, b"h3_mink", ctypes.byref(v)) == 1001
    assert lib.vv_set_debug_sync(0) == 0
    so = open(_lib.LIB_PATH, "rb").read()
    assert b"VAEVAR_" not in so and b"getenv" not in so


def test_launch_counters_abi():
    """vv_get_counter (host-side, no GPU needed): the named fused-path counters exist, unknown names fail cleanly."""
    from vaevar import _lib
    from vaevar.engine import Context

    for name in ("rowsplit", "fixup_ln", "splitk_fixup", "gather_scales", "h5_split"):
        assert Context.counter(name) >= 0
    with pytest.raises(_lib.VVError, match="unknown counter"):
        Context.counter("nope")


@pytest.mark.parametrize("var,val,msg", [("VAEVAR_GEMM_MATH", "fp8", "VAEVAR_GEMM_MATH"),
                                         ("VAEVAR_H3_MINK", "big", "not an integer")])
def test_context_env_validated_before_create(monkeypatch, var, val, msg):
    """A bad VAEVAR_* value raises before the native context exists (no handle or device buffers leak)."""
    from vaevar.engine import Context

    monkeypatch.setenv(var, val)
    with pytest.raises(ValueError, match=msg):
        Context(0)
