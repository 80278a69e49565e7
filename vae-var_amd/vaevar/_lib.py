"""ctypes binding of libvaevar.so (C-ABI: include/vaevar.h).

There is no fallback: if the HIP library is missing or fails to load, importing
this module raises, so a GPU run can never silently use a CPU path.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VAEVAR_LIB", os.path.join(HERE, "libvaevar.so"))

c_int, c_int64, c_float, c_double, c_void_p, c_char_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_float,
                                                          ctypes.c_double, ctypes.c_void_p, ctypes.c_char_p)
P = ctypes.POINTER


class VVConfig(ctypes.Structure):
    _fields_ = [
        ("img_size", c_int * 2),
        ("patch_size", c_int * 2),
        ("stride", c_int * 2),
        ("n_groups", c_int),
        ("inchans", c_int * 8),
        ("outchans", c_int * 8),
        ("enc_dim", c_int),
        ("embed_dim", c_int),
        ("window_size", c_int),
        ("n_enc_levels", c_int),
        ("enc_depths", c_int * 4),
        ("enc_heads", c_int * 4),
        ("n_lg_layers", c_int),
        ("lg_depths", c_int * 8),
        ("lg_heads", c_int * 8),
        ("arch", c_int),
        ("window_hw", c_int * 2),
    ]

    @classmethod
    def from_dict(cls, cfg: dict) -> "VVConfig":
        c = cls()
        c.img_size[:] = list(cfg["img_size"])
        c.patch_size[:] = list(cfg["patch_size"])
        c.stride[:] = list(cfg["stride"])
        ins, outs = list(cfg["inchans_list"]), list(cfg["outchans_list"])
        if len(ins) != len(outs) or len(ins) > 8:
            raise ValueError("inchans_list and outchans_list must have equal length <= 8")
        c.n_groups = len(ins)
        c.inchans[: len(ins)] = ins
        c.outchans[: len(outs)] = outs
        c.enc_dim = cfg["enc_dim"]
        c.embed_dim = cfg["embed_dim"]
        ws = cfg["window_size"]
        c.window_size = ws if isinstance(ws, int) else int(ws[0])
        c.arch = {"lgunet": 0, "lgunet1": 1}[cfg.get("arch", "lgunet")]
        c.window_hw[:] = [ws, ws] if isinstance(ws, int) else [int(ws[0]), int(ws[1])]
        c.n_enc_levels = len(cfg["enc_depths"])
        c.enc_depths[: c.n_enc_levels] = list(cfg["enc_depths"])
        c.enc_heads[: c.n_enc_levels] = list(cfg["enc_heads"])
        if len(cfg["enc_heads"]) != c.n_enc_levels or len(cfg["lg_heads"]) != len(cfg["lg_depths"]):
            raise ValueError("enc_heads / lg_heads must match enc_depths / lg_depths in length")
        c.n_lg_layers = len(cfg["lg_depths"])
        c.lg_depths[: c.n_lg_layers] = list(cfg["lg_depths"])
        c.lg_heads[: c.n_lg_layers] = list(cfg["lg_heads"])
        return c


_SIGS = {
    "vv_version": (c_int, []),
    "vv_last_error": (c_int, [c_char_p, c_int]),
    "vv_lgunet_param_count": (c_int, [P(VVConfig), P(c_int)]),
    "vv_lgunet_param_info": (c_int, [P(VVConfig), c_int, c_char_p, c_int, P(c_int64), P(c_int)]),
    "vv_ctx_create": (c_int, [c_int, P(c_void_p)]),
    "vv_ctx_destroy": (c_int, [c_void_p]),
    "vv_model_create": (c_int, [c_void_p, P(VVConfig), c_int, c_int, P(c_int)]),
    "vv_model_destroy": (c_int, [c_void_p, c_int]),
    "vv_load_weights": (c_int, [c_void_p, c_int, P(c_void_p), c_int]),
    "vv_model_forward": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "vv_model_backward": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "vv_model_workspace_bytes": (c_int, [c_void_p, c_int, P(c_int64)]),
    "vv_bind_problem": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_float]),
    "vv_closure": (c_int, [c_void_p, c_void_p, c_void_p, P(c_double), P(c_double), c_void_p]),
    "vv_closure_async": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vv_decode": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "vv_state_ptr": (c_int, [c_void_p, P(c_void_p)]),
    "vv_metrics": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                           c_void_p, c_void_p, c_void_p]),
    "vv_set_obs_operator": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "vv_obs_augment": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "vv_dot": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, P(c_double), c_void_p]),
    "vv_abssum": (c_int, [c_void_p, c_void_p, c_int64, P(c_double), c_void_p]),
    "vv_absmax": (c_int, [c_void_p, c_void_p, c_int64, P(c_float), c_void_p]),
    "vv_reduce_batch": (c_int, [c_void_p, c_int, P(c_int), P(c_void_p), P(c_void_p), c_int64, c_void_p, c_int,
                                P(c_double), c_void_p]),
    "vv_reduce_enqueue": (c_int, [c_void_p, c_int, P(c_int), P(c_void_p), P(c_void_p), c_int64, c_void_p, c_void_p]),
    "vv_axpy": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_int64, c_void_p]),
    "vv_axpby": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_float, c_int64, c_void_p]),
    "vv_scale": (c_int, [c_void_p, c_void_p, c_float, c_int64, c_void_p]),
    "vv_copy": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "vv_lbfgs_two_loop": (c_int, [c_void_p, c_void_p, P(c_void_p), P(c_void_p), P(c_float), c_int, c_float, c_int64,
                                  c_void_p]),
    "vv_adam": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float,
                        c_float, c_int, c_void_p]),
    "vv_profile_start": (c_int, [c_void_p]),
    "vv_profile_stop": (c_int, [c_void_p, P(c_double), P(c_double), P(c_double), P(c_int), c_int]),
    "vv_nearest_map": (c_int, [c_int, c_int, P(c_int)]),
    "vv_set_gemm_math": (c_int, [c_void_p, c_int]),
    "vv_set_closure_graph": (c_int, [c_void_p, c_int]),
    "vv_get_closure_graph": (c_int, [c_void_p, c_int, P(ctypes.c_longlong)]),
    "vv_get_counter": (c_int, [ctypes.c_char_p, P(ctypes.c_longlong)]),
    "vv_integrate": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                             c_int, c_void_p]),
    "vv_get_gemm_math": (c_int, [c_void_p, P(c_int)]),
    "vv_set_tuning": (c_int, [c_void_p, ctypes.c_char_p, c_int]),
    "vv_get_tuning": (c_int, [c_void_p, ctypes.c_char_p, P(c_int)]),
    "vv_set_debug_sync": (c_int, [c_int]),
    "vv_attention_global": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "vv_gemm_register_weight": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "vv_gemm": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "vv_gemm_epi": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                            c_int, c_void_p]),
    "vv_gelu_eval": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "vv_sc4dvar_bind": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_float, c_void_p, c_int, P(c_double), P(c_double), c_int,
                                P(c_double), P(c_double), P(c_double), c_double, c_int]),
    "vv_sc4dvar_closure": (c_int, [c_void_p, c_void_p, c_void_p, P(c_double), P(c_double), c_void_p]),
    "vv_sc4dvar_transform": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "vv_resample_nearest": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
}

EXPORTED = sorted(_SIGS)


class VVError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libvaevar.so not found at {LIB_PATH}: build it with `make -C vae-var_amd/csrc` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    # torch must be imported first so that its HIP runtime is the one libvaevar binds to
    import torch  # noqa: F401

    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    buf = ctypes.create_string_buffer(1024)
    lib.vv_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise VVError(f"libvaevar {what} failed (status {rc}): {last_error()}")


def nearest_map(in_size: int, out_size: int):
    """F.interpolate(mode='nearest') source indices used by the engine (quirk Q3)."""
    m = (c_int * out_size)()
    check(lib.vv_nearest_map(in_size, out_size, m), "nearest_map")
    return list(m)


def param_list(cfg: dict):
    """[(state_dict name, shape)] in libvaevar order (networks_old.LGUnet_all parameters)."""
    c = VVConfig.from_dict(cfg)
    n = c_int()
    check(lib.vv_lgunet_param_count(ctypes.byref(c), ctypes.byref(n)), "param_count")
    out = []
    name = ctypes.create_string_buffer(256)
    shape = (c_int64 * 8)()
    nd = c_int()
    for i in range(n.value):
        check(lib.vv_lgunet_param_info(ctypes.byref(c), i, name, 256, shape, ctypes.byref(nd)), "param_info")
        out.append((name.value.decode(), tuple(int(shape[k]) for k in range(nd.value))))
    return out
