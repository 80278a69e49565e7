"""Synthetic 3D/4D-Var problems (background, observations, operator, errors).

Shapes follow the reference's `one_step_DA(gt, xb, yo, H, R, 'vae4dvar')`
(`da_4dvar.py:1179-1306`): xb (C,Hs,Ws); yo, H, R (T,C,Hs,Ws).

Observation error R follows `data_reader.__init__` (`da_4dvar.py:106-127`):
obs_var = obs_std^2 * model_std_c^2, with the `modify_tp` rescalings, and
`get_static_info` (`da_4dvar.py:630-634`): R[0] = obs_var,
R[t] = obs_var + q[t-1]; the synthetic case uses q_type = -1 (q = 0).
Observations are the truth (`get_obs_gt`, `da_4dvar.py:445-449`), seen
through a random column mask like the `free_*` obs types
(`da_4dvar.py:277-292`: one lat/lon mask shared by every channel and time).
SURVEY §8 d1 defines the synthetic truth and background.
"""
from __future__ import annotations

import numpy as np

from . import config as C
from .synth import smooth_field, splitmix_uniform


def obs_variance(nch: int, obs_std: float, modify_tp: int, std: np.ndarray) -> np.ndarray:
    v = (np.float32(obs_std) ** 2 * std.astype(np.float32) ** 2).astype(np.float32)
    if nch == 69:
        if modify_tp == 1:
            v[56:] /= 4
        elif modify_tp == 2:
            v[56:] /= 16
            v[2] /= 16
        elif modify_tp == 3:
            v[56:] /= 16
            v[2] /= 16
            v[30:56] /= 16
        elif modify_tp == 4:
            v[56:] /= 16
            v[2] /= 16
            v[17:30] /= 4
    return v


def make_problem(nch: int = 69, Hs: int = 128, Ws: int = 256, T: int = 1, seed: int = 20250620,
                 obs_frac: float = 0.01, obs_std: float = 0.005, modify_tp: int = 2) -> dict:
    mean = np.asarray(C.MODEL_MEAN[:nch], dtype=np.float32)
    std = np.asarray(C.MODEL_STD[:nch], dtype=np.float32)
    std_tr = np.asarray(C.STD_TR[:nch], dtype=np.float32)
    s = smooth_field(seed, (nch, Hs, Ws))
    gt0 = mean[:, None, None] + std[:, None, None] * s
    gts = [gt0]
    for t in range(1, T):
        ds = smooth_field(seed + 1000 + t, (nch, Hs, Ws))
        gts.append(gts[-1] + np.float32(0.05) * std[:, None, None] * ds)
    gt = np.stack(gts, 0).astype(np.float32)
    sp = smooth_field(seed + 1, (nch, Hs, Ws))
    xb = (gt0 + np.float32(0.1) * std[:, None, None] * sp).astype(np.float32)
    u = splitmix_uniform(seed + 2, Hs * Ws).reshape(Hs, Ws)
    col = (u < obs_frac).astype(np.float32)
    H = np.broadcast_to(col, (T, nch, Hs, Ws)).astype(np.float32).copy()
    yo = gt.copy()
    ov = obs_variance(nch, obs_std, modify_tp, std)
    R = np.broadcast_to(ov[None, :, None, None], (T, nch, Hs, Ws)).astype(np.float32).copy()
    return {"gt": gt, "xb": xb, "yo": yo, "H": H, "R": R, "mean": mean, "std": std, "std_tr": std_tr}
