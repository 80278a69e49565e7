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


# ---------------------------------------------------------------------------------------------------------------
# Real-observation operator: obs_interpolater (da_4dvar.py:62-94) maps the 13 model pressure
# levels to dim_out log-spaced levels; the loss compares observations with x_aug (da_4dvar.py:1196-1206) and
# R is interpolated the same way (get_R_matrix_from_gt, da_4dvar.py:729-756).
HEIGHT_LEVEL = [50, 100, 150, 200, 250, 300, 400, 500, 600, 700, 850, 925, 1000]


class ObsInterpolater:
    """obs_interpolater(dim_in, dim_out) (da_4dvar.py:62-94): interp (dim_out, dim_in) and interp_inv (dim_in,
    dim_out), weights linear in log-pressure, computed in float64 and stored as fp32 like the reference's
    torch.zeros(...) assignment."""

    def __init__(self, dim_in: int = 13, dim_out: int = 40):
        self.dim_in, self.dim_out = dim_in, dim_out
        self.height_level = HEIGHT_LEVEL
        self.height_level_new = np.round(np.exp(np.linspace(3.91202301, 6.90775528, dim_out)))
        self.interp = self._weights(self.height_level_new, self.height_level)
        self.interp_inv = self._weights(self.height_level, self.height_level_new)

    @staticmethod
    def _weights(dst, src) -> np.ndarray:
        w = np.zeros((len(dst), len(src)), np.float32)
        for i, h in enumerate(dst):
            for j, s in enumerate(src):
                if h == s:
                    w[i, j] = 1
                elif j + 1 < len(src) and s < h < src[j + 1]:
                    d = np.log(src[j + 1]) - np.log(s)
                    w[i, j] = (np.log(src[j + 1]) - np.log(h)) / d
                    w[i, j + 1] = (np.log(h) - np.log(s)) / d
        return w


def obs_augment_np(interp: np.ndarray, x: np.ndarray) -> np.ndarray:
    """x_aug for (T, 4 + 5*n_in, H, W) host fields (problem generation only; the closure runs it on the GPU)."""
    n_out, n_in = interp.shape
    parts = [x[:, :4]]
    for i in range(5):
        mat = x[:, 4 + i * n_in:4 + (i + 1) * n_in]
        parts.append(np.einsum("oj,tjhw->tohw", interp, mat, dtype=np.float32))
    return np.concatenate(parts, 1).astype(np.float32)


def make_real_problem(nch: int = 69, Hs: int = 128, Ws: int = 256, T: int = 1, seed: int = 20250622,
                      dim_out: int = 40, obs_frac: float = 0.01, level_frac: float = 0.5, obs_std: float = 0.005,
                      modify_tp: int = 2) -> dict:
    """A synthetic 'real*' observation problem: yo = x_aug(gt) in the 4 + 5*dim_out observation channels, H marks
    observed (channel, lat, lon) entries as get_real_obs does (a random station column mask, each station
    reporting a random subset of the interpolated levels), R = get_R_matrix_from_gt of the static R."""
    assert nch == 69, "the level structure is the 69-channel ERA5 layout"
    p = make_problem(nch=nch, Hs=Hs, Ws=Ws, T=T, seed=seed, obs_frac=obs_frac, obs_std=obs_std, modify_tp=modify_tp)
    oi = ObsInterpolater(13, dim_out)
    ca = 4 + 5 * dim_out
    col = p["H"][0, 0]
    u = splitmix_uniform(seed + 3, ca * Hs * Ws).reshape(ca, Hs, Ws)
    H = np.broadcast_to((col[None] * (u < level_frac)).astype(np.float32), (T, ca, Hs, Ws)).copy()
    p.update(yo=obs_augment_np(oi.interp, p["gt"]), H=H, R=obs_augment_np(oi.interp, p["R"]), interp=oi.interp)
    return p
