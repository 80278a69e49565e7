"""sc4dvar — the static-B 4D-Var mode of cyclic_4dvar.one_step_DA (da_4dvar.py:1064-1177) on libvaevar.

  BMatrix          init_b_matrix (da_4dvar.py:520-526): the statistics of dataset/bq_info_lr/*.npy
  Sc4dvarProblem   get_static_info (:608-628) + loss / closure (:1071-1107): J(w) = sum(w^2)/2 +
                   obs_coeff * sum_t H (x_t - yo_t)^2 / R / 2 with x_0 = transform(w, xb) (:878-931) and
                   x_t = integrate(x_{t-1}) (detached, :1080); every FLOP in the HIP library (vv_sc4dvar_*)
  one_step_sc4dvar w = 0 (:1116), LBFGS(history_size=10, max_iter=5, strong_wolfe) (:1119), Nit outer steps
                   (:1124-1170), xhat = transform(w, xb) (:1173)
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import torch

from ._lib import check, lib
from .engine import Context, LGUnet, _ptr, _stream
from .lbfgs import LBFGS

KEYS = ("len_scale", "reg_coeff", "std_sur", "vert_eig_value", "vert_eig_vec")


class BMatrix:
    """The B-matrix statistics as float64 arrays (init_b_matrix; len_scale is multiplied by scale_factor)."""

    def __init__(self, len_scale, reg_coeff, std_sur, vert_eig_value, vert_eig_vec, scale_factor: float = 1.0):
        self.len_scale = np.ascontiguousarray(len_scale, np.float64)
        self.reg_coeff = np.ascontiguousarray(reg_coeff, np.float64)
        self.std_sur = np.ascontiguousarray(std_sur, np.float64)
        self.vert_eig_value = np.ascontiguousarray(vert_eig_value, np.float64)
        self.vert_eig_vec = np.ascontiguousarray(vert_eig_vec, np.float64)
        self.scale_factor = float(scale_factor)
        C = self.len_scale.shape[0]
        if (self.reg_coeff.shape[0] != C or self.reg_coeff.shape[1] not in (13, 26) or self.std_sur.shape != (4,)
                or self.vert_eig_value.shape != (5, 13) or self.vert_eig_vec.shape != (5, 13, 13)):
            raise ValueError("B-matrix statistics of unexpected shape")

    @classmethod
    def from_dir(cls, coeff_dir: str, scale_factor: float = 1.0) -> "BMatrix":
        """--coeff_dir (default dataset/bq_info_lr/): one .npy per statistic (loaded without pickle)."""
        return cls(*[np.load(os.path.join(coeff_dir, k + ".npy"), allow_pickle=False) for k in KEYS],
                   scale_factor=scale_factor)

    @classmethod
    def from_npz(cls, path: str, scale_factor: float = 1.0) -> "BMatrix":
        with np.load(path, allow_pickle=False) as z:
            return cls(*[z[k] for k in KEYS], scale_factor=scale_factor)


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class Sc4dvarProblem:
    """The sc4dvar closure bound to device buffers: prob = dict(xb (69,Hs,Ws), yo/H/R (T,C_obs,Hs,Ws), mean, std);
    flow: the networks_old LGUnet_all forecast model for T > 1; obs_interp: obs_interpolater.interp for 'real*'."""

    def __init__(self, bmat: BMatrix, prob: dict, flow: LGUnet | None = None, obs_coeff: float = 1.0,
                 device: int = 0, obs_interp=None, hpad: int = 112):
        dev = torch.device("cuda", device)

        def t(a):
            if isinstance(a, torch.Tensor):
                return a.to(device=dev, dtype=torch.float32).contiguous()
            return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32).to(dev)

        self.xb, self.yo, self.H, self.R = t(prob["xb"]), t(prob["yo"]), t(prob["H"]), t(prob["R"])
        self.mean, self.std = t(prob["mean"]), t(prob["std"])
        if self.xb.dim() != 3 or self.xb.shape[0] != 69:
            raise ValueError(f"xb must be (69, Hs, Ws), got {tuple(self.xb.shape)}")
        self.C, self.Hs, self.Ws = self.xb.shape
        if self.yo.dim() != 4 or self.yo.shape[-2:] != self.xb.shape[-2:]:
            raise ValueError(f"yo must be (T, C_obs, {self.Hs}, {self.Ws}), got {tuple(self.yo.shape)}")
        if self.H.shape != self.yo.shape or self.R.shape[-2:] != self.yo.shape[-2:] or self.R.shape[0] != self.yo.shape[0]:
            raise ValueError("H must match yo; R must be (T, C_obs, Hs, Ws)")
        self.T = self.yo.shape[0]
        if self.T > 1 and flow is None:
            raise ValueError("a window of T > 1 needs the flow model")
        self.ctx = flow.ctx if flow is not None else Context.get(device)
        self.obs_coeff = float(obs_coeff)
        self.bmat, self.flow = bmat, flow
        if obs_interp is None:
            obs_interp = prob.get("interp")
        self.interp = None if obs_interp is None else t(obs_interp)
        n_out = self.interp.shape[0] if self.interp is not None else 0
        c_obs = 4 + 5 * n_out if n_out else self.C
        if self.yo.shape[1] != c_obs or self.R.shape[1] != c_obs:
            raise ValueError(f"yo / R have {self.yo.shape[1]} / {self.R.shape[1]} channels, expected {c_obs}")
        self.w_shape = (self.C, 128, 256)
        b = bmat
        check(lib.vv_sc4dvar_bind(self.ctx.h, flow.id if flow is not None else -1, self.T, self.C, self.Hs, self.Ws,
                                  _ptr(self.xb), _ptr(self.yo), _ptr(self.H), _ptr(self.R), _ptr(self.mean),
                                  _ptr(self.std), self.obs_coeff,
                                  _ptr(self.interp) if self.interp is not None else None, n_out,
                                  _dp(b.len_scale), _dp(b.reg_coeff), b.reg_coeff.shape[1], _dp(b.std_sur),
                                  _dp(b.vert_eig_value), _dp(b.vert_eig_vec), b.scale_factor, hpad), "sc4dvar_bind")
        self.n_evals = 0

    def closure(self, w: torch.Tensor, grad: torch.Tensor | None):
        """(J_b, J_o) as Python floats; grad <- dJ/dw if given."""
        jb, jo = ctypes.c_double(), ctypes.c_double()
        check(lib.vv_sc4dvar_closure(self.ctx.h, _ptr(w), _ptr(grad) if grad is not None else None,
                                     ctypes.byref(jb), ctypes.byref(jo), _stream()), "sc4dvar_closure")
        self.n_evals += 1
        return jb.value, jo.value

    def loss_f32(self, jb: float, jo: float) -> float:
        """cal_loss_bg(w) + obs_coeff * cal_loss_obs(xhat) with the reference's fp32 scalar arithmetic."""
        return float(np.float32(jb) + np.float32(np.float32(self.obs_coeff) * np.float32(jo)))

    def transform(self, w: torch.Tensor) -> torch.Tensor:
        """xhat (69,Hs,Ws) = transform(w, xb) (da_4dvar.py:878-931)."""
        out = torch.empty(self.C, self.Hs, self.Ws, device=w.device, dtype=torch.float32)
        check(lib.vv_sc4dvar_transform(self.ctx.h, _ptr(w.contiguous()), _ptr(out), _stream()), "sc4dvar_transform")
        return out


def one_step_sc4dvar(prob: Sc4dvarProblem, nit: int, history_size: int = 10, max_iter: int = 5,
                     log_terms: bool = True, replay=None):
    """cyclic_4dvar.one_step_DA(..., 'sc4dvar') (da_4dvar.py:1114-1177) without the CPU metric logging:
    returns dict(xa, w, J=[(J_b, J_o) per outer pass], n_eval, n_iter, seconds)."""
    w = torch.zeros(prob.w_shape, device=prob.xb.device, dtype=torch.float32)
    opt = LBFGS(prob.ctx, w, lr=1, history_size=history_size, max_iter=max_iter, line_search_fn="strong_wolfe")
    opt.replay = list(replay) if replay is not None else None

    def closure(ww, g):
        jb, jo = prob.closure(ww, g)
        return prob.loss_f32(jb, jo)

    js = []
    n0 = prob.n_evals
    t0 = time.time()
    for kk in range(nit + 1):
        if log_terms:
            js.append(prob.closure(w, None))  # loss_total / loss_bg / loss_obs of the log line (:1132-1136)
        if kk < nit:
            opt.step(closure)
    xa = prob.transform(w)
    torch.cuda.synchronize()
    n_log = (nit + 1) if log_terms else 0
    return {"xa": xa, "w": w, "J": js, "n_eval": prob.n_evals - n0 - n_log, "n_iter": opt.state["n_iter"],
            "seconds": time.time() - t0}
