"""Latitude-weighted WRMSE / Bias on the device (vv_metrics) — the per-channel diagnostics one_step_DA logs at
every outer pass (da_4dvar.py:1256-1262): Metrics.WRMSE (utils/metrics.py:526-545 -> weighted_rmse_torch,
:282-294) and Metrics.Bias (:473-474 -> type_weighted_bias_torch 'all', :65-82, :265-267), both on fields
normalised by the model mean/std and scaled back by the float64 model std."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import config as C
from ._lib import check, lib
from .engine import Context, _ptr, _stream

Z500 = 11  # channel index the reference prints as "RMSE (z500)" (da_4dvar.py:1254)


def _ptr64(t: torch.Tensor):
    if not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
        raise ValueError("expected a contiguous float64 device tensor")
    return ctypes.c_void_p(t.data_ptr())


class Metrics:
    def __init__(self, ctx: Context, mean=None, std=None, device: int = 0):
        dev = torch.device("cuda", device)
        mean = C.MODEL_MEAN if mean is None else mean
        std = C.MODEL_STD if std is None else std
        self.ctx = ctx
        self.mean = torch.as_tensor(np.asarray(mean, np.float32)).to(dev)
        self.std = torch.as_tensor(np.asarray(std, np.float32)).to(dev)
        self.scale = torch.as_tensor(np.asarray(std, np.float64)).to(dev)  # data_std = model_std (float64)

    def wrmse_bias(self, pred: torch.Tensor, gt: torch.Tensor):
        """pred, gt (C,H,W) or (B,C,H,W) physical fields on the device -> (wrmse[C], bias[C]) float64 tensors."""
        if pred.dim() == 3:
            pred, gt = pred.unsqueeze(0), gt.unsqueeze(0)
        B, Cc, H, W = pred.shape
        if gt.shape != pred.shape or Cc != self.mean.numel():
            raise ValueError(f"shape mismatch {tuple(pred.shape)} {tuple(gt.shape)} C={self.mean.numel()}")
        pred, gt = pred.float().contiguous(), gt.to(pred.device, torch.float32).contiguous()
        w = torch.empty(Cc, device=pred.device, dtype=torch.float64)
        b = torch.empty_like(w)
        check(lib.vv_metrics(self.ctx.h, _ptr(pred), _ptr(gt), _ptr(self.mean), _ptr(self.std), _ptr64(self.scale), B,
                             Cc, H, W, _ptr64(w), _ptr64(b), _stream()), "metrics")
        return w, b
