"""ORACLE (test infrastructure only) — torch-CPU restatement of the
vae4dvar inner loop of `da_4dvar.py`.

  loss(z)        da_4dvar.py:1183-1208
  closure()      da_4dvar.py:1242-1246
  integrate      da_4dvar.py:666-681 (interpolation=True, detach=False)
  one_step_DA    da_4dvar.py:1179-1306 (vae4dvar branch, without the CPU
                 metric logging of :1256-1269)
  x_aug          da_4dvar.py:1196-1206 (obs_type 'real*': F.linear of each
                 13-level variable by obs_interpolater.interp, :62-94)
  R_aug          get_R_matrix_from_gt, da_4dvar.py:729-756
  decoder_hr     nf_model/vae.py:87-90, with the target grid parametrised
                 (the reference hard-codes 721x1440; at 128x256 every
                 nearest interpolation is the identity, SURVEY §8 d)

The optimiser is torch.optim.LBFGS itself (history_size=10, max_iter=10,
line_search_fn="strong_wolfe", `da_4dvar.py:1240`) — the reference's own
third-party dependency, run on CPU.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .lgunet_ref import lgunet_forward


def oracle_problem(prob, dec_p, dec_cfg, flow_p=None, flow_cfg=None, obs_coeff=1.0):
    """RefProblem over the oracle's own network restatement."""
    dec_fn = lambda z: lgunet_forward(dec_p, dec_cfg, z)
    flow_fn = (lambda x: lgunet_forward(flow_p, flow_cfg, x)) if flow_p is not None else None
    return RefProblem(prob, dec_fn, dec_cfg["img_size"], flow_fn, obs_coeff, interp=prob.get("interp"))


def obs_interp_ref(dim_in=13, dim_out=40):
    """obs_interpolater.get_interp / get_interp_inv (da_4dvar.py:62-94), torch fp32 matrices."""
    import numpy as np

    hl = [50, 100, 150, 200, 250, 300, 400, 500, 600, 700, 850, 925, 1000]
    hn = np.round(np.exp(np.linspace(3.91202301, 6.90775528, dim_out)))

    def table(a, b):
        m = torch.zeros(len(a), len(b))
        for i in range(len(a)):
            for j in range(len(b)):
                if a[i] == b[j]:
                    m[i, j] = 1
                elif a[i] > b[j] and a[i] < b[j + 1]:
                    m[i, j] = (np.log(b[j + 1]) - np.log(a[i])) / (np.log(b[j + 1]) - np.log(b[j]))
                    m[i, j + 1] = (np.log(a[i]) - np.log(b[j])) / (np.log(b[j + 1]) - np.log(b[j]))
        return m

    return table(hn, hl), table(hl, hn)


def x_aug_ref(x_pred, interp, nlev=13):
    """da_4dvar.py:1196-1206 on (T, 69, H, W)."""
    parts = [x_pred[:, :4]]
    for i in range(5):
        mat = x_pred[:, 4 + i * nlev:4 + (i + 1) * nlev]
        parts.append(F.linear(mat.transpose(1, 3), interp).transpose(1, 3))
    return torch.cat(parts, 1)


class RefProblem:
    def __init__(self, prob: dict, dec_fn, lat, flow_fn=None, obs_coeff: float = 1.0, interp=None):
        """dec_fn(z) / flow_fn(x): the decoder and flow networks (the oracle's
        `lgunet_forward` restatement, or the reference modules themselves
        when make_golden.py pins this restatement)."""
        t = lambda a: torch.as_tensor(a, dtype=torch.float32)
        self.xb, self.yo, self.H, self.R = t(prob["xb"]), t(prob["yo"]), t(prob["H"]), t(prob["R"])
        self.mean, self.std, self.std_tr = t(prob["mean"]), t(prob["std"]), t(prob["std_tr"])
        self.C = self.xb.shape[0]
        self.Hs, self.Ws = self.xb.shape[1:]
        self.T = self.yo.shape[0]
        self.dec_fn, self.flow_fn = dec_fn, flow_fn
        self.obs_coeff = obs_coeff
        self.lat = tuple(lat)
        self.interp = None if interp is None else t(interp)

    def decoder_hr(self, z):
        x = self.dec_fn(z)
        return F.interpolate(x, (self.Hs, self.Ws))

    def integrate(self, xa):
        za = (xa - self.mean.reshape(-1, 1, 1)) / self.std.reshape(-1, 1, 1)
        z = F.interpolate(za.unsqueeze(0), self.lat)
        z = self.flow_fn(z)[:, : self.C]
        z = F.interpolate(z, (self.Hs, self.Ws))
        return z.reshape(self.C, self.Hs, self.Ws) * self.std.reshape(-1, 1, 1) + self.mean.reshape(-1, 1, 1)

    def trajectory(self, z):
        x = self.decoder_hr(z)
        x = (x * self.std_tr.reshape(1, -1, 1, 1)) * self.std.reshape(1, -1, 1, 1) + self.xb
        x = x[0]
        xs = [x]
        for _ in range(self.T - 1):
            x = self.integrate(x)[: self.C]
            xs.append(x)
        return torch.stack(xs, 0)

    def loss_terms(self, z):
        loss_reg = torch.sum(z ** 2) / 2
        xp = self.trajectory(z)
        if self.interp is not None:
            xp = x_aug_ref(xp, self.interp)
        loss_obs = torch.sum(self.H * (xp - self.yo) ** 2 / self.R) / 2
        return loss_reg, loss_obs

    def loss(self, z):
        r, o = self.loss_terms(z)
        return r + self.obs_coeff * o

    def analysis(self, z):
        out = self.decoder_hr(z)  # da_4dvar.py:1301-1306
        return out[0] * self.std_tr.reshape(-1, 1, 1) * self.std.reshape(-1, 1, 1) + self.xb


def one_step_da_ref(rp: RefProblem, nit: int, latent_shape, history_size=10, max_iter=10, log=None):
    """Restated vae4dvar driver: z=0, Nit outer L-BFGS steps, returns (xa, z, J per outer pass)."""
    z = torch.zeros((1,) + tuple(latent_shape), requires_grad=True)
    lbfgs = torch.optim.LBFGS([z], history_size=history_size, max_iter=max_iter, line_search_fn="strong_wolfe")
    n_eval = [0]

    def closure():
        lbfgs.zero_grad()
        obj = rp.loss(z)
        obj.backward()
        n_eval[0] += 1
        return obj

    js = []
    for kk in range(nit + 1):
        with torch.no_grad():
            r, o = rp.loss_terms(z)
            js.append((float(r), float(o)))
        if log is not None:
            log(kk, js[-1])
        if kk < nit:
            lbfgs.step(closure)
    with torch.no_grad():
        xa = rp.analysis(z)
    return xa, z.detach(), js, n_eval[0], lbfgs.state[lbfgs._params[0]]["n_iter"]


def lat_weights_ref(num_lat):
    """utils/metrics.py:4-9 lat / latitude_weighting_factor_torch with s from :287-289 (fp32)."""
    j = torch.arange(start=0, end=num_lat)
    lat = 90.0 - j * 180.0 / float(num_lat - 1)
    c = torch.cos(3.1416 / 180.0 * lat)
    return num_lat * c / torch.sum(c)


def wrmse_ref(pred_n, gt_n, data_std):
    """Metrics.WRMSE (utils/metrics.py:526-545 -> weighted_rmse_torch :291-294, _channels :282-289); pred_n,
    gt_n (N,C,H,W) normalised; data_std float64 numpy (the reference passes model_std)."""
    w = lat_weights_ref(pred_n.shape[2]).reshape(1, 1, -1, 1)
    r = torch.sqrt(torch.mean(w * (pred_n - gt_n) ** 2.0, dim=(-1, -2)))
    return torch.mean(r, dim=0) * data_std


def bias_ref(pred_n, gt_n, data_std):
    """Metrics.Bias (utils/metrics.py:473-474 -> type_weighted_bias_torch 'all' :265-267, :65-82)."""
    d = pred_n - gt_n
    w = lat_weights_ref(d.shape[2]).reshape(1, 1, -1, 1)
    return torch.mean(torch.mean(w * d, dim=(-1, -2)), dim=0) * data_std


def run_cycles_ref(make_rp, xb0, forecast_fn, n_cycles, nit, latent_shape):
    """run_assimilation (da_4dvar.py:1314-1342) restated: per cycle xa = one_step_DA(xb), xb <- integrate(xa,
    forecast, 1); make_rp(cycle, xb) builds that cycle's RefProblem. Returns the analyses, backgrounds and J."""
    xb = xb0
    out = []
    for k in range(n_cycles):
        rp = make_rp(k, xb)
        xa, _, js, _, _ = one_step_da_ref(rp, nit, latent_shape)
        out.append({"xb": xb, "xa": xa.detach(), "J": js})
        with torch.no_grad():
            xb = forecast_fn(xa.detach())
    return out
