"""The assimilation cycle of cyclic_4dvar in the vae4dvar mode on the HIP engine.

  run_assimilation        da_4dvar.py:1314-1342  obs -> one_step_DA -> save results -> xb = integrate(xa, fcst, 1)
  get_current_states      da_4dvar.py:683-696    resume from da_cycle_results/<name>/{current_time.txt, xb.npy}
  save_ckpt               da_4dvar.py:698-702
  save_eval_result        da_4dvar.py:704-714    metrics_list entries as <key>.npy (+ xb_/xa_ fields on request)
  get_state (layout)      da_4dvar.py:148-166    ERA5 channel order and per-variable .npy file names

The state stays on the device for the whole cycle: analysis, forecast (vv_integrate) and the WRMSE/Bias
diagnostics (vv_metrics) run on the GPU; only checkpoints and metric vectors go to the host. Observation and
truth access is a provider object (the reference reads them from petrel/S3, out of scope here).
"""
from __future__ import annotations

import datetime as _dt
import os

import numpy as np
import torch

from . import config as C
from .da import one_step_da
from .engine import DAProblem, LGUnet, integrate
from .metrics import Metrics

SINGLE_LEVEL = ["u10", "v10", "t2m", "msl"]
MULTI_LEVEL = ["z", "q", "u", "v", "t"]
HEIGHT_LEVEL = [50, 100, 150, 200, 250, 300, 400, 500, 600, 700, 850, 925, 1000]
CHANNELS = SINGLE_LEVEL + [f"{v}{h}" for v in MULTI_LEVEL for h in HEIGHT_LEVEL]  # the 69 state channels


def _stamp(t: _dt.datetime) -> str:
    return t.strftime("%Y-%m-%dT%H:%M:%S")


class StateFiles:
    """data_reader.get_state's layout (da_4dvar.py:148-166) under a local root instead of the S3 bucket:
    single/<year>/<YYYY-MM-DD>/<HH:MM:SS>-<vname>.npy and <year>/<YYYY-MM-DD>/<HH:MM:SS>-<vname>-<level>.0.npy,
    each one (H, W) float32 field; channels stacked in CHANNELS order."""

    def __init__(self, root: str, shape=(721, 1440)):
        self.root, self.shape = root, tuple(shape)

    def _paths(self, t: _dt.datetime):
        day, hms = _stamp(t).split("T")
        for v in SINGLE_LEVEL:
            yield os.path.join(self.root, "single", str(t.year), day, f"{hms}-{v}.npy")
        for v in MULTI_LEVEL:
            for h in HEIGHT_LEVEL:
                yield os.path.join(self.root, str(t.year), day, f"{hms}-{v}-{float(h)}.npy")

    def get_state(self, t: _dt.datetime) -> np.ndarray:
        return np.concatenate([np.load(p).reshape(1, *self.shape) for p in self._paths(t)], 0).astype(np.float32)

    def put_state(self, t: _dt.datetime, x: np.ndarray) -> None:
        for p, f in zip(self._paths(t), np.asarray(x, np.float32)):
            os.makedirs(os.path.dirname(p), exist_ok=True)
            np.save(p, f)


class SyntheticObs:
    """get_obs_info for the non-'real' observation types (da_4dvar.py:758-763): gt = the truth states of the window
    (get_obs_gt, :445-455: current time and da_win-1 steps of step_int_time), yo = gt, H a fixed mask, R the static
    R. `truth(t)` returns the (C,Hs,Ws) truth at time t (e.g. StateFiles.get_state)."""

    def __init__(self, truth, H: np.ndarray, R: np.ndarray, da_win: int = 1,
                 step_int_time: _dt.timedelta = _dt.timedelta(hours=1)):
        self.truth, self.H, self.R = truth, H, R
        self.da_win, self.step = da_win, step_int_time

    def get_obs_info(self, t: _dt.datetime):
        gt = np.stack([self.truth(t + i * self.step) for i in range(self.da_win)], 0).astype(np.float32)
        return gt, self.H, self.R, gt  # yo, H, R, gt


class SyntheticRealObs:
    """get_obs_info for obs_type 'real_simu_nofiltering' (da_4dvar.py:764-792): the truth window gt, its level
    interpolation gt_aug = x_aug(gt) (obs_interpolater, :770-776), yo = gt_aug * H (no filtering mask, :783-792),
    R = get_R_matrix_from_gt (:729-756), all in the 4 + 5*n_out observation channels; x_aug runs on the GPU
    (vv_obs_augment). H: (da_win, 4 + 5*n_out, Hs, Ws) station mask; R: the static (da_win, 69, Hs, Ws) R."""

    def __init__(self, ctx, truth, H, R, interp, da_win: int = 1,
                 step_int_time: _dt.timedelta = _dt.timedelta(hours=1), device: int = 0):
        from .engine import obs_augment

        self.dev = torch.device("cuda", device)
        self.truth, self.da_win, self.step = truth, da_win, step_int_time
        self.interp = torch.as_tensor(np.asarray(interp, np.float32)).to(self.dev)
        self.H = torch.as_tensor(np.asarray(H, np.float32)).to(self.dev)
        self._aug = lambda x: obs_augment(ctx, self.interp, x)
        self.R = self._aug(torch.as_tensor(np.asarray(R, np.float32)).to(self.dev))

    def get_obs_info(self, t: _dt.datetime):
        gt = np.stack([self.truth(t + i * self.step) for i in range(self.da_win)], 0).astype(np.float32)
        gt_d = torch.from_numpy(gt).to(self.dev)
        yo = self._aug(gt_d) * self.H
        return yo, self.H, self.R, gt_d


class CyclicVAE4DVar:
    """cyclic_4dvar restricted to da_mode 'vae4dvar' (da_4dvar.py:1179-1306, 1314-1342)."""

    def __init__(self, decoder: LGUnet, forecast: LGUnet, obs, start_time: _dt.datetime, end_time: _dt.datetime,
                 Nit: int, name: str, out_dir: str = "da_cycle_results", cycle_time=_dt.timedelta(hours=6),
                 flow: LGUnet | None = None, obs_coeff: float = 1.0, save_interval: int = 1, xb0=None,
                 mean=None, std=None, std_tr=None, obs_interp=None, save_field: bool = False, device: int = 0):
        self.dec, self.fcst, self.flow, self.obs = decoder, forecast, flow, obs
        self.start_time, self.end_time, self.cycle_time = start_time, end_time, cycle_time
        self.Nit, self.name, self.obs_coeff, self.save_interval = Nit, name, obs_coeff, save_interval
        self.dir = os.path.join(out_dir, name)
        self.obs_interp, self.save_field = obs_interp, save_field
        dev = torch.device("cuda", device)
        nch = decoder.out_ch if hasattr(decoder, "out_ch") else C.NCHANNEL
        self.mean = np.asarray(C.MODEL_MEAN[:nch] if mean is None else mean, np.float32)
        self.std = np.asarray(C.MODEL_STD[:nch] if std is None else std, np.float32)
        self.std_tr = np.asarray(C.STD_TR[:nch] if std_tr is None else std_tr, np.float32)
        self.mean_d = torch.from_numpy(self.mean).to(dev)
        self.std_d = torch.from_numpy(self.std).to(dev)
        self.metric = Metrics(decoder.ctx, self.mean, C.MODEL_STD[:nch] if std is None else std, device)
        # the reference's full key set (da_4dvar.py:511), so da_cycle_results/<name>/*.npy match file for file; the
        # vae4dvar branch fills bg_/ana_ wrmse and bias (:1285-1291), the others stay empty (mse: other modes,
        # error_obs: use_eval only)
        self.metrics_list = {"bg_wrmse": [], "ana_wrmse": [], "bg_mse": [], "ana_mse": [], "bg_bias": [],
                             "ana_bias": [], "error_obs": []}
        self.dev = dev
        os.makedirs(self.dir, exist_ok=True)  # init_file_dir (:605-606)
        self._xb0 = xb0
        self.load_eval_ckpts()
        self.get_current_states()

    # -- checkpoint / resume ---------------------------------------------------------------------------------
    def get_current_states(self):
        p = os.path.join(self.dir, "current_time.txt")
        self.current_time = _dt.datetime.fromisoformat(open(p).read().strip()) if os.path.exists(p) else self.start_time
        p = os.path.join(self.dir, "xb.npy")
        if os.path.exists(p):
            self.xb = torch.from_numpy(np.load(p)).to(self.dev)
        else:
            if self._xb0 is None:
                raise ValueError("no checkpoint and no initial background (get_initial_state reads ERA5)")
            self.xb = torch.as_tensor(np.asarray(self._xb0, np.float32)).to(self.dev)
        return self.current_time, self.xb

    def save_ckpt(self, finish: bool = False):
        if not finish:
            np.save(os.path.join(self.dir, "xb"), self.xb.cpu().numpy())
            with open(os.path.join(self.dir, "current_time.txt"), "w") as f:
                f.write(self.current_time.isoformat(sep=" "))

    def load_eval_ckpts(self):
        for k in self.metrics_list:
            p = os.path.join(self.dir, k + ".npy")
            if os.path.exists(p):
                self.metrics_list[k] = list(np.load(p))

    def save_eval_result(self, finish: bool = False):
        for k, v in self.metrics_list.items():
            np.save(os.path.join(self.dir, k), np.asarray(v))
        if not finish and self.save_field:
            stamp = self.current_time.isoformat(sep=" ")
            np.save(os.path.join(self.dir, f"xb_{stamp}"), self.xb.cpu().numpy())
            np.save(os.path.join(self.dir, f"xa_{stamp}"), self.xa.cpu().numpy())

    # -- the cycle ---------------------------------------------------------------------------------------------
    def one_step_DA(self, gt, xb, yo, H, R):
        prob = {"xb": xb, "yo": yo, "H": H, "R": R, "mean": self.mean, "std": self.std, "std_tr": self.std_tr}
        p = DAProblem(self.dec, prob, flow=self.flow, obs_coeff=self.obs_coeff, obs_interp=self.obs_interp)
        gt_d = torch.as_tensor(np.asarray(gt, np.float32)).to(self.dev) if not isinstance(gt, torch.Tensor) else gt
        res = one_step_da(p, self.Nit, gt=gt_d, metrics=self.metric)
        # da_4dvar.py:1285-1291: pass kk == 0 -> bg_*, `elif kk == Nit` -> ana_* (so Nit = 0 records only bg_*)
        w0, b0 = res["metrics"][0]
        self.metrics_list["bg_wrmse"].append(w0)
        self.metrics_list["bg_bias"].append(b0)
        if self.Nit > 0:
            w1, b1 = res["metrics"][self.Nit]
            self.metrics_list["ana_wrmse"].append(w1)
            self.metrics_list["ana_bias"].append(b1)
        self.last = res
        return res["xa"]

    def run_assimilation(self, log=None):
        epoch = 0
        while self.current_time + self.cycle_time <= self.end_time:
            yo, H, R, gt = self.obs.get_obs_info(self.current_time)
            self.xa = self.one_step_DA(gt, self.xb, yo, H, R)
            self.save_eval_result(finish=False)
            self.xb = integrate(self.fcst, self.xa, self.mean_d, self.std_d, 1)
            if log is not None:
                log(self.current_time, self.last)
            self.current_time = self.current_time + self.cycle_time
            if epoch % self.save_interval == 0:
                self.save_ckpt(finish=False)
            epoch += 1
        self.save_eval_result(finish=True)
