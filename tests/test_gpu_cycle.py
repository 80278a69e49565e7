"""The assimilation cycle (run_assimilation da_4dvar.py:1314-1342, checkpoint/resume :683-702,
device WRMSE/Bias :1256-1291) on the GPU against the oracle's restated cycle (oracle/da_ref.py run_cycles_ref)
and the G9-pinned metric restatement. Tiny networks (BASELINE config-1 decoder, tiny flow as the forecast
model) so the CPU oracle runs the same cycles in seconds. Tolerances: ~5x what the HIP path achieves (r06, profiles/r06/parity_margins.jsonl; SURVEY §8 c6 allows rel 1e-3
after L-BFGS)."""
import datetime as dt
import os

import numpy as np
import pytest
import torch

from conftest import GOLD, check, check_bitwise

pytestmark = pytest.mark.gpu

T0 = dt.datetime(2018, 1, 1, 0)


def _truth(t):
    from vaevar import config as C
    from vaevar.synth import smooth_field

    k = int((t - T0).total_seconds() // 3600)
    mean = np.asarray(C.MODEL_MEAN[:4], np.float32)[:, None, None]
    std = np.asarray(C.MODEL_STD[:4], np.float32)[:, None, None]
    return (mean + std * smooth_field(5000 + k, (4, 32, 64), sigma=3.0)).astype(np.float32)


def _setup():
    from vaevar.problem import obs_variance
    from vaevar.synth import smooth_field, splitmix_uniform
    from vaevar import config as C

    std = np.asarray(C.MODEL_STD[:4], np.float32)
    H = np.broadcast_to((splitmix_uniform(77, 32 * 64).reshape(32, 64) < 0.1).astype(np.float32),
                        (1, 4, 32, 64)).copy()
    R = np.broadcast_to(obs_variance(4, 0.005, 2, std)[None, :, None, None], (1, 4, 32, 64)).astype(np.float32).copy()
    xb0 = (_truth(T0) + 0.1 * std[:, None, None] * smooth_field(78, (4, 32, 64), sigma=3.0)).astype(np.float32)
    return H, R, xb0


def test_cycle_vs_oracle_and_resume(tmp_path):
    from oracle.da_ref import RefProblem, bias_ref, run_cycles_ref, wrmse_ref
    from oracle.lgunet_ref import lgunet_forward, synth_params
    from vaevar import config as C
    from vaevar.cycle import CyclicVAE4DVar, SyntheticObs
    from vaevar.engine import LGUnet

    H, R, xb0 = _setup()
    dec = LGUnet(C.TINY, 1, 1).load_synthetic()
    fc = LGUnet(C.TINY_FLOW, 1, 1).load_synthetic()  # the forecast model (same context as the decoder)
    obs = SyntheticObs(_truth, H, R)
    end = T0 + dt.timedelta(hours=18)
    cyc = CyclicVAE4DVar(dec, fc, obs, T0, end, Nit=1, name="tiny", out_dir=str(tmp_path), xb0=xb0)
    xas = []
    cyc.run_assimilation(log=lambda t, res: xas.append(res["xa"].cpu().numpy()))
    assert len(xas) == 3 and cyc.current_time == end
    # checkpoint written as the reference does (xb.npy + current_time.txt)
    d = os.path.join(str(tmp_path), "tiny")
    assert open(os.path.join(d, "current_time.txt")).read() == "2018-01-01 18:00:00"
    assert np.array_equal(np.load(os.path.join(d, "xb.npy")), cyc.xb.cpu().numpy())
    assert np.load(os.path.join(d, "ana_wrmse.npy")).shape == (3, 4)

    # the oracle's restated cycle on the same inputs
    torch.set_num_threads(16)
    dp, fp = synth_params(C.TINY), synth_params(C.TINY_FLOW)
    mean = torch.tensor(C.MODEL_MEAN[:4], dtype=torch.float32)
    std = torch.tensor(C.MODEL_STD[:4], dtype=torch.float32)

    def make_rp(k, xb):
        gt = _truth(T0 + dt.timedelta(hours=6 * k))[None]
        prob = {"xb": xb, "yo": gt, "H": H, "R": R, "mean": mean, "std": std,
                "std_tr": np.asarray(C.STD_TR[:4], np.float32)}
        return RefProblem(prob, lambda z: lgunet_forward(dp, C.TINY, z), C.TINY["img_size"])

    def fcst(xa):
        z = ((xa - mean.reshape(-1, 1, 1)) / std.reshape(-1, 1, 1)).unsqueeze(0)
        z = lgunet_forward(fp, C.TINY_FLOW, z)[:, :4]
        return z.reshape(4, 32, 64) * std.reshape(-1, 1, 1) + mean.reshape(-1, 1, 1)

    ref = run_cycles_ref(make_rp, torch.from_numpy(xb0), fcst, 3, 1, (4, 32, 64))
    for k in range(3):
        xr = ref[k]["xa"].numpy()
        e = float(np.linalg.norm(xas[k] - xr) / np.linalg.norm(xr - ref[k]["xb"].numpy()))
        gt = torch.from_numpy(_truth(T0 + dt.timedelta(hours=6 * k)))[None]
        xn = ((ref[k]["xa"] - mean.reshape(-1, 1, 1)) / std.reshape(-1, 1, 1))[None]
        gn = ((gt[0] - mean.reshape(-1, 1, 1)) / std.reshape(-1, 1, 1))[None]
        w = wrmse_ref(xn, gn, np.asarray(C.MODEL_STD[:4], np.float64)).numpy()
        b = bias_ref(xn, gn, np.asarray(C.MODEL_STD[:4], np.float64)).numpy()
        ew = float(np.abs(cyc.metrics_list["ana_wrmse"][k] - w).max() / np.abs(w).max())
        eb = float(np.abs(cyc.metrics_list["ana_bias"][k] - b).max() / np.abs(w).max())
        print(f"cycle {k}: xa increment rel {e:.1e}, ana WRMSE rel {ew:.1e}, bias rel {eb:.1e}")
        check(f"cycle {k} xa increment", e, 2e-4)
        check(f"cycle {k} ana WRMSE", ew, 1e-6)
        check(f"cycle {k} ana bias", eb, 1e-6)

    # resume: a new driver over the same directory continues from the checkpoint (get_current_states)
    cyc2 = CyclicVAE4DVar(dec, fc, obs, T0, end + dt.timedelta(hours=6), Nit=1, name="tiny", out_dir=str(tmp_path))
    assert cyc2.current_time == end
    check_bitwise("cycle resume xb", cyc2.xb, cyc.xb)
    assert len(cyc2.metrics_list["ana_wrmse"]) == 3
    cyc2.run_assimilation()
    assert len(cyc2.metrics_list["ana_wrmse"]) == 4


@pytest.mark.parametrize("tag,Hs,Ws,seed", [("s", 128, 256, 901), ("l", 721, 1440, 902)])
def test_metrics_kernel_g9(tag, Hs, Ws, seed):
    """vv_metrics vs the genuine Metrics.WRMSE / Bias (G9)."""
    from vaevar import config as C
    from vaevar.engine import Context
    from vaevar.metrics import Metrics
    from vaevar.problem import make_problem

    g = np.load(os.path.join(GOLD, "g9_metrics.npz"))
    p = make_problem(nch=69, Hs=Hs, Ws=Ws, T=1, seed=seed)
    m = Metrics(Context.get(0))
    w, b = m.wrmse_bias(torch.from_numpy(p["xb"]).cuda(), torch.from_numpy(p["gt"][0]).cuda())
    ew = float(np.abs(w.cpu().numpy() - g["wrmse_" + tag]).max() / np.abs(g["wrmse_" + tag]).max())
    eb = float(np.abs(b.cpu().numpy() - g["bias_" + tag]).max() / np.abs(g["bias_" + tag]).max())
    print(f"G9 {Hs}x{Ws}: WRMSE rel {ew:.1e}, Bias rel {eb:.1e}")
    check(f"G9 {Hs}x{Ws} WRMSE", ew, 5e-7)
    check(f"G9 {Hs}x{Ws} Bias", eb, 1e-6)


def test_cycle_real_obs_matches_manual_composition(tmp_path):
    """obs_type 'real_simu_nofiltering' through the cycle driver (full decoder, 69ch 128x256, the flow stand-in as
    the forecast, 2 cycles, Nit=1) equals the same steps composed by hand from DAProblem / one_step_da / integrate
    bit for bit; the observation-space fields have 4 + 5*40 channels."""
    from vaevar import config as C
    from vaevar.cycle import CyclicVAE4DVar, SyntheticRealObs
    from vaevar.da import one_step_da
    from vaevar.engine import DAProblem, LGUnet, integrate, obs_augment
    from vaevar.problem import ObsInterpolater, make_problem
    from vaevar.synth import smooth_field, splitmix_uniform

    oi = ObsInterpolater(13, 40)
    mean = np.asarray(C.MODEL_MEAN, np.float32)[:, None, None]
    std = np.asarray(C.MODEL_STD, np.float32)[:, None, None]

    def truth(t):
        k = int((t - T0).total_seconds() // 3600)
        return (mean + std * smooth_field(6000 + k, (69, 128, 256))).astype(np.float32)

    p = make_problem(nch=69, Hs=128, Ws=256, T=1, seed=8080, obs_frac=0.03)
    H = (splitmix_uniform(81, 204 * 128 * 256).reshape(1, 204, 128, 256) < 0.03).astype(np.float32)
    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    fc = LGUnet(C.FLOW, 1, 1).load_synthetic()
    obs = SyntheticRealObs(dec.ctx, truth, H, p["R"], oi.interp)
    end = T0 + dt.timedelta(hours=12)
    cyc = CyclicVAE4DVar(dec, fc, obs, T0, end, Nit=1, name="real", out_dir=str(tmp_path), xb0=p["xb"],
                         obs_interp=oi.interp)
    xas = []
    cyc.run_assimilation(log=lambda t, res: xas.append(res["xa"].clone()))
    assert len(xas) == 2
    # by hand
    interp = torch.from_numpy(oi.interp).cuda()
    Rd = obs_augment(dec.ctx, interp, torch.from_numpy(p["R"]).cuda())
    xb = torch.from_numpy(p["xb"]).cuda()
    for k in range(2):
        gt = torch.from_numpy(truth(T0 + dt.timedelta(hours=6 * k)))[None].cuda()
        Hd = torch.from_numpy(H).cuda()
        yo = obs_augment(dec.ctx, interp, gt) * Hd
        assert yo.shape[1] == 204
        prob = DAProblem(dec, {"xb": xb, "yo": yo, "H": Hd, "R": Rd, "mean": cyc.mean, "std": cyc.std,
                               "std_tr": cyc.std_tr}, obs_interp=oi.interp)
        xa = one_step_da(prob, nit=1)["xa"]
        check_bitwise(f"real-obs cycle {k} xa vs hand composition", xa, xas[k])
        xb = integrate(fc, xa, cyc.mean_d, cyc.std_d, 1)
    check_bitwise("real-obs cycle xb vs hand composition", xb, cyc.xb)
    w = np.asarray(cyc.metrics_list["ana_wrmse"])
    assert w.shape == (2, 69) and np.isfinite(w).all()
