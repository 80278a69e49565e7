"""ORACLE (survey container only) — generate golden fixtures from the REAL
reference (`/root/reference`, imported through oracle/ref_harness.py) and pin
the oracle's restatement against it.

Run:  PYTHONDONTWRITEBYTECODE=1 python -B oracle/make_golden.py [--full]

Writes small .npz fixtures to tests/golden/ (inputs are regenerated from the
counter-hash RNG in vae-var_amd/vaevar/synth.py; only outputs and small inputs
are stored):

  g1_tiny_decoder.npz   G1: tiny networks_old.LGUnet_all: z, cotangent, out, d<out,cot>/dz
  g2_swin_block.npz     G2: single SwinTransformerBlock (shift 0 / 2): x, out, grad, attn_mask
  g4_nearest_maps.npz   G4: nearest index maps of F.interpolate 721<->128, 1440<->256
  g5_tiny_lbfgs.npz     G5: restated vae4dvar loop on the tiny decoder (Nit=2): J per outer pass, xa
  g5b_tiny_4dvar.npz    tiny decoder + tiny flow, T=2: J terms and dJ/dz of one closure
  g6_one_step_da_c5.npz G6 (--g6, ~5 min): the genuine cyclic_4dvar.one_step_DA(..., 'vae4dvar') at 721x1440, T=2,
                        Nit=1 (config 5): printed J per outer pass, sampled xa + sums
  g8_real_obs.npz       G8 (--g8, ~3 min): the genuine obs_interpolater(13, 40) matrices, get_R_matrix_from_gt on a
                        small R, and cyclic_4dvar.one_step_DA(..., 'vae4dvar') with obs_type 'real' at 721x1440,
                        T=1, Nit=1 (J per outer pass, sampled xa)
  g9_metrics.npz        G9: the genuine utils.metrics.Metrics WRMSE / Bias as one_step_DA calls them
                        (da_4dvar.py:1256-1262) at 128x256 and 721x1440
  g7_tiny_lgunet1.npz   G7: tiny networks.LGUnet_all_1 (RoPE, -inf mask, global LG window, 3 levels): out
  g14_sc4dvar_reference.npz  G14 (~2 min): the genuine sc4dvar get_static_info / transform / loss + backward / Nit=1
                        L-BFGS pass with the oracle's float64 SHT as the torch_harmonics stub (float64 and float32 runs)
  g15_config5_trajectory.npz  G15 (--g15, ~25 min): the genuine one_step_DA at 721x1440, T=2, Nit=5 (config 5's
                        budget): J per pass, line-search steps, sampled xa
  g16_config4_trajectory.npz  G16 (--g16, ~20 min): config 4 (T=6, decoder + flow stand-in) with torch.optim.LBFGS,
                        Nit 10 at 128x256: J per pass, line-search steps, sampled xa
  g13_config3_trajectory.npz  G13 (--g13, ~30 min): config 3 (T=2, decoder + flow stand-in) with torch.optim.LBFGS,
                        Nit 10 at 128x256: J per pass, line-search steps, sampled xa
  g3_full_decoder.npz   G3 (--full): full parameters0_old decoder @128x256: sampled out/grad + sums,
                        and one config-2 closure (J_b, J_o, sampled dJ/dz)
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vae-var_amd"))

from oracle import ref_harness  # noqa: E402
from oracle.lgunet_ref import lgunet_forward, param_shapes, synth_params, swin_block, shift_mask  # noqa: E402
from oracle.da_ref import RefProblem, oracle_problem, one_step_da_ref  # noqa: E402
from vaevar import config as C  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402
from vaevar.synth import smooth_field, uniform_sym, param_value  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")


def build_ref(tr, cfg, prefix=""):
    torch.manual_seed(0)
    m = tr.LGUnet_all(rank=0, **cfg)
    p = synth_params(cfg)
    sd = m.state_dict()
    missing = [k for k in sd if k not in p]
    assert all(k.endswith("relative_position_index") or k.endswith("attn_mask") for k in missing), missing[:5]
    extra = [k for k in p if k not in sd]
    assert not extra, extra[:5]
    for k, v in p.items():
        assert tuple(sd[k].shape) == tuple(v.shape), (k, sd[k].shape, v.shape)
    m.load_state_dict(p, strict=False)
    m.eval()
    return m, p


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def g1(tr):
    cfg = C.TINY
    m, p = build_ref(tr, cfg)
    z = torch.from_numpy(0.5 * smooth_field(101, (1, 4, 32, 64), sigma=2.0)).requires_grad_(True)
    cot = torch.from_numpy(uniform_sym(102, (1, 4, 32, 64), 1.0))
    out = m(z)
    (out * cot).sum().backward()
    # the oracle restatement on the same inputs
    z2 = z.detach().clone().requires_grad_(True)
    out2 = lgunet_forward(p, cfg, z2)
    (out2 * cot).sum().backward()
    e_out, e_g = rel(out2.detach(), out.detach()), rel(z2.grad, z.grad)
    print(f"G1 tiny decoder: restatement vs reference rel out {e_out:.2e} grad {e_g:.2e}")
    assert e_out < 1e-5 and e_g < 1e-5
    np.savez(os.path.join(GOLD, "g1_tiny_decoder.npz"), z=z.detach().numpy(), cot=cot.numpy(),
             out=out.detach().numpy(), grad=z.grad.numpy())


def g2(sb):
    out = {}
    for shift in (0, 2):
        torch.manual_seed(0)
        blk = sb.SwinTransformerBlock(dim=32, input_resolution=(16, 32), num_heads=2, window_size=4,
                                      shift_size=shift)
        pre = f"g2.s{shift}"
        sd = blk.state_dict()
        p = {}
        for k, v in sd.items():
            if k.endswith("relative_position_index") or k.endswith("attn_mask"):
                continue
            p[f"{pre}.{k}"] = torch.from_numpy(param_value(f"{pre}.{k}", tuple(v.shape)))
        blk.load_state_dict({k[len(pre) + 1:]: v for k, v in p.items()}, strict=False)
        x = torch.from_numpy(uniform_sym(200 + shift, (1, 16, 32, 32), 1.0)).requires_grad_(True)
        cot = torch.from_numpy(uniform_sym(210 + shift, (1, 16, 32, 32), 1.0))
        y = blk(x)
        (y * cot).sum().backward()
        x2 = x.detach().clone().requires_grad_(True)
        y2 = swin_block(x2, p, pre, 2, 4, shift)
        (y2 * cot).sum().backward()
        print(f"G2 shift {shift}: rel out {rel(y2.detach(), y.detach()):.2e} grad {rel(x2.grad, x.grad):.2e}")
        assert rel(y2.detach(), y.detach()) < 1e-5 and rel(x2.grad, x.grad) < 1e-5
        out[f"x_s{shift}"] = x.detach().numpy()
        out[f"cot_s{shift}"] = cot.numpy()
        out[f"out_s{shift}"] = y.detach().numpy()
        out[f"grad_s{shift}"] = x.grad.numpy()
        if shift:
            ref_mask = blk.attn_mask.numpy()
            assert np.array_equal(ref_mask, shift_mask(16, 32, 4, shift).numpy())
            out["attn_mask_s2"] = ref_mask
            out["rel_index"] = blk.attn.relative_position_index.numpy()
    np.savez(os.path.join(GOLD, "g2_swin_block.npz"), **out)


def g4():
    import torch.nn.functional as F

    out = {}
    for (a, b), key in (((721, 128), "lat_721_to_128"), ((128, 721), "lat_128_to_721"),
                        ((1440, 256), "lon_1440_to_256"), ((256, 1440), "lon_256_to_1440")):
        ramp = torch.arange(a, dtype=torch.float32).view(1, 1, a, 1)
        m = F.interpolate(ramp, (b, 1)).view(-1).to(torch.int64).numpy()
        out[key] = m.astype(np.int32)
    np.savez(os.path.join(GOLD, "g4_nearest_maps.npz"), **out)
    print("G4 nearest maps written")


def tiny_problem(T=1):
    return make_problem(nch=4, Hs=32, Ws=64, T=T, seed=777, obs_frac=0.1)


def g5(tr):
    cfg = C.TINY
    m, p = build_ref(tr, cfg)
    prob = tiny_problem()
    rp = RefProblem(prob, m, cfg["img_size"])
    t0 = time.time()
    xa, z, js, nev, nit = one_step_da_ref(rp, 2, (4, 32, 64))
    print(f"G5 reference-module L-BFGS: J {js}  evals {nev} iters {nit} ({time.time() - t0:.1f}s)")
    ro = oracle_problem(prob, p, cfg)
    xa2, z2, js2, nev2, nit2 = one_step_da_ref(ro, 2, (4, 32, 64))
    print(f"G5 oracle restatement:     J {js2}  evals {nev2} iters {nit2}; xa rel {rel(xa2, xa):.2e}")
    np.savez(os.path.join(GOLD, "g5_tiny_lbfgs.npz"), J=np.array(js, np.float64), n_eval=nev, n_iter=nit,
             xa=xa.numpy(), z=z.numpy())


def g5b(tr):
    cfg, fcfg = C.TINY, C.TINY_FLOW
    m, p = build_ref(tr, cfg)
    fm, fp = build_ref(tr, fcfg)
    prob = tiny_problem(T=2)
    z = torch.from_numpy(0.3 * smooth_field(303, (1, 4, 32, 64), sigma=2.0)).requires_grad_(True)
    rp = RefProblem(prob, m, cfg["img_size"], fm)
    r, o = rp.loss_terms(z)
    (r + o).backward()
    ro = oracle_problem(prob, p, cfg, fp, fcfg)
    z2 = z.detach().clone().requires_grad_(True)
    r2, o2 = ro.loss_terms(z2)
    (r2 + o2).backward()
    print(f"G5b tiny 4D-Var T=2: J_b {float(r):.6e} J_o {float(o):.6e}; oracle rel J_o "
          f"{abs(float(o2) - float(o)) / abs(float(o)):.2e} grad {rel(z2.grad, z.grad):.2e}")
    np.savez(os.path.join(GOLD, "g5b_tiny_4dvar.npz"), z=z.detach().numpy(), J_b=float(r), J_o=float(o),
             grad=z.grad.numpy())


def sample_idx(n, k=4096, seed=909):
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n, size=k, replace=False)).astype(np.int64)


def g3(tr):
    cfg = C.DECODER
    t0 = time.time()
    m, p = build_ref(tr, cfg)
    print(f"G3 built full decoder in {time.time() - t0:.1f}s")
    z = torch.from_numpy(0.5 * smooth_field(401, (1, 32, 128, 256))).requires_grad_(True)
    cot = torch.from_numpy(uniform_sym(402, (1, 69, 128, 256), 1.0))
    t0 = time.time()
    out = m(z)
    (out * cot).sum().backward()
    print(f"G3 reference fwd+bwd {time.time() - t0:.1f}s")
    z2 = z.detach().clone().requires_grad_(True)
    out2 = lgunet_forward(p, cfg, z2)
    (out2 * cot).sum().backward()
    print(f"G3 restatement rel out {rel(out2.detach(), out.detach()):.2e} grad {rel(z2.grad, z.grad):.2e}")
    io = sample_idx(out.numel())
    ig = sample_idx(z.numel(), seed=910)
    o = out.detach().numpy().reshape(-1).astype(np.float64)
    g = z.grad.numpy().reshape(-1).astype(np.float64)
    res = dict(idx_out=io, out_sample=o[io].astype(np.float32), out_sum=o.sum(), out_sumsq=(o * o).sum(),
               out_abssum=np.abs(o).sum(), idx_grad=ig, grad_sample=g[ig].astype(np.float32), grad_sum=g.sum(),
               grad_sumsq=(g * g).sum(), grad_abssum=np.abs(g).sum())
    # one config-2 closure (T=1, 128x256 state) at a non-zero latent
    prob = make_problem(nch=69, Hs=128, Ws=256, T=1, seed=20250620)
    rp = RefProblem(prob, m, cfg["img_size"])
    zc = torch.from_numpy(0.3 * smooth_field(403, (1, 32, 128, 256))).requires_grad_(True)
    rr, oo = rp.loss_terms(zc)
    (rr + oo).backward()
    gc = zc.grad.numpy().reshape(-1).astype(np.float64)
    res.update(J_b=float(rr), J_o=float(oo), cgrad_sample=gc[ig].astype(np.float32), cgrad_sumsq=(gc * gc).sum(),
               cgrad_sum=gc.sum())
    print(f"G3 closure J_b {float(rr):.6e} J_o {float(oo):.6e} |g| {np.sqrt((gc * gc).sum()):.6e}")
    np.savez(os.path.join(GOLD, "g3_full_decoder.npz"), **res)


def ref_cfg_l1(cfg):
    c = {k: v for k, v in cfg.items() if k != "arch"}
    c.update(in_chans=sum(cfg["inchans_list"]), out_chans=sum(cfg["outchans_list"]), Weather_T=1, drop_path=0.0,
             use_checkpoint=False, inp_length=1, use_mlp=False)
    return c


def g7():
    """G7: the real networks.LGUnet_all_1 on TINY_FCST with synthetic weights; pins oracle/lgunet1_ref.py."""
    import importlib

    from oracle.lgunet1_ref import lgunet1_forward, synth_params as synth1

    L1 = importlib.import_module("networks.LGUnet_all")
    cfg = C.TINY_FCST
    torch.manual_seed(0)
    m = L1.LGUnet_all_1(**ref_cfg_l1(cfg))
    p = synth1(cfg)
    sd = m.state_dict()
    assert set(sd) == set(p), (set(sd) ^ set(p))
    m.load_state_dict(p, strict=True)
    m.eval()
    x = torch.from_numpy(smooth_field(701, (1, C.in_channels(cfg)) + tuple(cfg["img_size"])))
    with torch.no_grad():
        y = m(x)
        yo = lgunet1_forward(p, cfg, x)
    print(f"G7 tiny LGUnet_all_1: out {tuple(y.shape)} oracle rel {rel(yo, y):.2e}")
    np.savez(os.path.join(GOLD, "g7_tiny_lgunet1.npz"), out=y.numpy())


class LineSearchRecorder:
    """Records (t, ls_func_evals) of every torch.optim.lbfgs._strong_wolfe call the reference's LBFGS makes, for
    the fixed-step replay comparison of SURVEY §8 c6 (vaevar.lbfgs.LBFGS.replay)."""

    def __enter__(self):
        import torch.optim.lbfgs as tl

        self.tl, self.orig, self.steps = tl, tl._strong_wolfe, []

        def rec(*a, **k):
            out = self.orig(*a, **k)
            self.steps.append((float(out[2]), int(out[3])))
            return out

        tl._strong_wolfe = rec
        return self

    def __exit__(self, *exc):
        self.tl._strong_wolfe = self.orig
        return False


def genuine_one_step_da(tr, T, nit, seed, tag):
    """Run the reference's own cyclic_4dvar.one_step_DA vae4dvar branch (da_4dvar.py:1179-1306) on CPU at 721x1440
    (SURVEY §8 c2 iv: object.__new__ + attributes, device 'cuda' rewritten to 'cpu'), synthetic weights, flow
    stand-in for T > 1, make_problem(seed) inputs. Returns (J per printed pass, xa, line-search steps, prob)."""
    import contextlib
    import importlib
    import io
    import re

    from torch.overrides import TorchFunctionMode

    class CPUMode(TorchFunctionMode):
        def __torch_function__(self, func, types, args=(), kwargs=None):
            kwargs = dict(kwargs or {})
            if "device" in kwargs and kwargs["device"] is not None and str(kwargs["device"]).startswith("cuda"):
                kwargs["device"] = "cpu"
            return func(*args, **kwargs)

    cwd = os.getcwd()
    os.chdir(ref_harness.REF)
    da = importlib.import_module("da_4dvar")
    metrics = importlib.import_module("utils.metrics")
    vae_mod = importlib.import_module("nf_model.vae")
    vae = vae_mod.VAE_lr("parameters0_old")
    os.chdir(cwd)
    dec_p = synth_params(C.DECODER)
    missing, unexpected = vae.dec.load_state_dict(dec_p, strict=False)
    assert not unexpected and all(k.endswith(("relative_position_index", "attn_mask")) for k in missing)
    flow = None
    if T > 1:
        flow_cfg = {k: v for k, v in C.FLOW.items() if k != "arch"}
        flow = tr.LGUnet_all(rank=0, **flow_cfg)
        missing, unexpected = flow.load_state_dict(synth_params(C.FLOW), strict=False)
        assert not unexpected and all(k.endswith(("relative_position_index", "attn_mask")) for k in missing)
    a = object.__new__(da.cyclic_4dvar)
    a.device = "cpu"
    a.da_win, a.obs_type, a.obs_coeff, a.Nit, a.use_eval = T, "synthetic", 1.0, nit, False
    a.nchannel, a.nlev, a.nlat, a.nlon, a.current_time = 69, 13, 721, 1440, tag
    a.metric = metrics.Metrics()
    a.metrics_list = {"bg_wrmse": [], "bg_bias": [], "ana_wrmse": [], "ana_bias": []}
    a.model_mean, a.model_std, a.model_mean_gpu, a.model_std_gpu = a.get_model_mean_std()
    a.vae, a.flow_model = vae, flow
    prob = make_problem(nch=69, Hs=721, Ws=1440, T=T, seed=seed)
    t = lambda k: torch.from_numpy(prob[k])
    old_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *args, **kw: self
    buf = io.StringIO()
    t0 = time.time()
    try:
        with CPUMode(), contextlib.redirect_stdout(buf), LineSearchRecorder() as ls:
            xa = a.one_step_DA(t("gt"), t("xb"), t("yo"), t("H"), t("R"), "vae4dvar")
    finally:
        torch.Tensor.cuda = old_cuda
    log = buf.getvalue()
    J = [(float(m.group(1)), float(m.group(2))) for m in re.finditer(r"loss reg: ([-0-9.e+]+) loss obs: ([-0-9.e+]+)", log)]
    print(f"{tag} one_step_DA 721x1440 T={T} Nit={nit}: {time.time() - t0:.0f}s, J per pass {J}", flush=True)
    return J, xa.detach().numpy().astype(np.float32), ls.steps, prob


def g6(tr):
    """G6: the genuine one_step_DA at 721x1440 with T=2 (flow stand-in), Nit=1, seed 20250620 (config 5's grid)."""
    J, xa, steps, prob = genuine_one_step_da(tr, 2, 1, 20250620, "G6")
    idx = sample_idx(xa.size, 8192, 606)
    flat = xa.reshape(-1).astype(np.float64)
    np.savez(os.path.join(GOLD, "g6_one_step_da_c5.npz"), J=np.array(J), idx_xa=idx, xa_sample=xa.reshape(-1)[idx],
             ls_t=np.array([x[0] for x in steps]), ls_evals=np.array([x[1] for x in steps]),
             xa_sum=flat.sum(), xa_sumsq=(flat * flat).sum(),
             dxa_sumsq=((flat - prob["xb"].reshape(-1).astype(np.float64)) ** 2).sum())


def g15(tr):
    """G15 (BASELINE config 5 at its budget): the genuine one_step_DA at 721x1440, T=2, Nit=5 (the bench's 50-iteration
    budget), seed 20250620: J per printed pass (4 digits), every line search's (t, evals), sampled xa + sums."""
    J, xa, steps, prob = genuine_one_step_da(tr, 2, 5, 20250620, "G15")
    idx = sample_idx(xa.size, 8192, 1515)
    flat = xa.reshape(-1).astype(np.float64)
    np.savez(os.path.join(GOLD, "g15_config5_trajectory.npz"), J=np.array(J), idx_xa=idx,
             xa_sample=xa.reshape(-1)[idx], ls_t=np.array([x[0] for x in steps]),
             ls_evals=np.array([x[1] for x in steps]), xa_sum=flat.sum(), xa_sumsq=(flat * flat).sum(),
             dxa_sumsq=((flat - prob["xb"].reshape(-1).astype(np.float64)) ** 2).sum())


def g8(tr):
    """G8: the real-observation operator of the genuine reference — obs_interpolater (da_4dvar.py:
    62-94), get_R_matrix_from_gt (:729-756) and the vae4dvar loss with x_aug (:1196-1206) inside the genuine
    one_step_DA at 721x1440, T=1, Nit=1, on make_real_problem(seed=20250622) inputs and synthetic weights."""
    import contextlib
    import importlib
    import io
    import re

    from torch.overrides import TorchFunctionMode
    from vaevar.problem import make_real_problem

    class CPUMode(TorchFunctionMode):
        def __torch_function__(self, func, types, args=(), kwargs=None):
            kwargs = dict(kwargs or {})
            if "device" in kwargs and kwargs["device"] is not None and str(kwargs["device"]).startswith("cuda"):
                kwargs["device"] = "cpu"
            return func(*args, **kwargs)

    cwd = os.getcwd()
    os.chdir(ref_harness.REF)
    da = importlib.import_module("da_4dvar")
    metrics = importlib.import_module("utils.metrics")
    vae_mod = importlib.import_module("nf_model.vae")
    vae = vae_mod.VAE_lr("parameters0_old")
    os.chdir(cwd)
    old_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *args, **kw: self
    try:
        oi = da.obs_interpolater(13, 40)
        interp, interp_inv = oi.interp.numpy().copy(), oi.interp_inv.numpy().copy()
        # get_R_matrix_from_gt on a small spatially varying R (T=2, 69, 4, 8)
        a = object.__new__(da.cyclic_4dvar)
        a.nlev, a.obs_interp = 13, oi
        rs = make_problem(nch=69, Hs=4, Ws=8, T=2, seed=811)["R"]
        rs = (rs * (1.0 + 0.5 * smooth_field(812, rs.shape, sigma=1.0) ** 2)).astype(np.float32)
        a.static_info = {"R": torch.from_numpy(rs)}
        r_aug = a.get_R_matrix_from_gt(None, None).numpy().copy()
        # the genuine one_step_DA with obs_type 'real'
        dec_p = synth_params(C.DECODER)
        missing, unexpected = vae.dec.load_state_dict(dec_p, strict=False)
        assert not unexpected and all(k.endswith(("relative_position_index", "attn_mask")) for k in missing)
        b = object.__new__(da.cyclic_4dvar)
        b.device = "cpu"
        b.da_win, b.obs_type, b.obs_coeff, b.Nit, b.use_eval = 1, "real", 1.0, 1, False
        b.nchannel, b.nlev, b.nlat, b.nlon, b.current_time = 69, 13, 721, 1440, "G8"
        b.metric = metrics.Metrics()
        b.metrics_list = {"bg_wrmse": [], "bg_bias": [], "ana_wrmse": [], "ana_bias": []}
        b.model_mean, b.model_std, b.model_mean_gpu, b.model_std_gpu = b.get_model_mean_std()
        b.vae, b.obs_interp = vae, oi
        prob = make_real_problem(Hs=721, Ws=1440, T=1, seed=20250622)
        t = lambda k: torch.from_numpy(prob[k])
        buf = io.StringIO()
        t0 = time.time()
        with CPUMode(), contextlib.redirect_stdout(buf), LineSearchRecorder() as ls:
            xa = b.one_step_DA(t("gt"), t("xb"), t("yo"), t("H"), t("R"), "vae4dvar")
    finally:
        torch.Tensor.cuda = old_cuda
    log = buf.getvalue()
    J = [(float(m.group(1)), float(m.group(2))) for m in re.finditer(r"loss reg: ([-0-9.e+]+) loss obs: ([-0-9.e+]+)", log)]
    xa = xa.detach().numpy().astype(np.float32)
    idx = sample_idx(xa.size, 8192, 808)
    flat = xa.reshape(-1).astype(np.float64)
    print(f"G8 real-obs one_step_DA 721x1440 T=1 Nit=1: {time.time() - t0:.0f}s, J per pass {J}")
    np.savez(os.path.join(GOLD, "g8_real_obs.npz"), interp=interp, interp_inv=interp_inv, r_aug=r_aug, J=np.array(J),
             ls_t=np.array([x[0] for x in ls.steps]), ls_evals=np.array([x[1] for x in ls.steps]),
             idx_xa=idx, xa_sample=xa.reshape(-1)[idx], xa_sum=flat.sum(),
             dxa_sumsq=((flat - prob["xb"].reshape(-1).astype(np.float64)) ** 2).sum())


def g9():
    """G9: Metrics.WRMSE / Metrics.Bias (utils/metrics.py) exactly as one_step_DA's logging calls
    them (da_4dvar.py:1256-1262): normalised by model_mean_gpu/model_std_gpu (fp32), scaled by model_std (f64)."""
    import importlib

    cwd = os.getcwd()
    os.chdir(ref_harness.REF)
    da = importlib.import_module("da_4dvar")
    metrics = importlib.import_module("utils.metrics")
    os.chdir(cwd)
    a = object.__new__(da.cyclic_4dvar)
    a.device = "cpu"
    mean, std, mean_g, std_g = a.get_model_mean_std()
    m = metrics.Metrics()
    out = {}
    for tag, (Hs, Ws, seed) in {"s": (128, 256, 901), "l": (721, 1440, 902)}.items():
        p = make_problem(nch=69, Hs=Hs, Ws=Ws, T=1, seed=seed)
        xhat, gt = torch.from_numpy(p["xb"]), torch.from_numpy(p["gt"][0])
        xn = (xhat - mean_g.reshape(-1, 1, 1)) / std_g.reshape(-1, 1, 1)
        gn = (gt - mean_g.reshape(-1, 1, 1)) / std_g.reshape(-1, 1, 1)
        w = m.WRMSE(xn.unsqueeze(0), gn.unsqueeze(0), None, None, std)
        b = m.Bias(xn.unsqueeze(0), gn.unsqueeze(0), None, None, std)
        out["wrmse_" + tag] = w.numpy()
        out["bias_" + tag] = b.numpy()
        print(f"G9 {Hs}x{Ws}: wrmse dtype {w.dtype}, z500 {float(w[11]):.6g}, bias z500 {float(b[11]):.6g}")
    np.savez(os.path.join(GOLD, "g9_metrics.npz"), model_std=std, **out)


def g10(tr):
    """G10 (BASELINE config 2 at its full budget): the reference's networks_old.LGUnet_all decoder
    with torch.optim.LBFGS(history 10, max_iter 10, strong Wolfe) on the restated vae4dvar closure
    (da_4dvar.py:1183-1246; the genuine one_step_DA hard-codes 721x1440, so the 128x256-state case is restated,
    exactly as G5), Nit = 10 outer passes: J per pass, every line search's (t, evals), sampled xa. The decoder
    parameters are frozen (requires_grad False): the latent gradient is the same computation, the unused
    weight gradients (quirk Q5) only cost time."""
    cfg = C.DECODER
    m, p = build_ref(tr, cfg)
    for v in m.parameters():
        v.requires_grad_(False)
    prob = make_problem(nch=69, Hs=128, Ws=256, T=1, seed=20250620)
    rp = RefProblem(prob, m, cfg["img_size"])
    t0 = time.time()
    with LineSearchRecorder() as ls:
        xa, z, js, nev, nit = one_step_da_ref(rp, 10, (32, 128, 256),
                                              log=lambda k, j: print(f"G10 pass {k}: J_b {j[0]:.6e} J_o {j[1]:.6e} "
                                                                     f"({time.time() - t0:.0f}s)", flush=True))
    xa = xa.numpy().astype(np.float32)
    idx = sample_idx(xa.size, 8192, 1010)
    flat = xa.reshape(-1).astype(np.float64)
    print(f"G10 config-2 trajectory: {time.time() - t0:.0f}s, evals {nev}, iters {nit}, J {js}")
    np.savez(os.path.join(GOLD, "g10_config2_trajectory.npz"), J=np.array(js, np.float64), n_eval=nev, n_iter=nit,
             ls_t=np.array([x[0] for x in ls.steps]), ls_evals=np.array([x[1] for x in ls.steps]),
             idx_xa=idx, xa_sample=xa.reshape(-1)[idx], xa_sum=flat.sum(),
             dxa_sumsq=((flat - prob["xb"].reshape(-1).astype(np.float64)) ** 2).sum())


def g13(tr):
    """G13 (BASELINE config 3 at its full budget): the reference's networks_old.LGUnet_all decoder AND
    the flow stand-in (the same module class with C.FLOW's channel lists) inside the restated 4D-Var closure with
    T = 2 (da_4dvar.py:1183-1208: the flow applied once through integrate, :666-681), torch.optim.LBFGS(history 10,
    max_iter 10, strong Wolfe), Nit = 10 outer passes at 128x256: J per pass, every line search's (t, evals),
    sampled xa. Parameters frozen as in G10 (the unused weight gradients only cost time)."""
    m, _ = build_ref(tr, C.DECODER)
    fm, _ = build_ref(tr, {k: v for k, v in C.FLOW.items() if k != "arch"})
    for v in list(m.parameters()) + list(fm.parameters()):
        v.requires_grad_(False)
    prob = make_problem(nch=69, Hs=128, Ws=256, T=2, seed=20250620)
    rp = RefProblem(prob, m, C.DECODER["img_size"], fm)
    t0 = time.time()
    with LineSearchRecorder() as ls:
        xa, z, js, nev, nit = one_step_da_ref(rp, 10, (32, 128, 256),
                                              log=lambda k, j: print(f"G13 pass {k}: J_b {j[0]:.6e} J_o {j[1]:.6e} "
                                                                     f"({time.time() - t0:.0f}s)", flush=True))
    xa = xa.numpy().astype(np.float32)
    idx = sample_idx(xa.size, 8192, 1313)
    flat = xa.reshape(-1).astype(np.float64)
    print(f"G13 config-3 trajectory: {time.time() - t0:.0f}s, evals {nev}, iters {nit}, J {js}")
    np.savez(os.path.join(GOLD, "g13_config3_trajectory.npz"), J=np.array(js, np.float64), n_eval=nev, n_iter=nit,
             ls_t=np.array([x[0] for x in ls.steps]), ls_evals=np.array([x[1] for x in ls.steps]),
             idx_xa=idx, xa_sample=xa.reshape(-1)[idx], xa_sum=flat.sum(),
             dxa_sumsq=((flat - prob["xb"].reshape(-1).astype(np.float64)) ** 2).sum())


class _RecordingLBFGS(torch.optim.LBFGS):
    """torch.optim.LBFGS as da_4dvar.py:1119 builds it, recording every closure value; with `fixed` set, step()
    instead puts the control variable at `fixed`, evaluates the reference's closure once and records J and dJ/dw
    (one genuine loss + backward, da_4dvar.py:1099-1107)."""

    fixed = None
    log = None

    def step(self, closure):
        w = self.param_groups[0]["params"][0]
        if _RecordingLBFGS.fixed is not None:
            with torch.no_grad():
                w.copy_(_RecordingLBFGS.fixed)
            v = closure()
            _RecordingLBFGS.log.append((float(v.detach()), w.grad.detach().clone()))
            return v

        def rec():
            v = closure()
            _RecordingLBFGS.log.append((float(v.detach()), None))
            return v

        out = super().step(rec)
        _RecordingLBFGS.w = w.detach().clone()
        return out


G14_NIT = 2


def g14(tr):
    """G14: the reference's OWN sc4dvar code around the SHT — get_static_info (da_4dvar.py:608-638:
    zonal kernel, its SHT, sph_scale, R), transform (:878-931: the 11/len^2 scaling, balance regression, std_sur,
    vertical EOFs, partial_x / partial_y incl. torch.gradient, the 721x1440 interpolation, + xb), and the loss +
    backward and L-BFGS pass of one_step_DA(..., 'sc4dvar') (:1064-1177) — with the oracle's float64 SHT installed as
    torch_harmonics.RealSHT / InverseRealSHT (absent here; the SHT itself stays unpinned). B statistics: the
    reference's dataset/bq_info_lr; obs_var from the genuine data_reader (:106-127, modify_tp 2), q_type -1.
    Two runs: (a) float64 default dtype (the B statistics as float64) — the restatement must match it to float64
    rounding; (b) the reference as it runs (float32; the SHT stub computes in float64 and rounds to float32) — the
    GPU fixture."""
    import contextlib
    import importlib
    import io

    from oracle.sc4dvar_ref import SHT, Sc4dvarRef, load_bq

    class RealSHTStub(torch.nn.Module):
        def __init__(self, nlat, nlon, grid="equiangular"):
            super().__init__()
            assert grid == "equiangular"
            self.s = SHT(nlat, nlon)

        def forward(self, x):
            y = self.s.forward(x.to(torch.float64))
            return y.to(torch.complex128 if x.dtype == torch.float64 else torch.complex64)

    class InverseRealSHTStub(RealSHTStub):
        def forward(self, a):
            y = self.s.inverse(a.to(torch.complex128))
            return y.to(torch.float64 if a.dtype == torch.complex128 else torch.float32)

    cwd = os.getcwd()
    os.chdir(ref_harness.REF)
    da = importlib.import_module("da_4dvar")
    metrics = importlib.import_module("utils.metrics")
    os.chdir(cwd)
    da.RealSHT, da.InverseRealSHT = RealSHTStub, InverseRealSHTStub
    da.Client = lambda *a, **k: None
    lbfgs_orig = torch.optim.LBFGS
    da.optim.LBFGS = _RecordingLBFGS  # da.optim is torch.optim: restored below
    coeff_dir = os.path.join(ref_harness.REF, "dataset", "bq_info_lr")
    # 3e-4 of the 721x1440 columns observed (~300, as the 1 % of a 128x256 grid): at 1 % the B-transformed problem is
    # so stiff that the first line search ends at t ~ 7e-9 with J unchanged in fp32 and L-BFGS stops (tolerance_change)
    prob = make_problem(nch=69, Hs=721, Ws=1440, T=1, seed=1414, obs_frac=3e-4)
    ws = {"w1": uniform_sym(1401, (69, 128, 256), 0.5), "w2": 0.3 * smooth_field(1402, (69, 128, 256), sigma=3.0)}
    old_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *args, **kw: self
    idx = sample_idx(69 * 721 * 1440, 8192, 1414)
    gidx = sample_idx(69 * 128 * 256, 8192, 1415)
    st = lambda v, tag: v.astype(np.float32) if tag == "f32" else v  # the float32 run's values are float32
    try:
        res = {}
        for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
            torch.set_default_dtype(dt)
            a = object.__new__(da.cyclic_4dvar)
            a.device, a.hpad, a.nchannel, a.nlev, a.nlat, a.nlon = "cpu", 112, 69, 13, 721, 1440
            a.da_win, a.q_type, a.scale_factor, a.obs_coeff, a.obs_type, a.Nit = 1, -1, 1.0, 1.0, "synthetic", G14_NIT
            a.use_eval, a.current_time = False, "G14"
            a.metric = metrics.Metrics()
            a.metrics_list = {"bg_wrmse": [], "bg_bias": [], "ana_wrmse": [], "ana_bias": []}
            a.b_matrix = a.init_b_matrix(coeff_dir)
            if dt == torch.float64:  # init_b_matrix's .float() kept out of the float64 run
                a.b_matrix = {k: torch.from_numpy(np.load(os.path.join(coeff_dir, k + ".npy"))).double() for k in a.b_matrix}
                a.b_matrix["len_scale"] = a.b_matrix["len_scale"] * a.scale_factor
            a.q_matrix = a.init_q_matrix(coeff_dir)
            a.model_mean, a.model_std, a.model_mean_gpu, a.model_std_gpu = a.get_model_mean_std()
            a.obs_interp = da.obs_interpolater(13, 40)
            a.data_reader = da.data_reader("synthetic", 0.005, a.model_std, 1, None, None, a.obs_interp, modify_tp=2)
            with contextlib.redirect_stdout(io.StringIO()):
                a.static_info = a.get_static_info()
            R = a.static_info["R"]
            r_ch = R[0, :, 0, 0].double().numpy()
            assert torch.equal(R, R[:, :, :1, :1].expand_as(R)), "R is spatially constant"
            xb = torch.from_numpy(prob["xb"]).to(dt)
            t0 = time.time()
            for wk in ("w1", "w2"):
                w = torch.from_numpy(ws[wk]).to(dt)
                with torch.no_grad():
                    inc = a.transform(w, 0.0)
                    x = a.transform(w, xb)
                fi = inc.reshape(-1).double().numpy()
                fx = x.reshape(-1).double().numpy()
                res[f"{tag}_{wk}_inc"] = st(fi[idx], tag)
                res[f"{tag}_{wk}_inc_sumsq"] = float((fi * fi).sum())
                res[f"{tag}_{wk}_inc_sum"] = float(fi.sum())
                if tag == "f32":
                    res[f"{tag}_{wk}_x"] = st(fx[idx], tag)
            print(f"G14 {tag}: genuine transform x2 at 721x1440 ({time.time() - t0:.1f}s)", flush=True)
            # one genuine loss + backward at w1 (one_step_DA's own closure, T = 1)
            g = {k: torch.from_numpy(prob[k]).to(dt) for k in ("gt", "yo", "H")}
            _RecordingLBFGS.fixed, _RecordingLBFGS.log = torch.from_numpy(ws["w1"]).to(dt), []
            with contextlib.redirect_stdout(io.StringIO()):
                a.one_step_DA(g["gt"], xb, g["yo"], g["H"], R, "sc4dvar")
            J, grad = _RecordingLBFGS.log[0]
            gg = grad.reshape(-1).double().numpy()
            res[f"{tag}_J"], res[f"{tag}_grad"] = J, st(gg[gidx], tag)
            res[f"{tag}_grad_sumsq"] = float((gg * gg).sum())
            print(f"G14 {tag}: genuine sc4dvar loss at w1 J {J:.10e} |g| {np.sqrt((gg * gg).sum()):.6e}", flush=True)
            if tag == "f32":
                # the genuine Nit = G14_NIT passes (LBFGS history 10, max_iter 5, strong Wolfe) from w = 0
                _RecordingLBFGS.fixed, _RecordingLBFGS.log = None, []
                with contextlib.redirect_stdout(io.StringIO()), LineSearchRecorder() as ls:
                    xhat = a.one_step_DA(g["gt"], xb, g["yo"], g["H"], R, "sc4dvar")
                fx = xhat.detach().reshape(-1).double().numpy()
                xbf = prob["xb"].reshape(-1).astype(np.float64)
                wf = _RecordingLBFGS.w.double()
                jo_f = 0.5 * float(((g["H"][0].double() * (xhat.detach().double() - g["yo"][0].double()) ** 2)
                                    / R[0].double()).sum())
                res["J_final"] = (0.5 * float((wf * wf).sum()), jo_f)
                res.update(lbfgs_J=np.array([v for v, _ in _RecordingLBFGS.log]),
                           ls_t=np.array([t for t, _ in ls.steps]), ls_evals=np.array([n for _, n in ls.steps]),
                           xa_inc=(fx - xbf)[idx].astype(np.float32), xa_dsumsq=float(((fx - xbf) ** 2).sum()))
                print(f"G14 f32: genuine Nit={G14_NIT} passes: evals {len(_RecordingLBFGS.log)}, J {res['lbfgs_J'][0]:.6e} -> "
                      f"final (J_b, J_o) {res['J_final']}, line searches {ls.steps}", flush=True)
            res[f"{tag}_R"] = r_ch
            # the restatement on the same inputs
            torch.set_default_dtype(torch.float32)
            p64 = dict(prob, R=R.double().numpy())
            ref = Sc4dvarRef(load_bq(coeff_dir), p64, const_dtype=dt)
            for wk in ("w1", "w2"):
                w = torch.from_numpy(ws[wk]).double()
                inc = ref.state(w) - ref.xb
                e = rel(inc.reshape(-1).numpy()[idx], res[f"{tag}_{wk}_inc"])
                print(f"G14 {tag} {wk}: restatement vs reference transform increment rel {e:.2e}", flush=True)
                assert e < (1e-11 if tag == "f64" else 1e-5), e
            wr = torch.from_numpy(ws["w1"]).double().requires_grad_(True)
            lv = ref.loss(wr)
            lv.backward()
            ej = abs(float(lv) - res[f"{tag}_J"]) / abs(res[f"{tag}_J"])
            eg = rel(wr.grad.reshape(-1).numpy()[gidx], res[f"{tag}_grad"])
            print(f"G14 {tag}: restatement vs reference loss J rel {ej:.2e} grad rel {eg:.2e}", flush=True)
            assert ej < (1e-11 if tag == "f64" else 1e-5) and eg < (1e-10 if tag == "f64" else 1e-4), (ej, eg)
    finally:
        torch.Tensor.cuda = old_cuda
        torch.optim.LBFGS = lbfgs_orig
        torch.set_default_dtype(torch.float32)
    np.savez(os.path.join(GOLD, "g14_sc4dvar_reference.npz"), idx=idx, gidx=gidx, seed=1414, obs_frac=3e-4, nit=G14_NIT,
             **res)


def g16(tr):
    """G16 (BASELINE config 4 at full size): the reference's networks_old.LGUnet_all decoder and the flow stand-in in
    the restated 4D-Var closure with T = 6 (five integrate steps, da_4dvar.py:1183-1208, :666-681),
    torch.optim.LBFGS(history 10, max_iter 10, strong Wolfe), Nit = G16_NIT outer passes at 128x256 (r05: 10, the
    bench's full budget; r04: 3), seed 20250620 (the bench's config-4 rank-0 analysis): J per pass, every line search's
    (t, evals), sampled xa. Parameters frozen as in G10/G13 (the unused weight gradients only cost time)."""
    m, _ = build_ref(tr, C.DECODER)
    fm, _ = build_ref(tr, {k: v for k, v in C.FLOW.items() if k != "arch"})
    for v in list(m.parameters()) + list(fm.parameters()):
        v.requires_grad_(False)
    prob = make_problem(nch=69, Hs=128, Ws=256, T=6, seed=20250620)
    rp = RefProblem(prob, m, C.DECODER["img_size"], fm)
    t0 = time.time()
    with LineSearchRecorder() as ls:
        xa, z, js, nev, nit = one_step_da_ref(rp, G16_NIT, (32, 128, 256),
                                              log=lambda k, j: print(f"G16 pass {k}: J_b {j[0]:.6e} J_o {j[1]:.6e} "
                                                                     f"({time.time() - t0:.0f}s)", flush=True))
    xa = xa.numpy().astype(np.float32)
    idx = sample_idx(xa.size, 8192, 1616)
    flat = xa.reshape(-1).astype(np.float64)
    print(f"G16 config-4 trajectory: {time.time() - t0:.0f}s, evals {nev}, iters {nit}, J {js}")
    np.savez(os.path.join(GOLD, "g16_config4_trajectory.npz"), J=np.array(js, np.float64), n_eval=nev, n_iter=nit,
             nit=G16_NIT, ls_t=np.array([x[0] for x in ls.steps]), ls_evals=np.array([x[1] for x in ls.steps]),
             idx_xa=idx, xa_sample=xa.reshape(-1)[idx], xa_sum=flat.sum(),
             dxa_sumsq=((flat - prob["xb"].reshape(-1).astype(np.float64)) ** 2).sum())


G16_NIT = int(os.environ.get("G16_NIT", "10"))


def g11():
    """G11: the reference's networks.LGUnet_all.LGUnet_all_1 at the full 0.25-degree
    configuration (training_options.yaml:64-119: 69ch 721x1440, 16,200-token global LG window), synthetic weights,
    one forward on a smooth input: sampled outputs + sums."""
    import importlib

    from oracle.lgunet1_ref import synth_params as synth1

    L1 = importlib.import_module("networks.LGUnet_all")
    cfg = C.FCST
    torch.manual_seed(0)
    t0 = time.time()
    m = L1.LGUnet_all_1(**ref_cfg_l1(cfg))
    p = synth1(cfg)
    m.load_state_dict(p, strict=True)
    m.eval()
    del p
    x = torch.from_numpy(smooth_field(1101, (1, C.in_channels(cfg)) + tuple(cfg["img_size"])))
    with torch.no_grad():
        y = m(x)
    y = y.numpy()
    idx = sample_idx(y.size, 16384, 1111)
    flat = y.reshape(-1).astype(np.float64)
    print(f"G11 LGUnet_all_1 0.25deg forward {tuple(y.shape)}: {time.time() - t0:.0f}s, sumsq {(flat * flat).sum():.6e}")
    np.savez(os.path.join(GOLD, "g11_fcst_025deg.npz"), idx=idx, out_sample=y.reshape(-1)[idx], out_sum=flat.sum(),
             out_sumsq=(flat * flat).sum(), out_abssum=np.abs(flat).sum(), shape=np.array(y.shape))


def g12(tr):
    """G12 (BASELINE config 4's 6-step window): the reference's networks_old.LGUnet_all
    tiny decoder and tiny flow model, T = 6 (five integrate steps in the loss, da_4dvar.py:1190-1194): one closure
    (J_b, J_o, dJ/dz) at a non-zero latent, and one outer pass of torch.optim.LBFGS (Nit = 1) with every line
    search's (t, evals) recorded."""
    cfg, fcfg = C.TINY, C.TINY_FLOW
    m, p = build_ref(tr, cfg)
    fm, fp = build_ref(tr, fcfg)
    prob = make_problem(nch=4, Hs=32, Ws=64, T=6, seed=779, obs_frac=0.1)
    rp = RefProblem(prob, m, cfg["img_size"], fm)
    z = torch.from_numpy(0.3 * smooth_field(1201, (1, 4, 32, 64), sigma=2.0)).requires_grad_(True)
    r, o = rp.loss_terms(z)
    (r + o).backward()
    ro = oracle_problem(prob, p, cfg, fp, fcfg)
    z2 = z.detach().clone().requires_grad_(True)
    r2, o2 = ro.loss_terms(z2)
    (r2 + o2).backward()
    print(f"G12 tiny 4D-Var T=6: J_b {float(r):.6e} J_o {float(o):.6e}; oracle rel J_o "
          f"{abs(float(o2) - float(o)) / abs(float(o)):.2e} grad {rel(z2.grad, z.grad):.2e}")
    with LineSearchRecorder() as ls:
        xa, zf, js, nev, nit = one_step_da_ref(rp, 1, (4, 32, 64))
    print(f"G12 L-BFGS Nit=1: J {js} evals {nev} iters {nit}")
    np.savez(os.path.join(GOLD, "g12_tiny_4dvar_t6.npz"), z=z.detach().numpy(), J_b=float(r), J_o=float(o),
             grad=z.grad.numpy(), J=np.array(js, np.float64), n_eval=nev, n_iter=nit, xa=xa.numpy(),
             ls_t=np.array([x[0] for x in ls.steps]), ls_evals=np.array([x[1] for x in ls.steps]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="also generate G3 (full decoder, ~1 min)")
    ap.add_argument("--only", default=None)
    ap.add_argument("--g6", action="store_true", help="also generate G6 (genuine one_step_DA at 721x1440, ~5 min)")
    ap.add_argument("--g8", action="store_true", help="also generate G8 (genuine real-obs one_step_DA, ~3 min)")
    ap.add_argument("--g10", action="store_true", help="also generate G10 (config-2 trajectory, Nit 10, ~10 min)")
    ap.add_argument("--g11", action="store_true", help="also generate G11 (0.25-deg LGUnet_all_1 forward, ~3 min)")
    ap.add_argument("--g13", action="store_true", help="also generate G13 (config-3 T=2 trajectory, Nit 10, ~30 min)")
    ap.add_argument("--g15", action="store_true", help="also generate G15 (genuine one_step_DA, config 5, Nit 5, ~25 min)")
    ap.add_argument("--g16", action="store_true", help="also generate G16 (config-4 T=6 trajectory, Nit 10, ~4 h on 8 threads)")
    a = ap.parse_args()
    os.makedirs(GOLD, exist_ok=True)
    torch.set_num_threads(int(os.environ.get("ORACLE_THREADS", "8")))
    cwd = os.getcwd()
    tr, sb = ref_harness.import_reference()
    os.chdir(cwd)
    steps = {"g1": lambda: g1(tr), "g2": lambda: g2(sb), "g4": g4, "g5": lambda: g5(tr), "g5b": lambda: g5b(tr),
             "g7": g7, "g9": g9, "g12": lambda: g12(tr), "g14": lambda: g14(tr)}
    if a.full:
        steps["g3"] = lambda: g3(tr)
    if a.g6:
        steps["g6"] = lambda: g6(tr)
    if a.g8:
        steps["g8"] = lambda: g8(tr)
    if a.g10:
        steps["g10"] = lambda: g10(tr)
    if a.g11:
        steps["g11"] = g11
    if a.g13:
        steps["g13"] = lambda: g13(tr)
    if a.g15:
        steps["g15"] = lambda: g15(tr)
    if a.g16:
        steps["g16"] = lambda: g16(tr)
    for k, f in steps.items():
        if a.only and k not in a.only.split(","):
            continue
        f()


if __name__ == "__main__":
    main()
