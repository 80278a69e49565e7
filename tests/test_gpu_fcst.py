"""Forecast network networks.LGUnet_all.LGUnet_all_1 and integrate() (a12 / f1) on the HIP
engine, against the G7 golden (real reference) and the oracle restatement (oracle/lgunet1_ref.py, itself pinned
bit-exact to the reference by G7). Forward only, as the reference uses it (da_4dvar.py:652, 1329).

Tolerance: out rel <= 1e-5 (tiny, G7) / 1e-4 (mid size), rel = max|a-b| / max|b|."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD, check

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def _model(cfg):
    from vaevar.engine import LGUnet

    return LGUnet(cfg, 1, 1).load_synthetic()


def test_fcst_tiny_g7():
    from vaevar import config as C
    from vaevar.synth import smooth_field

    cfg = C.TINY_FCST
    g = np.load(os.path.join(GOLD, "g7_tiny_lgunet1.npz"))
    x = torch.from_numpy(smooth_field(701, (1, C.in_channels(cfg)) + tuple(cfg["img_size"]))).cuda()
    out = _model(cfg).forward_raw(x)
    e = rel(out.cpu(), g["out"])
    print(f"G7 tiny LGUnet_all_1: out rel {e:.2e}")
    check("G7 out", e, 1e-5)


def test_fcst_025deg_g11():
    """G11: the full 0.25-degree forecast network (training_options.yaml:64-119: 69ch 721x1440, 427M parameters,
    LG layer 0 one 16,200-token global window) against the reference's own LGUnet_all_1 forward on CPU: 16,384
    sampled outputs and the sums over all 143M outputs."""
    path = os.path.join(GOLD, "g11_fcst_025deg.npz")
    from vaevar import config as C
    from vaevar.synth import smooth_field

    g = np.load(path)
    cfg = C.FCST
    x = torch.from_numpy(smooth_field(1101, (1, C.in_channels(cfg)) + tuple(cfg["img_size"]))).cuda()
    out = _model(cfg).forward_raw(x)
    assert tuple(out.shape) == tuple(g["shape"])
    o = out.cpu().numpy().reshape(-1).astype(np.float64)
    e = rel(o[g["idx"]], g["out_sample"])
    e_ss = abs((o * o).sum() - float(g["out_sumsq"])) / float(g["out_sumsq"])
    e_as = abs(np.abs(o).sum() - float(g["out_abssum"])) / float(g["out_abssum"])
    print(f"G11 LGUnet_all_1 0.25deg: sampled out rel {e:.2e}, sumsq rel {e_ss:.1e}, abssum rel {e_as:.1e}")
    check("G11 sampled out", e, 1e-5)
    check("G11 sumsq", e_ss, 1e-8)
    check("G11 abssum", e_as, 2e-9)


@pytest.mark.parametrize("name", ["MID_FCST", "BIG_FCST"])
def test_fcst_mid_vs_oracle(name):
    """Real FCST widths/heads/window on a 97x192 image: head_dim 32/32/64/192, [6,12] windows with the -inf
    row mask, 288-token global LG window (streaming kernel), patch (3,2)/stride 2 conv and overlapping
    ConvTranspose; on 193x384 the 1152-token global window runs as split GEMMs + row softmax."""
    from oracle.lgunet1_ref import lgunet1_forward, synth_params
    from vaevar import config as C
    from vaevar.synth import smooth_field

    cfg = getattr(C, name)
    x = smooth_field(702, (1, C.in_channels(cfg)) + tuple(cfg["img_size"]))
    out = _model(cfg).forward_raw(torch.from_numpy(x).cuda())
    torch.set_num_threads(16)
    with torch.no_grad():
        ref = lgunet1_forward(synth_params(cfg), cfg, torch.from_numpy(x))
    e = rel(out.cpu(), ref)
    print(f"{name} LGUnet_all_1 {cfg['img_size']}: out rel {e:.2e}")
    check(f"{name} out vs oracle", e, 1e-5)


def test_fcst_window_attention_mfma_vs_valu():
    """The exact-f32 MFMA window-attention kernel (win_mfma=1, default) against the VALU kernel (win_mfma=0) on
    the MID_FCST shapes (head_dim 32/64, [6,12] windows with and without the -inf row mask): both compute fp32
    products with fp32 sums, so the forecasts agree to rounding (rel <= 1e-5)."""
    from vaevar import config as C
    from vaevar.synth import smooth_field

    cfg = C.MID_FCST
    x = torch.from_numpy(smooth_field(704, (1, C.in_channels(cfg)) + tuple(cfg["img_size"]))).cuda()
    m = _model(cfg)
    try:
        m.ctx.set_tuning("win_mfma", 0)
        a = m.forward_raw(x).clone()
        m.ctx.set_tuning("win_mfma", 1)
        b = m.forward_raw(x).clone()
    finally:
        m.ctx.set_tuning("win_mfma", 1)
    e = rel(b.cpu(), a.cpu())
    print(f"window attention MFMA vs VALU: forecast rel {e:.2e}")
    assert torch.isfinite(b).all()
    check("forecast window attention MFMA vs VALU", e, 1e-5)


def test_fcst_backward_refused():
    from vaevar import config as C
    from vaevar._lib import VVError

    m = _model(C.TINY_FCST)
    x = torch.zeros(1, 5, 49, 96, device="cuda")
    m.forward_raw(x)
    with pytest.raises(VVError):
        m.backward_raw(torch.zeros(1, 10, 49, 96, device="cuda"), torch.empty_like(x))


@pytest.mark.parametrize("grid", [(49, 96), (61, 120)])
def test_integrate_forecast(grid):
    """integrate(x, forecast_model, 1): (x-mean)/std -> model -> [:C] -> *std+mean; a state grid other than
    the model grid goes through the nearest maps both ways (interpolation=True, quirk Q3)."""
    from oracle.lgunet1_ref import lgunet1_forward, synth_params
    from vaevar import config as C
    from vaevar.engine import integrate
    from vaevar.synth import smooth_field

    cfg = dict(C.TINY_FCST, outchans_list=[4, 6])   # in 5 channels -> out 10 (mean halves first: 2+3)
    Cs = C.in_channels(cfg)
    Hs, Ws = grid
    mean = torch.linspace(-1.0, 2.0, Cs)
    std = torch.linspace(0.5, 3.0, Cs)
    x = torch.from_numpy(smooth_field(703, (Cs, Hs, Ws))) * std.view(-1, 1, 1) + mean.view(-1, 1, 1)
    m = _model(cfg)
    out = integrate(m, x.cuda(), mean, std, steps=1)
    z = ((x - mean.view(-1, 1, 1)) / std.view(-1, 1, 1)).unsqueeze(0)
    H, W = cfg["img_size"]
    if (Hs, Ws) != (H, W):
        z = torch.nn.functional.interpolate(z, (H, W))
    with torch.no_grad():
        y = lgunet1_forward(synth_params(cfg), cfg, z)[:, :Cs]
    if (Hs, Ws) != (H, W):
        y = torch.nn.functional.interpolate(y, (Hs, Ws))
    ref = y.reshape(Cs, Hs, Ws) * std.view(-1, 1, 1) + mean.view(-1, 1, 1)
    e = rel(out.cpu(), ref)
    print(f"integrate {grid}: rel {e:.2e}")
    check(f"integrate {grid}", e, 5e-6)


def _attn_ref_fp64(qkv, heads):
    """softmax(q k^T) v per head in fp64 on the GPU (the global-window SD_attn without mask, Attention.py:599-664)."""
    N, C3 = qkv.shape
    C = C3 // 3
    hd = C // heads
    q, k, v = qkv.double().split(C, dim=1)
    out = torch.empty(N, C, dtype=torch.float64, device=qkv.device)
    for h in range(heads):
        sl = slice(h * hd, (h + 1) * hd)
        s = q[:, sl] @ k[:, sl].t()
        out[:, sl] = torch.softmax(s, dim=1) @ v[:, sl]
    return out


@pytest.mark.parametrize("N,C,heads,logit", [(300, 384, 2, 1.0), (1000, 1152, 6, 3.0), (777, 256, 4, 8.0),
                                             (2049, 384, 3, 2.0), (16200, 1152, 6, 1.0)])
def test_attention_global_vs_fp64(N, C, heads, logit):
    """vv_attention_global (the flash MFMA kernel of the 0.25-degree global LG window: fp16x3 products, fp32 online
    softmax) against fp64 softmax attention: N not a multiple of the 32-key stage or the 128-query block, head_dim
    64 / 96 / 192, logits up to ~|logit| x 20 (online-softmax rescales in most stages, one query spiked 6x), token
    norms of q and k spanning e^+-1 and of v e^+-4, and the full 16,200-token / 6-head / hd-192 shape. Error <=
    max(1e-5, 2x torch fp32's) of max |out|."""
    from vaevar.engine import Context

    ctx = Context.get(0)
    g = torch.Generator(device="cuda").manual_seed(N + C + heads)
    qkv = torch.randn(N, 3 * C, device="cuda", generator=g)
    qkv[:, :C] *= logit / (C // heads) ** 0.25
    qkv[:, C:2 * C] /= (C // heads) ** 0.25
    qkv[:, :2 * C] *= torch.exp(torch.empty(N, 1, device="cuda").uniform_(-1, 1, generator=g))
    qkv[:, 2 * C:] *= torch.exp(torch.empty(N, 1, device="cuda").uniform_(-4, 4, generator=g))
    qkv[N // 3, :C] *= 6.0  # one query with a logit spike
    out = ctx.attention_global(qkv, heads)
    ref = _attn_ref_fp64(qkv, heads)
    e = float((out.double() - ref).abs().max() / ref.abs().max())
    # the same attention in torch fp32 (what the reference computes) against fp64, for scale
    q, k, v = qkv.split(C, dim=1)
    hd = C // heads
    e32 = 0.0
    for h in range(heads):
        sl = slice(h * hd, (h + 1) * hd)
        o32 = torch.softmax(q[:, sl] @ k[:, sl].t(), dim=1) @ v[:, sl]
        e32 = max(e32, float((o32.double() - ref[:, sl]).abs().max() / ref.abs().max()))
    print(f"global attention N {N} C {C} heads {heads}: rel {e:.2e} (torch fp32: {e32:.2e})")
    assert torch.isfinite(out).all()
    check(f"global attention N {N} C {C} vs fp64 (bound max(1e-5, 2x torch fp32))", e, max(1e-5, 2 * e32))


def test_attention_global_rejects():
    from vaevar._lib import VVError
    from vaevar.engine import Context

    ctx = Context.get(0)
    qkv = torch.zeros(64, 3 * 80, device="cuda")
    with pytest.raises(VVError, match="1001"):
        ctx.attention_global(qkv, 5)  # head_dim 16
