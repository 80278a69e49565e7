"""CPU: the oracle restatement (oracle/) against the golden fixtures generated from the real reference
(oracle/make_golden.py imports /root/reference in the survey container). Pins the oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD


def gold(name):
    return np.load(os.path.join(GOLD, name))


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def test_g1_tiny_decoder():
    from oracle.lgunet_ref import lgunet_forward, synth_params
    from vaevar import config as C

    g = gold("g1_tiny_decoder.npz")
    p = synth_params(C.TINY)
    z = torch.from_numpy(g["z"]).requires_grad_(True)
    out = lgunet_forward(p, C.TINY, z)
    (out * torch.from_numpy(g["cot"])).sum().backward()
    assert rel(out.detach(), g["out"]) < 1e-6
    assert rel(z.grad, g["grad"]) < 1e-6


@pytest.mark.parametrize("shift", [0, 2])
def test_g2_swin_block(shift):
    from oracle.lgunet_ref import swin_block, shift_mask, rel_pos_index
    from vaevar.synth import param_value

    g = gold("g2_swin_block.npz")
    pre = f"g2.s{shift}"
    C = 32
    shapes = {"norm1.weight": (C,), "norm1.bias": (C,), "attn.relative_position_bias_table": (49, 2),
              "attn.qkv.weight": (3 * C, C), "attn.qkv.bias": (3 * C,), "attn.proj.weight": (C, C),
              "attn.proj.bias": (C,), "norm2.weight": (C,), "norm2.bias": (C,), "mlp.fc1.weight": (4 * C, C),
              "mlp.fc1.bias": (4 * C,), "mlp.fc2.weight": (C, 4 * C), "mlp.fc2.bias": (C,)}
    p = {f"{pre}.{k}": torch.from_numpy(param_value(f"{pre}.{k}", s)) for k, s in shapes.items()}
    x = torch.from_numpy(g[f"x_s{shift}"]).requires_grad_(True)
    y = swin_block(x, p, pre, 2, 4, shift)
    (y * torch.from_numpy(g[f"cot_s{shift}"])).sum().backward()
    assert rel(y.detach(), g[f"out_s{shift}"]) < 1e-6
    assert rel(x.grad, g[f"grad_s{shift}"]) < 1e-6
    if shift:
        assert np.array_equal(shift_mask(16, 32, 4, 2).numpy(), g["attn_mask_s2"])  # quirk Q1
        assert np.array_equal(rel_pos_index(4).numpy(), g["rel_index"])


def test_g4_nearest_maps():
    """F.interpolate(mode='nearest') index maps (quirk Q3): src = floor(dst * in/out) in fp32."""
    g = gold("g4_nearest_maps.npz")
    for key, (a, b) in (("lat_721_to_128", (721, 128)), ("lat_128_to_721", (128, 721)),
                        ("lon_1440_to_256", (1440, 256)), ("lon_256_to_1440", (256, 1440))):
        scale = np.float32(a) / np.float32(b)
        m = np.minimum(np.floor(np.arange(b, dtype=np.float32) * scale).astype(np.int64), a - 1)
        assert np.array_equal(m, g[key]), key


def test_g4_engine_nearest_maps():
    """The engine's own index maps (vv_nearest_map, used by the misfit kernels) equal the reference's."""
    from vaevar import _lib

    g = gold("g4_nearest_maps.npz")
    for key, (a, b) in (("lat_721_to_128", (721, 128)), ("lat_128_to_721", (128, 721)),
                        ("lon_1440_to_256", (1440, 256)), ("lon_256_to_1440", (256, 1440))):
        assert np.array_equal(np.array(_lib.nearest_map(a, b)), g[key]), key


def _tiny_problem(T):
    from vaevar.problem import make_problem

    return make_problem(nch=4, Hs=32, Ws=64, T=T, seed=777, obs_frac=0.1)


def test_g5b_tiny_4dvar_closure():
    from oracle.da_ref import oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C

    g = gold("g5b_tiny_4dvar.npz")
    ro = oracle_problem(_tiny_problem(2), synth_params(C.TINY), C.TINY, synth_params(C.TINY_FLOW), C.TINY_FLOW)
    z = torch.from_numpy(g["z"]).requires_grad_(True)
    r, o = ro.loss_terms(z)
    (r + o).backward()
    assert abs(float(r) - g["J_b"]) / g["J_b"] < 1e-6
    assert abs(float(o) - g["J_o"]) / g["J_o"] < 1e-6
    assert rel(z.grad, g["grad"]) < 1e-6


def test_g12_tiny_4dvar_t6():
    """G12: the T = 6 window (five integrate steps) — closure and one outer L-BFGS pass of the reference modules."""
    from oracle.da_ref import one_step_da_ref, oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C
    from vaevar.problem import make_problem

    g = gold("g12_tiny_4dvar_t6.npz")
    p = make_problem(nch=4, Hs=32, Ws=64, T=6, seed=779, obs_frac=0.1)
    ro = oracle_problem(p, synth_params(C.TINY), C.TINY, synth_params(C.TINY_FLOW), C.TINY_FLOW)
    z = torch.from_numpy(g["z"]).requires_grad_(True)
    r, o = ro.loss_terms(z)
    (r + o).backward()
    assert abs(float(r) - g["J_b"]) / g["J_b"] < 1e-6 and abs(float(o) - g["J_o"]) / g["J_o"] < 1e-6
    assert rel(z.grad, g["grad"]) < 1e-6
    xa, _, js, nev, nit = one_step_da_ref(ro, 1, (4, 32, 64))
    assert np.allclose(np.array(js), g["J"], rtol=1e-5)
    assert nev == int(g["n_eval"]) and nit == int(g["n_iter"])
    assert rel(xa, g["xa"]) < 1e-5


def test_g10_g11_fixtures_consistent():
    """G10 / G11 are outputs of the reference itself (too long to re-run here); check they are self-consistent."""
    g = gold("g10_config2_trajectory.npz")
    J = g["J"].sum(1)
    assert len(J) == 11 and np.all(np.diff(J) < 0)  # monotone decrease over the 10 outer passes
    assert int(g["n_iter"]) <= 100 and len(g["ls_t"]) == int(g["n_iter"]) and int(g["ls_evals"].sum()) + 10 == int(g["n_eval"])
    f = gold("g11_fcst_025deg.npz")
    assert tuple(f["shape"]) == (1, 138, 721, 1440) and np.isfinite(f["out_sample"]).all()
    assert float(f["out_sumsq"]) > 0 and len(f["idx"]) == len(f["out_sample"])


def test_g13_fixture_consistent_and_oracle_pass0():
    """G13 (config 3, T = 2, the reference modules + torch.optim.LBFGS) is self-consistent, and the oracle
    restatement of the T = 2 closure (decoder + flow through integrate) reproduces its pass-0 J at z = 0."""
    from oracle.da_ref import oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C
    from vaevar.problem import make_problem

    g = gold("g13_config3_trajectory.npz")
    J = g["J"].sum(1)
    assert len(J) == 11 and np.all(np.diff(J) < 0)
    assert int(g["n_iter"]) <= 100 and len(g["ls_t"]) == int(g["n_iter"])
    assert int(g["ls_evals"].sum()) + 10 == int(g["n_eval"])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    prob = make_problem(nch=69, Hs=128, Ws=256, T=2, seed=20250620)
    ro = oracle_problem(prob, synth_params(C.DECODER), C.DECODER, synth_params(C.FLOW), C.FLOW)
    with torch.no_grad():
        jb, jo = ro.loss_terms(torch.zeros(1, 32, 128, 256))
    assert float(jb) == 0.0
    assert abs(float(jo) - float(g["J"][0][1])) < 1e-5 * float(g["J"][0][1]), (float(jo), float(g["J"][0][1]))


def test_g15_g16_fixtures_consistent_and_oracle_pass0():
    """G15 (the genuine one_step_DA, config 5: 721x1440, T = 2, Nit 5) and G16 (config 4: T = 6, Nit 3, the reference
    modules + torch.optim.LBFGS) are self-consistent, and the oracle restatement of the T = 6 closure (decoder + five
    flow steps through integrate) reproduces G16's pass-0 J at z = 0."""
    from oracle.da_ref import oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C
    from vaevar.problem import make_problem

    g15 = gold("g15_config5_trajectory.npz")
    J = g15["J"].sum(1)
    assert len(J) == 6 and np.all(np.diff(J) < 0) and len(g15["ls_t"]) <= 50
    g = gold("g16_config4_trajectory.npz")
    J = g["J"].sum(1)
    assert len(J) == int(g["nit"]) + 1 and np.all(np.diff(J) < 0)
    assert len(g["ls_t"]) == int(g["n_iter"]) and int(g["ls_evals"].sum()) + int(g["nit"]) == int(g["n_eval"])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    prob = make_problem(nch=69, Hs=128, Ws=256, T=6, seed=20250620)
    ro = oracle_problem(prob, synth_params(C.DECODER), C.DECODER, synth_params(C.FLOW), C.FLOW)
    with torch.no_grad():
        jb, jo = ro.loss_terms(torch.zeros(1, 32, 128, 256))
    assert float(jb) == 0.0
    assert abs(float(jo) - float(g["J"][0][1])) < 1e-5 * float(g["J"][0][1]), (float(jo), float(g["J"][0][1]))


def test_g5_tiny_lbfgs_trajectory():
    from oracle.da_ref import one_step_da_ref, oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C

    g = gold("g5_tiny_lbfgs.npz")
    ro = oracle_problem(_tiny_problem(1), synth_params(C.TINY), C.TINY)
    xa, z, js, nev, nit = one_step_da_ref(ro, 2, (4, 32, 64))
    assert np.allclose(np.array(js), g["J"], rtol=1e-5)
    assert nev == int(g["n_eval"]) and nit == int(g["n_iter"])
    assert rel(xa, g["xa"]) < 1e-5


def test_g3_full_decoder_oracle():
    """Full parameters0_old decoder at 128x256 (216M params): oracle vs the reference's sampled outputs."""
    from oracle.lgunet_ref import lgunet_forward, synth_params
    from vaevar import config as C
    from vaevar.synth import smooth_field, uniform_sym

    g = gold("g3_full_decoder.npz")
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    p = synth_params(C.DECODER)
    z = torch.from_numpy(0.5 * smooth_field(401, (1, 32, 128, 256))).requires_grad_(True)
    cot = torch.from_numpy(uniform_sym(402, (1, 69, 128, 256), 1.0))
    out = lgunet_forward(p, C.DECODER, z)
    (out * cot).sum().backward()
    o = out.detach().numpy().reshape(-1)
    gr = z.grad.numpy().reshape(-1)
    assert rel(o[g["idx_out"]], g["out_sample"]) < 1e-6
    assert rel(gr[g["idx_grad"]], g["grad_sample"]) < 1e-6


def test_g7_tiny_lgunet1_oracle():
    """networks.LGUnet_all_1 restatement (RoPE, -inf mask, global LG window, 3 levels, patch (3,2)/s2)."""
    from oracle.lgunet1_ref import lgunet1_forward, synth_params
    from vaevar import config as C
    from vaevar.synth import smooth_field

    g = gold("g7_tiny_lgunet1.npz")
    cfg = C.TINY_FCST
    x = torch.from_numpy(smooth_field(701, (1, C.in_channels(cfg)) + tuple(cfg["img_size"])))
    with torch.no_grad():
        y = lgunet1_forward(synth_params(cfg), cfg, x)
    assert rel(y, g["out"]) < 1e-6


def _g8():
    path = os.path.join(GOLD, "g8_real_obs.npz")
    if not os.path.exists(path):
        pytest.skip("G8 fixture not generated (oracle/make_golden.py --g8)")
    return np.load(path)


def test_g8_obs_interpolater_matrices():
    """obs_interpolater(13, 40) (da_4dvar.py:62-94): the oracle's and the product host's restatements equal the
    genuine reference's interp / interp_inv bit for bit."""
    from oracle.da_ref import obs_interp_ref
    from vaevar.problem import ObsInterpolater

    g = _g8()
    a, b = obs_interp_ref(13, 40)
    o = ObsInterpolater(13, 40)
    assert np.array_equal(a.numpy(), g["interp"]) and np.array_equal(b.numpy(), g["interp_inv"])
    assert np.array_equal(o.interp, g["interp"]) and np.array_equal(o.interp_inv, g["interp_inv"])


def test_g8_r_matrix_from_gt():
    """get_R_matrix_from_gt (da_4dvar.py:729-756) on the G8 small R: oracle x_aug_ref (F.linear, as the reference)
    bit-exact; the host generator's einsum within fp32 rounding."""
    from oracle.da_ref import x_aug_ref
    from vaevar.problem import make_problem, obs_augment_np
    from vaevar.synth import smooth_field

    g = _g8()
    rs = make_problem(nch=69, Hs=4, Ws=8, T=2, seed=811)["R"]
    rs = (rs * (1.0 + 0.5 * smooth_field(812, rs.shape, sigma=1.0) ** 2)).astype(np.float32)
    ra = x_aug_ref(torch.from_numpy(rs), torch.from_numpy(g["interp"])).numpy()
    assert np.array_equal(ra, g["r_aug"])
    rn = obs_augment_np(g["interp"], rs)
    assert np.abs(rn - g["r_aug"]).max() <= 1e-6 * np.abs(g["r_aug"]).max()


@pytest.mark.parametrize("tag,Hs,Ws,seed", [("s", 128, 256, 901), ("l", 721, 1440, 902)])
def test_g9_metrics_oracle(tag, Hs, Ws, seed):
    """WRMSE / Bias restatement (oracle/da_ref.py) vs the genuine Metrics (G9)."""
    from oracle.da_ref import bias_ref, wrmse_ref
    from vaevar import config as C
    from vaevar.problem import make_problem

    g = gold("g9_metrics.npz")
    p = make_problem(nch=69, Hs=Hs, Ws=Ws, T=1, seed=seed)
    mean = torch.tensor(C.MODEL_MEAN, dtype=torch.float32).reshape(-1, 1, 1)
    std = torch.tensor(C.MODEL_STD, dtype=torch.float32).reshape(-1, 1, 1)
    xn = ((torch.from_numpy(p["xb"]) - mean) / std).unsqueeze(0)
    gn = ((torch.from_numpy(p["gt"][0]) - mean) / std).unsqueeze(0)
    assert np.array_equal(np.asarray(C.MODEL_STD, np.float64), g["model_std"])
    w = wrmse_ref(xn, gn, g["model_std"]).numpy()
    b = bias_ref(xn, gn, g["model_std"]).numpy()
    assert rel(w, g["wrmse_" + tag]) < 1e-6 and rel(b, g["bias_" + tag]) < 1e-6
