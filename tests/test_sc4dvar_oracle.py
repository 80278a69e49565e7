"""CPU: the sc4dvar oracle (oracle/sc4dvar_ref.py). torch_harmonics is absent and unpinned by the reference, so the
SHT restatement is pinned by its defining properties instead: the Clenshaw-Curtis rule integrates polynomials of
degree < nlat exactly, the Legendre table equals scipy's spherical harmonics (orthonormal, Condon-Shortley phase),
and the transform pair reproduces band-limited fields. The B-matrix transform is checked for linearity and its
autograd gradient against finite differences; the B statistics are the reference's own data files."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD

BQ = os.path.join(GOLD, "bq_info_lr.npz")


def test_clenshaw_curtis_exact():
    from oracle.sc4dvar_ref import clenshaw_curtis

    x, w = clenshaw_curtis(128)
    assert abs(x[0] - 1.0) < 1e-15 and abs(x[-1] + 1.0) < 1e-15  # north pole first
    for p in range(0, 128):
        exact = (1 - (-1) ** (p + 1)) / (p + 1)
        assert abs((w * x ** p).sum() - exact) < 1e-13, p


def test_legpoly_matches_scipy():
    from scipy.special import sph_harm_y

    from oracle.sc4dvar_ref import clenshaw_curtis, legpoly

    x, _ = clenshaw_curtis(128)
    P = legpoly(129, 128, x)
    th = np.arccos(np.clip(x, -1, 1))
    for m in (0, 1, 2, 3, 8, 31, 64, 100, 127):
        for l in sorted({m, m + 1, m + 2, (m + 127) // 2, 127}):
            if m <= l <= 127:
                y = sph_harm_y(l, m, th, 0.0).real
                assert np.abs(P[m, l] - y).max() < 1e-11, (m, l)
    assert np.all(P[128] == 0)  # the Nyquist order has no function below lmax


def test_sht_band_limited_roundtrip():
    from oracle.sc4dvar_ref import SHT

    s = SHT()
    g = torch.Generator().manual_seed(3)
    L = 48
    a = torch.zeros(128, 129, dtype=torch.complex128)
    for l in range(L):
        re = torch.randn(l + 1, generator=g, dtype=torch.float64)
        im = torch.randn(l + 1, generator=g, dtype=torch.float64)
        im[0] = 0.0
        a[l, :l + 1] = torch.complex(re, im)
    f = s.inverse(a)
    b = s.forward(f)
    # coefficients with l + L < nlat are reproduced exactly (the quadrature is exact there)
    assert float((b[:128 - L] - a[:128 - L]).abs().max()) < 1e-12
    # and the field itself: inverse(forward(f)) == f once the aliased high degrees are dropped
    f2 = s.inverse(torch.where(torch.arange(128)[:, None] < 128 - L, b, torch.zeros_like(b)))
    assert float((f2 - f).abs().max() / f.abs().max()) < 1e-12


def _problem(Hs=128, Ws=256, T=1, seed=11):
    from vaevar.problem import make_problem

    return make_problem(nch=69, Hs=Hs, Ws=Ws, T=T, seed=seed)


def test_transform_linear_and_gradient():
    from oracle.sc4dvar_ref import Sc4dvarRef, load_bq

    ref = Sc4dvarRef(load_bq(npz=BQ), _problem())
    g = torch.Generator().manual_seed(5)
    u = torch.randn(69, 128, 256, generator=g, dtype=torch.float64) * 0.1
    v = torch.randn(69, 128, 256, generator=g, dtype=torch.float64) * 0.1
    a = ref.transform(u + 2.0 * v)
    b = ref.transform(u) + 2.0 * ref.transform(v)
    assert float((a - b).abs().max() / b.abs().max()) < 1e-12
    # autograd gradient vs a central finite difference along a random direction
    uu = u.clone().requires_grad_(True)
    ref.loss(uu).backward()
    eps = 1e-4
    fd = (ref.loss(u + eps * v) - ref.loss(u - eps * v)) / (2 * eps)
    gd = float((uu.grad * v).sum())
    assert abs(gd - float(fd)) / abs(gd) < 1e-6


def test_bq_fixture_is_the_reference_data():
    """tests/golden/bq_info_lr.npz holds the reference's dataset/bq_info_lr/*.npy (oracle/make_bq_fixture.py)."""
    src = "/root/reference/dataset/bq_info_lr"
    if not os.path.isdir(src):
        pytest.skip("reference tree not present")
    with np.load(BQ) as z:
        for k in ("len_scale", "reg_coeff", "std_sur", "vert_eig_value", "vert_eig_vec"):
            assert np.array_equal(z[k], np.load(os.path.join(src, k + ".npy")))


def g14_inputs():
    """The inputs of G14 (oracle/make_golden.py g14), regenerated from the counter-hash RNG: the 721x1440 problem
    (T = 1, 3e-4 of the columns observed) with the genuine get_static_info R per channel, and the two w fields."""
    from vaevar.problem import make_problem
    from vaevar.synth import smooth_field, uniform_sym

    g = np.load(os.path.join(GOLD, "g14_sc4dvar_reference.npz"))
    p = make_problem(nch=69, Hs=721, Ws=1440, T=1, seed=int(g["seed"]), obs_frac=float(g["obs_frac"]))
    ws = {"w1": uniform_sym(1401, (69, 128, 256), 0.5), "w2": 0.3 * smooth_field(1402, (69, 128, 256), sigma=3.0)}
    return g, p, ws


@pytest.mark.parametrize("run", ["f64", "f32"])
def test_g14_oracle_vs_reference_code(run):
    """G14 pins the restatement to the reference's OWN sc4dvar code (get_static_info, transform, the one_step_DA
    loss + backward, da_4dvar.py:608-638, 878-931, 1064-1107) with the oracle's SHT injected as the torch_harmonics
    stub: to float64 rounding against the reference run with float64 as its default dtype, to float32 rounding
    against the reference as it runs (float32). The SHT itself stays unpinned (torch_harmonics absent)."""
    from oracle.sc4dvar_ref import Sc4dvarRef, load_bq

    g, p, ws = g14_inputs()
    R = np.broadcast_to(g[f"{run}_R"][None, :, None, None], p["R"].shape)
    ref = Sc4dvarRef(load_bq(npz=BQ), dict(p, R=R), const_dtype=torch.float64 if run == "f64" else torch.float32)
    tol_x, tol_j, tol_g = (1e-11, 1e-11, 1e-10) if run == "f64" else (1e-5, 1e-5, 1e-4)
    for wk in ("w1", "w2"):
        inc = (ref.state(torch.from_numpy(ws[wk]).double()) - ref.xb).reshape(-1).numpy()
        e = float(np.abs(inc[g["idx"]] - g[f"{run}_{wk}_inc"]).max() / np.abs(g[f"{run}_{wk}_inc"]).max())
        e_s = abs(float((inc * inc).sum()) - float(g[f"{run}_{wk}_inc_sumsq"])) / float(g[f"{run}_{wk}_inc_sumsq"])
        print(f"G14 {run} {wk}: transform increment rel {e:.2e}, sum of squares rel {e_s:.2e}")
        assert e < tol_x and e_s < tol_x
    w = torch.from_numpy(ws["w1"]).double().requires_grad_(True)
    lv = ref.loss(w)
    lv.backward()
    gr = w.grad.reshape(-1).numpy()
    e_j = abs(float(lv.detach()) - float(g[f"{run}_J"])) / float(g[f"{run}_J"])
    e_g = float(np.abs(gr[g["gidx"]] - g[f"{run}_grad"]).max() / np.abs(g[f"{run}_grad"]).max())
    print(f"G14 {run}: loss J rel {e_j:.2e}, dJ/dw rel {e_g:.2e}")
    assert e_j < tol_j and e_g < tol_g
