"""ORACLE (test infrastructure only) — torch-CPU float64 restatement of the sc4dvar B-matrix transform and loss of
`da_4dvar.py`.

  init_b_matrix     da_4dvar.py:520-526  (len_scale * scale_factor, reg_coeff, std_sur, vert_eig_value/_vec)
  get_static_info   da_4dvar.py:608-628  (zonal Gaussian kernel, its SHT, sph_scale)
  transform         da_4dvar.py:878-931  (SHT filter, balance regression, vertical EOFs, stream function /
                                          velocity potential -> wind, nearest interpolation, + xb)
  loss / closure    da_4dvar.py:1065-1107 (J_b = sum(w^2)/2, J_o over the window; the flow forecasts are
                                          integrate(..., detach=True), so they add to J but not to dJ/dw)

RealSHT / InverseRealSHT come from `torch_harmonics`, which is NOT installed here and is not pinned by the
reference (no requirements file). They are restated from the library's published algorithm (torch_harmonics
0.6/0.7 `sht.py`, `quadrature.py`, `legendre.py`) for grid="equiangular", norm="ortho", csphase=True:
  nodes      theta_k = pi k / (nlat-1), k = 0 .. nlat-1 (north pole first; np.flip(np.arccos(cost)))
  weights    Clenshaw-Curtis on [-1, 1] (clenshaw_curtiss_weights)
  legpoly    orthonormal associated Legendre functions with the Condon-Shortley phase, P[m][l][k], m < mmax,
             l < lmax; lmax = nlat, mmax = nlon // 2 + 1
  forward    X = 2 pi rfft(x, norm="forward");  a[l, m] = sum_k X[k, m] w_k P[m][l][k]
  inverse    X[k, m] = sum_l a[l, m] P[m][l][k];  x = irfft(X, n=nlon, norm="forward")
PARITY UNPINNED against torch_harmonics itself. What is pinned (tests/test_oracle_golden.py): the quadrature
integrates polynomials of degree < nlat exactly, the Legendre table equals scipy.special.sph_harm_y, and the
transform pair reproduces band-limited fields (SHT o iSHT = identity there).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.nn.functional as F

NLAT, NLON, NLEV = 128, 256, 13
DT = torch.float64


def clenshaw_curtis(n: int):
    """Nodes cos(theta_k), theta_k = pi k/(n-1) (descending x) and the Clenshaw-Curtis weights (Waldvogel's
    closed form; symmetric, so the node order of torch_harmonics' ascending `cost` does not change them)."""
    N = n - 1
    th = np.pi * np.arange(n) / N
    w = np.zeros(n)
    for k in range(n):
        s = 0.0
        for j in range(1, N // 2 + 1):
            b = 1.0 if 2 * j == N else 2.0
            s += b / (4.0 * j * j - 1.0) * np.cos(2.0 * j * th[k])
        c = 1.0 if k in (0, N) else 2.0
        w[k] = c / N * (1.0 - s)
    return np.cos(th), w


def legpoly(mmax: int, lmax: int, x: np.ndarray) -> np.ndarray:
    """P[m][l][k]: orthonormal associated Legendre functions at x_k with the Condon-Shortley phase
    (torch_harmonics legendre.legpoly, norm 'ortho')."""
    nmax = max(mmax, lmax)
    v = np.zeros((nmax, nmax, len(x)))
    v[0, 0, :] = 1.0 / np.sqrt(4 * np.pi)
    for l in range(1, nmax):
        v[l - 1, l, :] = np.sqrt(2 * l + 1) * x * v[l - 1, l - 1, :]
        v[l, l, :] = np.sqrt((2 * l + 1) * (1 + x) * (1 - x) / 2 / l) * v[l - 1, l - 1, :]
    for l in range(2, nmax):
        for m in range(0, l - 1):
            v[m, l, :] = (x * np.sqrt((2 * l - 1) / (l - m) * (2 * l + 1) / (l + m)) * v[m, l - 1, :]
                          - np.sqrt((l + m - 1) / (l - m) * (2 * l + 1) / (2 * l - 3) * (l - m - 1) / (l + m))
                          * v[m, l - 2, :])
    v = v[:mmax, :lmax]
    v[1::2] *= -1.0
    return v


class SHT:
    """RealSHT / InverseRealSHT(nlat, nlon, grid='equiangular') in float64."""

    def __init__(self, nlat: int = NLAT, nlon: int = NLON):
        self.nlat, self.nlon = nlat, nlon
        self.lmax, self.mmax = nlat, nlon // 2 + 1
        x, w = clenshaw_curtis(nlat)
        self.x, self.w = x, w
        P = legpoly(self.mmax, self.lmax, x)
        self.P = torch.from_numpy(P)                                  # inverse: pct
        self.W = torch.from_numpy(P * w[None, None, :])               # forward: pct * quadrature weights

    @staticmethod
    def _legendre(X: torch.Tensor, M: torch.Tensor) -> torch.Tensor:
        """out[..., i, m] = sum_j M[m, i, j] X[..., j, m] for complex X and the real table M (real and imaginary
        parts as separate real batched products; complex einsum is ~100x slower on the CPU)."""
        lead = X.shape[:-2]
        Xr = torch.view_as_real(X.reshape((-1,) + X.shape[-2:]))        # (B, j, m, 2)
        B, J, Mm = Xr.shape[0], Xr.shape[1], Xr.shape[2]
        Y = Xr.permute(2, 1, 0, 3).reshape(Mm, J, B * 2)                  # (m, j, B*2)
        O = torch.bmm(M, Y).reshape(Mm, M.shape[1], B, 2).permute(2, 1, 0, 3)
        return torch.view_as_complex(O.contiguous()).reshape(lead + (M.shape[1], Mm))

    def forward(self, f: torch.Tensor) -> torch.Tensor:
        X = 2.0 * math.pi * torch.fft.rfft(f, dim=-1, norm="forward")[..., :self.mmax]
        return self._legendre(X, self.W)                                 # a[l, m] = sum_k W[m, l, k] X[k, m]

    def inverse(self, a: torch.Tensor) -> torch.Tensor:
        X = self._legendre(a, self.P.transpose(1, 2))                    # X[k, m] = sum_l P[m, l, k] a[l, m]
        return torch.fft.irfft(X, n=self.nlon, dim=-1, norm="forward")


def load_bq(coeff_dir: str | None = None, npz: str | None = None, scale_factor: float = 1.0) -> dict:
    """init_b_matrix (da_4dvar.py:520-526), float64: from the reference's dataset/bq_info_lr/*.npy or the
    committed copy tests/golden/bq_info_lr.npz."""
    keys = ("len_scale", "reg_coeff", "std_sur", "vert_eig_value", "vert_eig_vec")
    if npz is not None:
        with np.load(npz) as z:
            d = {k: np.asarray(z[k], np.float64) for k in keys}
    else:
        d = {k: np.load(os.path.join(coeff_dir, k + ".npy")).astype(np.float64) for k in keys}
    d["len_scale"] = d["len_scale"] * scale_factor
    return {k: torch.from_numpy(v) for k, v in d.items()}


class Sc4dvarRef:
    """The sc4dvar closure state (da_4dvar.py:1064-1177) at state grid (Hs, Ws); nchannel 69, nlev 13."""

    def __init__(self, bq: dict, prob: dict, flow_fn=None, obs_coeff: float = 1.0, hpad: int = 112,
                 interp=None, const_dtype=torch.float32):
        """const_dtype: the dtype the reference forms partial_x / partial_y's constants in (its default dtype,
        float32; G14 also runs the reference with float64 as the default dtype and compares with float64 here)."""
        self.bq = {k: v.to(DT) for k, v in bq.items()}
        self.sht = SHT()
        L = self.bq["len_scale"]
        C = L.shape[0]
        # get_static_info (:614-628): zonal kernel exp(-i^2 / (8 len^2)) on the first hpad latitude rows
        kern = torch.zeros(C, NLAT, NLON, dtype=DT)
        for i in range(hpad):
            kern[:, i, :] = torch.exp(-(i ** 2) / (8 * L ** 2))[:, None]
        ck = self.sht.forward(kern)[:, :, 0]                                            # (C, lmax)
        l = torch.arange(NLAT, dtype=DT)
        self.sph_scale = 2 * np.pi * torch.sqrt(4 * np.pi / (2 * l + 1))                 # (lmax,) broadcast on m
        self.coeffs_kernel = ck
        self.C = C
        t = lambda a: torch.as_tensor(np.asarray(a), dtype=DT)
        self.xb, self.yo, self.H, self.R = t(prob["xb"]), t(prob["yo"]), t(prob["H"]), t(prob["R"])
        self.mean, self.std = t(prob["mean"]), t(prob["std"])
        self.T = self.yo.shape[0]
        self.Hs, self.Ws = self.xb.shape[-2:]
        self.flow_fn, self.obs_coeff = flow_fn, obs_coeff
        self.interp = None if interp is None else t(interp)
        # partial_x / partial_y constants (:908-916), as the reference forms them in fp32
        self.x_scaling = torch.sin(torch.linspace(1 / 180 * torch.pi, 179 / 180 * torch.pi, NLAT,
                                                  dtype=const_dtype)).to(DT).reshape(1, -1, 1)
        self.lat_coord = ((torch.arange(NLAT) * 111195 * 180).to(const_dtype) / (NLAT - 1)).to(DT)

    def horizontal(self, u: torch.Tensor) -> torch.Tensor:
        """isht(sph_scale * sht(u_c) * coeffs_kernel_c[:, 0]) * 11 / len_c^2  (:883-888)."""
        a = self.sht.forward(u) * (self.sph_scale[None, :, None] * self.coeffs_kernel[:, :, None])
        s = self.sht.inverse(a)
        return 11 * s / (self.bq["len_scale"].reshape(-1, 1, 1) ** 2)

    def transform(self, u: torch.Tensor) -> torch.Tensor:
        """da_4dvar.py:878-931 (without the final + xb and interpolation: `recon` on the 128x256 grid)."""
        nl = NLEV
        st = self.horizontal(u)
        reg = self.bq["reg_coeff"]
        if reg.shape[1] == nl:
            psi = st[4 + nl * 2:4 + nl * 3]
        else:
            psi = torch.cat([st[4:4 + nl], st[4 + nl * 2:4 + nl * 3]], 0)
        vmode = st + torch.einsum("ij,jhw->ihw", reg, psi)
        sfvp = vmode.clone()
        sfvp[0:4] = vmode[0:4] * self.bq["std_sur"].reshape(-1, 1, 1)
        for i in range(5):
            E = self.bq["vert_eig_vec"][i] @ torch.diag(torch.sqrt(self.bq["vert_eig_value"][i]))
            blk = vmode[4 + nl * i:4 + nl * (i + 1)].reshape(nl, -1)
            sfvp[4 + nl * i:4 + nl * (i + 1)] = (E @ blk).reshape(nl, NLAT, NLON)

        def partial_x(f):
            s1 = torch.cat([f[:, :, 1:], f[:, :, :1]], 2)
            s2 = torch.cat([f[:, :, -1:], f[:, :, :-1]], 2)
            return (s2 - s1) / (2 * 111195 * 180 / NLAT * self.x_scaling)

        def partial_y(f):
            return torch.gradient(f, spacing=(self.lat_coord,), dim=1)[0]

        recon = sfvp.clone()
        sf, vp = sfvp[4 + nl * 2:4 + nl * 3], sfvp[4 + nl * 3:4 + nl * 4]
        recon[4 + nl * 2:4 + nl * 3] = partial_y(sf) - partial_x(vp)
        recon[4 + nl * 3:4 + nl * 4] = -partial_x(sf) - partial_y(vp)
        return recon

    def state(self, u: torch.Tensor) -> torch.Tensor:
        """x = F.interpolate(recon, (Hs, Ws)) + xb  (:928)."""
        r = self.transform(u)
        if (self.Hs, self.Ws) != (NLAT, NLON):
            r = F.interpolate(r.unsqueeze(0), (self.Hs, self.Ws)).squeeze(0)
        return r + self.xb

    def integrate(self, x: torch.Tensor) -> torch.Tensor:
        """integrate(x, flow, 1, True) (:666-681): interpolation=True, detach=True."""
        z = ((x - self.mean.reshape(-1, 1, 1)) / self.std.reshape(-1, 1, 1)).unsqueeze(0)
        if (self.Hs, self.Ws) != (NLAT, NLON):
            z = F.interpolate(z, (NLAT, NLON))
        z = self.flow_fn(z.to(torch.float32)).to(DT)[:, :self.C].detach()
        if (self.Hs, self.Ws) != (NLAT, NLON):
            z = F.interpolate(z, (self.Hs, self.Ws))
        return z.reshape(self.C, self.Hs, self.Ws) * self.std.reshape(-1, 1, 1) + self.mean.reshape(-1, 1, 1)

    def loss_terms(self, u: torch.Tensor):
        """(J_b, J_o) of loss(w) = cal_loss_bg(w) + obs_coeff * cal_loss_obs(transform(w, xb)) (:1099-1101)."""
        x = self.state(u)
        xs = [x]
        for _ in range(self.T - 1):
            x = self.integrate(x)
            xs.append(x)
        xp = torch.stack(xs, 0)
        if self.interp is not None:
            parts = [xp[:, :4]]
            for i in range(5):
                m = xp[:, 4 + i * NLEV:4 + (i + 1) * NLEV]
                parts.append(F.linear(m.transpose(1, 3), self.interp).transpose(1, 3))
            xp = torch.cat(parts, 1)
        jb = torch.sum(u ** 2) / 2
        jo = torch.sum(self.H * (xp - self.yo) ** 2 / self.R) / 2
        return jb, jo

    def loss(self, u: torch.Tensor) -> torch.Tensor:
        jb, jo = self.loss_terms(u)
        return jb + self.obs_coeff * jo
