"""ORACLE (test infrastructure only) — torch-CPU fp32 restatement of the
reference forecast network `networks.LGUnet_all.LGUnet_all_1`,
forward only (it is used by `integrate(xa, forecast_model, 1)`, da_4dvar.py:1329,
and at initialisation, :652 — never differentiated).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this module, and only as the checker. The product path
(vae-var_amd/) never imports it. Pinned against the real reference by
`oracle/make_golden.py` (fixture tests/golden/g7_tiny_lgunet1.npz).

Reference map (all under /root/reference):
  LGUnet_all_1.forward          networks/LGUnet_all.py:772-776
  Enc_net.forward               networks/LGUnet_all.py:578-592
  Transformer_Encoder.forward   networks/LGUnet_all.py:397-411  (downsample BEFORE the blocks, :236-246)
  PatchEmbed (kernel != stride) networks/LGUnet_all.py:25-50
  PatchMerging                  networks/LGUnet_all.py:77-96
  LG_net.forward                networks/LGUnet_all.py:722-740 (layer 0: one global window, :689, :696)
  Dec_net.forward               networks/LGUnet_all.py:624-650 (quirk Q2 channel order)
  Transformer_Decoder.forward   networks/LGUnet_all.py:471-480
  Windowattn_block.forward      networks/utils/Blocks.py:143-159 (pre-norm, LN eps 1e-6)
  SD_attn.forward / create_mask networks/utils/Attention.py:499-664 (RoPE on q,k; -inf mask by row)
  rope2                         networks/utils/positional_encodings.py:230-270

Differences from networks_old (oracle/lgunet_ref.py), all reproduced here:
  * 2-D RoPE on q and k (window-local coordinates) instead of a relative-position bias;
  * shifted-window mask value -inf (not -100), applied only when the last shift is > 0 AND the window
    does not span the full width (Attention.py:609-612);
  * rectangular windows [wh, ww], shift [wh//2, ww//2] on odd blocks (LGUnet_all.py:202, 288, 523);
  * LayerNorm eps 1e-6 everywhere (norm_layer partial, LGUnet_all.py:550, 597, 657);
  * LG layer 0 is a single window over the whole LG grid, no shift (LGUnet_all.py:689, 696, 506-517);
  * any number of encoder levels; PatchEmbed / ConvTranspose kernels may overlap (patch (3,2), stride 2).
The windowing is written as explicit index maps, independent of the reference's roll/partition code.
"""
from __future__ import annotations

from functools import lru_cache

import torch
import torch.nn.functional as F

EPS = 1e-6


@lru_cache(maxsize=None)
def window_index(H: int, W: int, wh: int, ww: int, sh: int, sw: int) -> torch.Tensor:
    """Token index (h*W+w) at each window-order position; window position (r, c) of the rolled image
    holds token ((r+sh)%H, (c+sw)%W) (torch.roll by (-sh, -sw))."""
    R = (torch.arange(H // wh).view(-1, 1, 1, 1) * wh + torch.arange(wh).view(1, 1, -1, 1) + sh) % H
    C = (torch.arange(W // ww).view(1, -1, 1, 1) * ww + torch.arange(ww).view(1, 1, 1, -1) + sw) % W
    return (R * W + C).reshape(-1)


@lru_cache(maxsize=None)
def shift_mask(H: int, W: int, wh: int, ww: int, sh: int) -> torch.Tensor:
    """(nW, N, N) additive mask: the labels of create_mask depend on the (rolled) row only, because the
    w-slices are (0,-ww), (-ww,0) [empty], (0,None) [all columns]; -inf where labels differ."""
    rows = torch.arange(H)
    lab = torch.where(rows < H - wh, 0, torch.where(rows < H - sh, 1, 2))
    lab = lab.view(H, 1).expand(H, W)
    win = lab.reshape(H // wh, wh, W // ww, ww).permute(0, 2, 1, 3).reshape(-1, wh * ww)
    diff = win.unsqueeze(1) - win.unsqueeze(2)
    return torch.where(diff != 0, torch.tensor(float("-inf")), torch.tensor(0.0))


@lru_cache(maxsize=None)
def rope_tables(wh: int, ww: int, hd: int):
    """(cos1, sin1, cos2, sin2) of rope2 over window-local (row, col), each (wh*ww, d) in fp32."""
    half = hd // 2
    d1, d2 = half // 2, half - half // 2
    rr = torch.arange(wh).view(-1, 1).expand(wh, ww).reshape(-1)
    cc = torch.arange(ww).view(1, -1).expand(wh, ww).reshape(-1)
    f1 = 10000 ** -(torch.arange(0, d1) / d1)
    f2 = 10000 ** -(torch.arange(0, d2) / d2)
    a1 = rr.unsqueeze(-1) * f1
    a2 = cc.unsqueeze(-1) * f2
    return torch.cos(a1), torch.sin(a1), torch.cos(a2), torch.sin(a2)


def rope(x: torch.Tensor, wh: int, ww: int) -> torch.Tensor:
    """x: (..., N=wh*ww, hd): split [d1, d2, d1, d2] and rotate pairs (x11, x12) by row, (x21, x22) by col."""
    hd = x.shape[-1]
    c1, s1, c2, s2 = rope_tables(wh, ww, hd)
    d1, d2 = c1.shape[-1], c2.shape[-1]
    x11, x21, x12, x22 = x.split([d1, d2, d1, d2], dim=-1)
    return torch.cat([x11 * c1 - x12 * s1, x21 * c2 - x22 * s2, x12 * c1 + x11 * s1, x22 * c2 + x21 * s2], dim=-1)


def layer_norm(x, p, name):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], EPS)


def linear(x, p, name, bias=True):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"] if bias else None)


def window_block(x, p, pre, heads, wh, ww, sh, sw):
    """Windowattn_block (pre_norm): x += proj(SD_attn(norm(x))); x += mlp(norm2(x)). x: (B, H, W, C)."""
    B, H, W, C = x.shape
    hd = C // heads
    N = wh * ww
    nW = (H // wh) * (W // ww)
    roll = sw > 0                                   # Attention.py:614-619 (shift_size[-1] > 0)
    masked = sw > 0 and ww != W                     # Attention.py:609-612
    idx = window_index(H, W, wh, ww, sh if roll else 0, sw if roll else 0)
    xn = layer_norm(x, p, pre + ".norm").reshape(B, H * W, C)
    xw = xn[:, idx].reshape(B * nW, N, C)
    qkv = linear(xw, p, pre + ".attn.qkv").reshape(B * nW, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = rope(q, wh, ww) * (hd ** -0.5)              # q = rope(q) * scale (Attention.py:634-639)
    k = rope(k, wh, ww)
    s = q @ k.transpose(-2, -1)
    if masked:
        m = shift_mask(H, W, wh, ww, sh)
        s = (s.view(B, nW, heads, N, N) + m.view(1, nW, 1, N, N)).view(B * nW, heads, N, N)
    a = torch.softmax(s, dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B * nW, N, C)
    back = torch.empty(B, H * W, C, dtype=o.dtype)
    back[:, idx] = o.reshape(B, nW * N, C)          # window_reverse + roll back by (sh, sw)
    x = x + linear(back, p, pre + ".attn.proj").reshape(B, H, W, C)
    h = F.gelu(linear(layer_norm(x, p, pre + ".norm2"), p, pre + ".mlp.fc1"))
    return x + linear(h, p, pre + ".mlp.fc2")


def swin_layer(x, p, pre, depth, heads, wh, ww):
    for b in range(depth):
        sh, sw = (0, 0) if b % 2 == 0 else (wh // 2, ww // 2)
        x = window_block(x, p, f"{pre}.blocks.{b}", heads, wh, ww, sh, sw)
    return x


def patch_merging(x, p, pre):
    B, H, W, C = x.shape
    v = x.reshape(B, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 4, 2, 5).reshape(B, H // 2, W // 2, 4 * C)
    return linear(layer_norm(v, p, pre + ".norm"), p, pre + ".reduction", bias=False)


def patch_expand(x, p, pre):
    x = linear(x, p, pre + ".expand", bias=False)
    B, H, W, C2 = x.shape
    c = C2 // 4
    x = x.reshape(B, H, W, 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(B, 2 * H, 2 * W, c)
    return layer_norm(x, p, pre + ".norm")


def grids(cfg):
    """Token grid of every encoder level, the LG grid and the LG layer-0 window."""
    sh, sw = cfg["stride"]
    Himg, Wimg = cfg["img_size"]
    L = len(cfg["enc_depths"])
    H0, W0 = Himg // sh, Wimg // sw
    lvl = [(H0 >> l, W0 >> l) for l in range(L)]
    lg = (Himg // (sh * 2 ** (L - 1)), Wimg // (sw * 2 ** (L - 1)))  # LG_net img // lg_patch_size
    return lvl, lg


def lgunet1_forward(p: dict, cfg: dict, data: torch.Tensor, prefix: str = "") -> torch.Tensor:
    pf = prefix
    wh, ww = cfg["window_size"]
    enc_dim = cfg["enc_dim"]
    depths, heads = cfg["enc_depths"], cfg["enc_heads"]
    L = len(depths)
    sh, sw = cfg["stride"]
    B = data.shape[0]
    lvl, lg = grids(cfg)
    assert lvl[-1] == lg, (lvl, lg)

    groups = torch.split(data, list(cfg["inchans_list"]), dim=1)
    lasts, skips = [], []
    for g, d in enumerate(groups):
        e = f"{pf}enc.enc_list.{g}"
        t = F.conv2d(d, p[e + ".patch_embed.proj.weight"], p[e + ".patch_embed.proj.bias"], stride=(sh, sw))
        t = t.flatten(2).transpose(1, 2) + p[e + ".absolute_pos_embed"]
        t = t.reshape(B, lvl[0][0], lvl[0][1], enc_dim)
        sk = []
        for l in range(L):
            if l > 0:
                t = patch_merging(t, p, f"{e}.layers.{l}.downsample")
            t = swin_layer(t, p, f"{e}.layers.{l}", depths[l], heads[l], wh, ww)
            sk.append(t)
        lasts.append(layer_norm(t, p, e + ".norm"))
        skips.append(sk)
    x = linear(torch.cat(lasts, -1), p, f"{pf}enc.proj")

    Hg, Wg = lg
    E = x.shape[-1]
    x = (x.reshape(B, Hg * Wg, E) + p[f"{pf}net.pos_embed"]).reshape(B, Hg, Wg, E)
    for li, (dep, nh) in enumerate(zip(cfg["lg_depths"], cfg["lg_heads"])):
        pre = f"{pf}net.layers.{li}"
        if li == 0:   # "window_block": one window over the whole LG grid, never shifted
            for b in range(dep):
                x = window_block(x, p, f"{pre}.blocks.{b}", nh, Hg, Wg, 0, 0)
        else:
            x = swin_layer(x, p, pre, dep, nh, wh, ww)

    cL = enc_dim * 2 ** (L - 1)
    parts = torch.split(linear(x, p, f"{pf}dec.proj"), cL, dim=-1)
    means, stds = [], []
    for g, cout in enumerate(cfg["outchans_list"]):
        d = f"{pf}dec.dec_list.{g}"
        t = parts[g]
        for i in range(L):
            lev = L - 1 - i
            t = linear(torch.cat([t, skips[g][lev]], -1), p, f"{d}.concat_back_dim.{i}")
            t = swin_layer(t, p, f"{d}.layers_up.{i}", depths[lev], heads[lev], wh, ww)
            if i < L - 1:
                t = patch_expand(t, p, f"{d}.layers_up.{i}.upsample")
        t = layer_norm(t, p, f"{d}.norm_up")
        o = F.conv_transpose2d(t.permute(0, 3, 1, 2), p[f"{pf}dec.final_proj_list.{g}.weight"],
                               p[f"{pf}dec.final_proj_list.{g}.bias"], stride=(sh, sw))
        means.append(o[:, : cout // 2])
        stds.append(o[:, cout // 2:])
    return torch.cat(means + stds, dim=1)


def param_shapes(cfg: dict, prefix: str = "") -> dict:
    enc_dim, E = cfg["enc_dim"], cfg["embed_dim"]
    depths, heads = cfg["enc_depths"], cfg["enc_heads"]
    kh, kw = cfg["patch_size"]
    L = len(depths)
    lvl, lg = grids(cfg)
    cl = [enc_dim * 2 ** l for l in range(L)]
    out = {}

    def blk(pre, C):
        for n in ("norm", "norm2"):
            out[f"{pre}.{n}.weight"] = (C,)
            out[f"{pre}.{n}.bias"] = (C,)
        out[pre + ".attn.qkv.weight"] = (3 * C, C)
        out[pre + ".attn.qkv.bias"] = (3 * C,)
        out[pre + ".attn.proj.weight"] = (C, C)
        out[pre + ".attn.proj.bias"] = (C,)
        out[pre + ".mlp.fc1.weight"] = (4 * C, C)
        out[pre + ".mlp.fc1.bias"] = (4 * C,)
        out[pre + ".mlp.fc2.weight"] = (C, 4 * C)
        out[pre + ".mlp.fc2.bias"] = (C,)

    for g, cin in enumerate(cfg["inchans_list"]):
        e = f"{prefix}enc.enc_list.{g}"
        out[e + ".absolute_pos_embed"] = (1, lvl[0][0] * lvl[0][1], enc_dim)
        out[e + ".patch_embed.proj.weight"] = (enc_dim, cin, kh, kw)
        out[e + ".patch_embed.proj.bias"] = (enc_dim,)
        for l in range(L):
            for b in range(depths[l]):
                blk(f"{e}.layers.{l}.blocks.{b}", cl[l])
            if l > 0:
                out[f"{e}.layers.{l}.downsample.reduction.weight"] = (cl[l], 2 * cl[l])
                out[f"{e}.layers.{l}.downsample.norm.weight"] = (2 * cl[l],)
                out[f"{e}.layers.{l}.downsample.norm.bias"] = (2 * cl[l],)
        out[e + ".norm.weight"] = (cl[-1],)
        out[e + ".norm.bias"] = (cl[-1],)
    ng = len(cfg["inchans_list"])
    out[f"{prefix}enc.proj.weight"] = (E, cl[-1] * ng)
    out[f"{prefix}enc.proj.bias"] = (E,)
    out[f"{prefix}net.pos_embed"] = (1, lg[0] * lg[1], E)
    for li, dep in enumerate(cfg["lg_depths"]):
        for b in range(dep):
            blk(f"{prefix}net.layers.{li}.blocks.{b}", E)
    nd = len(cfg["outchans_list"])
    for g in range(nd):
        d = f"{prefix}dec.dec_list.{g}"
        for i in range(L):
            lev = L - 1 - i
            for b in range(depths[lev]):
                blk(f"{d}.layers_up.{i}.blocks.{b}", cl[lev])
            if i < L - 1:
                out[f"{d}.layers_up.{i}.upsample.expand.weight"] = (2 * cl[lev], cl[lev])
                out[f"{d}.layers_up.{i}.upsample.norm.weight"] = (cl[lev] // 2,)
                out[f"{d}.layers_up.{i}.upsample.norm.bias"] = (cl[lev] // 2,)
            out[f"{d}.concat_back_dim.{i}.weight"] = (cl[lev], 2 * cl[lev])
            out[f"{d}.concat_back_dim.{i}.bias"] = (cl[lev],)
        out[d + ".norm_up.weight"] = (enc_dim,)
        out[d + ".norm_up.bias"] = (enc_dim,)
    for g, cout in enumerate(cfg["outchans_list"]):
        out[f"{prefix}dec.final_proj_list.{g}.weight"] = (enc_dim, cout, kh, kw)
        out[f"{prefix}dec.final_proj_list.{g}.bias"] = (cout,)
    out[f"{prefix}dec.proj.weight"] = (cl[-1] * nd, E)
    out[f"{prefix}dec.proj.bias"] = (cl[-1] * nd,)
    return out


def synth_params(cfg: dict, prefix: str = "", base_seed: int = 20250620) -> dict:
    from vaevar.synth import param_value

    return {k: torch.from_numpy(param_value(k, s, base_seed)) for k, s in param_shapes(cfg, prefix).items()}
