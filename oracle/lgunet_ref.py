"""ORACLE (test infrastructure only) — torch-CPU fp32 restatement of the
reference Swin-U-Net `networks_old.transformer.LGUnet_all`.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this module, and only as the checker / the timed CPU baseline.
The product path (vae-var_amd/) never imports it.

It is pinned against the real reference modules by `oracle/make_golden.py`,
which imports `/root/reference` in the survey container and writes the
fixtures under `tests/golden/` (see tests/test_oracle_golden.py).

Reference map (all under /root/reference):
  LGUnet_all.forward            networks_old/transformer.py:747-752
  Enc_net.forward               networks_old/transformer.py:554-568
  Transformer_Encoder.forward   networks_old/transformer.py:390-404
  PatchEmbed.forward            networks_old/transformer.py:41-49
  PatchMerging.forward          networks_old/transformer.py:76-96
  LG_net.forward                networks_old/transformer.py:698-712
  Dec_net.forward               networks_old/transformer.py:599-625
  Transformer_Decoder.forward   networks_old/transformer.py:466-474
  PatchExpand.forward           networks_old/transformer.py:106-118
  SwinTransformerBlock          networks_old/utils/swinblock.py:189-309
  WindowAttention.forward       networks_old/utils/swinblock.py:133-172
  shift mask (quirk Q1)         networks_old/utils/swinblock.py:236-262

The implementation is written as explicit index maps (window order <-> token
order) rather than roll/partition/reverse, so it is an independent
restatement; the golden fixtures pin it to the reference.
"""
from __future__ import annotations

import math
from functools import lru_cache

import torch
import torch.nn.functional as F

EPS_BLOCK = 1e-5   # nn.LayerNorm default inside SwinTransformerBlock (swinblock.py:211)
EPS_OUTER = 1e-6   # partial(nn.LayerNorm, eps=1e-6) (transformer.py:528, 573)


# ----------------------------------------------------------------------------
# index maps
# ----------------------------------------------------------------------------
@lru_cache(maxsize=None)
def window_index(H: int, W: int, ws: int, shift: int) -> torch.Tensor:
    """Token index (h*W+w) held at each window-order position.

    Window order = (window row, window col, row-in-window, col-in-window);
    with a cyclic shift the window position (r, c) holds token
    ((r+shift)%H, (c+shift)%W) (torch.roll by -shift, swinblock.py:275).
    """
    R = (torch.arange(H // ws).view(-1, 1, 1, 1) * ws + torch.arange(ws).view(1, 1, -1, 1) + shift) % H
    C = (torch.arange(W // ws).view(1, -1, 1, 1) * ws + torch.arange(ws).view(1, 1, 1, -1) + shift) % W
    return (R * W + C).reshape(-1)


@lru_cache(maxsize=None)
def shift_mask(H: int, W: int, ws: int, shift: int) -> torch.Tensor:
    """(nW, ws*ws, ws*ws) additive mask for a shifted block (quirk Q1).

    The reference's w-slices are (0,-ws), (-ws,0), (0,None): the middle one is
    empty and the last covers every column, so the label of a pixel depends
    on its row only and only the last window row is masked
    (swinblock.py:240-258). Value -100 where labels differ.
    """
    rows = torch.arange(H)
    lab = torch.where(rows < H - ws, 0, torch.where(rows < H - shift, 1, 2))
    lab = lab.view(H, 1).expand(H, W)
    win = lab.reshape(H // ws, ws, W // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    diff = win.unsqueeze(1) - win.unsqueeze(2)
    return torch.where(diff != 0, torch.tensor(-100.0), torch.tensor(0.0))


@lru_cache(maxsize=None)
def rel_pos_index(ws: int) -> torch.Tensor:
    """Relative position index (ws^2, ws^2) (swinblock.py:93-103)."""
    i = torch.arange(ws * ws)
    ri, ci = i // ws, i % ws
    dr = ri.view(-1, 1) - ri.view(1, -1) + ws - 1
    dc = ci.view(-1, 1) - ci.view(1, -1) + ws - 1
    return dr * (2 * ws - 1) + dc


# ----------------------------------------------------------------------------
# building blocks
# ----------------------------------------------------------------------------
def layer_norm(x, p, name, eps):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


def linear(x, p, name, bias=True):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"] if bias else None)


def swin_block(x, p, pre, heads, ws, shift):
    """x: (B, H, W, C) -> (B, H, W, C)   (swinblock.py:265-309)."""
    B, H, W, C = x.shape
    hd = C // heads
    idx = window_index(H, W, ws, shift)
    nW = (H // ws) * (W // ws)
    N = ws * ws

    xn = layer_norm(x, p, pre + ".norm1", EPS_BLOCK).reshape(B, H * W, C)
    xw = xn[:, idx].reshape(B * nW, N, C)
    qkv = linear(xw, p, pre + ".attn.qkv").reshape(B * nW, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * (hd ** -0.5), qkv[1], qkv[2]
    s = q @ k.transpose(-2, -1)
    table = p[pre + ".attn.relative_position_bias_table"]
    bias = table[rel_pos_index(ws).reshape(-1)].reshape(N, N, heads).permute(2, 0, 1)
    s = s + bias.unsqueeze(0)
    if shift > 0:
        m = shift_mask(H, W, ws, shift)
        s = (s.view(B, nW, heads, N, N) + m.view(1, nW, 1, N, N)).view(B * nW, heads, N, N)
    a = torch.softmax(s, dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B * nW, N, C)
    o = linear(o, p, pre + ".attn.proj").reshape(B, nW * N, C)
    back = torch.empty_like(o)
    back[:, idx] = o
    x = x + back.reshape(B, H, W, C)
    h = linear(layer_norm(x, p, pre + ".norm2", EPS_BLOCK), p, pre + ".mlp.fc1")
    h = F.gelu(h)
    return x + linear(h, p, pre + ".mlp.fc2")


def patch_merging(x, p, pre):
    """(B,H,W,C) -> (B,H/2,W/2,2C): cat order x[0::2,0::2], x[1::2,0::2], x[0::2,1::2], x[1::2,1::2]."""
    B, H, W, C = x.shape
    v = x.reshape(B, H // 2, 2, W // 2, 2, C)          # (b, h, dh, w, dw, c)
    v = v.permute(0, 1, 3, 4, 2, 5).reshape(B, H // 2, W // 2, 4 * C)  # feature = (dw*2+dh)*C + c
    v = layer_norm(v, p, pre + ".norm", EPS_OUTER)
    return linear(v, p, pre + ".reduction", bias=False)


def patch_expand(x, p, pre):
    """(B,H,W,C) -> (B,2H,2W,C/2): 'b h w (p1 p2 c) -> b (h p1) (w p2) c' then LN."""
    x = linear(x, p, pre + ".expand", bias=False)
    B, H, W, C2 = x.shape
    c = C2 // 4
    x = x.reshape(B, H, W, 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(B, 2 * H, 2 * W, c)
    return layer_norm(x, p, pre + ".norm", EPS_OUTER)


def basic_layer(x, p, pre, depth, heads, ws):
    for b in range(depth):
        x = swin_block(x, p, f"{pre}.blocks.{b}", heads, ws, 0 if b % 2 == 0 else ws // 2)
    return x


# ----------------------------------------------------------------------------
# full network
# ----------------------------------------------------------------------------
def lgunet_forward(p: dict, cfg: dict, data: torch.Tensor, prefix: str = "") -> torch.Tensor:
    """Forward of LGUnet_all (transformer.py:747-752). data: (B, sum(inchans), H, W)."""
    pf = prefix
    ws = cfg["window_size"]
    enc_dim = cfg["enc_dim"]
    depths = cfg["enc_depths"]
    heads = cfg["enc_heads"]
    L = len(depths)
    assert L == 2, "restatement covers the 2-level encoder of parameters0_old.yaml"
    B, _, Himg, Wimg = data.shape
    sh, sw = cfg["stride"]
    H0, W0 = Himg // sh, Wimg // sw

    # ---- Enc_net (transformer.py:554-568)
    groups = torch.split(data, list(cfg["inchans_list"]), dim=1)
    lasts, skips = [], []
    for g, d in enumerate(groups):
        e = f"{pf}enc.enc_list.{g}"
        t = F.conv2d(d, p[e + ".patch_embed.proj.weight"], p[e + ".patch_embed.proj.bias"], stride=(sh, sw))
        t = t.flatten(2).transpose(1, 2) + p[e + ".absolute_pos_embed"]
        t = t.reshape(B, H0, W0, enc_dim)
        t = basic_layer(t, p, f"{e}.layers.0", depths[0], heads[0], ws)
        s0 = t
        t = patch_merging(t, p, f"{e}.layers.1.downsample")
        t = basic_layer(t, p, f"{e}.layers.1", depths[1], heads[1], ws)
        s1 = t
        lasts.append(layer_norm(t, p, e + ".norm", EPS_OUTER))
        skips.append((s0, s1))
    x = linear(torch.cat(lasts, -1), p, f"{pf}enc.proj")

    # ---- LG_net (transformer.py:698-712)
    Bx, H1, W1, E = x.shape
    x = (x.reshape(B, H1 * W1, E) + p[f"{pf}net.pos_embed"]).reshape(B, H1, W1, E)
    for li, (dep, nh) in enumerate(zip(cfg["lg_depths"], cfg["lg_heads"])):
        x = basic_layer(x, p, f"{pf}net.layers.{li}", dep, nh, ws)

    # ---- Dec_net (transformer.py:599-625)
    c1 = enc_dim * 2 ** (L - 1)
    dp = linear(x, p, f"{pf}dec.proj")
    parts = torch.split(dp, c1, dim=-1)
    means, stds = [], []
    for g, cout in enumerate(cfg["outchans_list"]):
        d = f"{pf}dec.dec_list.{g}"
        s0, s1 = skips[g]
        t = parts[g]
        # layers_up[0]: dim c1, res (H1,W1), PatchExpand
        t = linear(torch.cat([t, s1], -1), p, f"{d}.concat_back_dim.0")
        t = basic_layer(t, p, f"{d}.layers_up.0", depths[1], heads[1], ws)
        t = patch_expand(t, p, f"{d}.layers_up.0.upsample")
        # layers_up[1]: dim enc_dim, res (H0,W0)
        t = linear(torch.cat([t, s0], -1), p, f"{d}.concat_back_dim.1")
        t = basic_layer(t, p, f"{d}.layers_up.1", depths[0], heads[0], ws)
        t = layer_norm(t, p, f"{d}.norm_up", EPS_OUTER)
        o = F.conv_transpose2d(t.permute(0, 3, 1, 2), p[f"{pf}dec.final_proj_list.{g}.weight"],
                               p[f"{pf}dec.final_proj_list.{g}.bias"], stride=(sh, sw))
        means.append(o[:, : cout // 2])
        stds.append(o[:, cout // 2:])
    # quirk Q2: all mean halves first, then all std halves (transformer.py:616-623)
    return torch.cat(means + stds, dim=1)


# ----------------------------------------------------------------------------
# parameter enumeration (state_dict names and shapes, without buffers)
# ----------------------------------------------------------------------------
def param_shapes(cfg: dict, prefix: str = "") -> dict:
    ws = cfg["window_size"]
    enc_dim, E = cfg["enc_dim"], cfg["embed_dim"]
    depths, heads = cfg["enc_depths"], cfg["enc_heads"]
    sh, sw = cfg["stride"]
    kh, kw = cfg["patch_size"]
    H0, W0 = cfg["img_size"][0] // sh, cfg["img_size"][1] // sw
    H1, W1 = H0 // 2, W0 // 2
    c1 = enc_dim * 2
    out = {}

    def blk(pre, C, nh):
        out[pre + ".norm1.weight"] = (C,)
        out[pre + ".norm1.bias"] = (C,)
        out[pre + ".attn.relative_position_bias_table"] = ((2 * ws - 1) ** 2, nh)
        out[pre + ".attn.qkv.weight"] = (3 * C, C)
        out[pre + ".attn.qkv.bias"] = (3 * C,)
        out[pre + ".attn.proj.weight"] = (C, C)
        out[pre + ".attn.proj.bias"] = (C,)
        out[pre + ".norm2.weight"] = (C,)
        out[pre + ".norm2.bias"] = (C,)
        out[pre + ".mlp.fc1.weight"] = (4 * C, C)
        out[pre + ".mlp.fc1.bias"] = (4 * C,)
        out[pre + ".mlp.fc2.weight"] = (C, 4 * C)
        out[pre + ".mlp.fc2.bias"] = (C,)

    for g, cin in enumerate(cfg["inchans_list"]):
        e = f"{prefix}enc.enc_list.{g}"
        out[e + ".absolute_pos_embed"] = (1, H0 * W0, enc_dim)
        out[e + ".patch_embed.proj.weight"] = (enc_dim, cin, kh, kw)
        out[e + ".patch_embed.proj.bias"] = (enc_dim,)
        for b in range(depths[0]):
            blk(f"{e}.layers.0.blocks.{b}", enc_dim, heads[0])
        out[e + ".layers.1.downsample.reduction.weight"] = (c1, 4 * enc_dim)
        out[e + ".layers.1.downsample.norm.weight"] = (4 * enc_dim,)
        out[e + ".layers.1.downsample.norm.bias"] = (4 * enc_dim,)
        for b in range(depths[1]):
            blk(f"{e}.layers.1.blocks.{b}", c1, heads[1])
        out[e + ".norm.weight"] = (c1,)
        out[e + ".norm.bias"] = (c1,)
    ng = len(cfg["inchans_list"])
    out[f"{prefix}enc.proj.weight"] = (E, c1 * ng)
    out[f"{prefix}enc.proj.bias"] = (E,)
    out[f"{prefix}net.pos_embed"] = (1, H1 * W1, E)
    for li, (dep, nh) in enumerate(zip(cfg["lg_depths"], cfg["lg_heads"])):
        for b in range(dep):
            blk(f"{prefix}net.layers.{li}.blocks.{b}", E, nh)
    nd = len(cfg["outchans_list"])
    for g, cout in enumerate(cfg["outchans_list"]):
        d = f"{prefix}dec.dec_list.{g}"
        for b in range(depths[1]):
            blk(f"{d}.layers_up.0.blocks.{b}", c1, heads[1])
        out[d + ".layers_up.0.upsample.expand.weight"] = (2 * c1, c1)
        out[d + ".layers_up.0.upsample.norm.weight"] = (c1 // 2,)
        out[d + ".layers_up.0.upsample.norm.bias"] = (c1 // 2,)
        for b in range(depths[0]):
            blk(f"{d}.layers_up.1.blocks.{b}", enc_dim, heads[0])
        out[d + ".concat_back_dim.0.weight"] = (c1, 2 * c1)
        out[d + ".concat_back_dim.0.bias"] = (c1,)
        out[d + ".concat_back_dim.1.weight"] = (enc_dim, 2 * enc_dim)
        out[d + ".concat_back_dim.1.bias"] = (enc_dim,)
        out[d + ".norm_up.weight"] = (enc_dim,)
        out[d + ".norm_up.bias"] = (enc_dim,)
    for g, cout in enumerate(cfg["outchans_list"]):
        out[f"{prefix}dec.final_proj_list.{g}.weight"] = (enc_dim, cout, kh, kw)
        out[f"{prefix}dec.final_proj_list.{g}.bias"] = (cout,)
    out[f"{prefix}dec.proj.weight"] = (c1 * nd, E)
    out[f"{prefix}dec.proj.bias"] = (c1 * nd,)
    return out


def synth_params(cfg: dict, prefix: str = "", base_seed: int = 20250620) -> dict:
    """Synthetic fp32 parameters keyed by state_dict name (vaevar.synth)."""
    from vaevar.synth import param_value

    return {k: torch.from_numpy(param_value(k, s, base_seed)) for k, s in param_shapes(cfg, prefix).items()}
