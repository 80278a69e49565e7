"""Deterministic synthetic weights and inputs (counter-hash RNG).

The reference ships no checkpoints (`nf_model/ckpts/*.pt`,
`../fengwu-lite/...` are absent), so every parity case and every benchmark
runs on synthetic weights. They are generated from a splitmix64 counter hash
keyed by the parameter's state_dict name, so the same name always yields the
same bits on any machine, and weights never need to be committed.

Scales follow the reference's initialisers loosely (`trunc_normal_(std=.02)`
for Linear weights and position tables, `transformer.py:381-388`), but biases
and LayerNorm affine terms are made non-trivial on purpose so parity tests
exercise them.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix_uniform(seed: int, n: int) -> np.ndarray:
    """n float32 values in [0,1): splitmix64(seed + (i+1)*golden) >> 40 * 2^-24."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        x = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * _GOLDEN
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)


def uniform_sym(seed: int, shape, bound: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = splitmix_uniform(seed, n)
    return ((u * np.float32(2.0) - np.float32(1.0)) * np.float32(bound)).reshape(shape)


def param_value(name: str, shape, base_seed: int = 20250620) -> np.ndarray:
    """Synthetic value of one state_dict entry, chosen by its name."""
    seed = fnv1a64(name) ^ base_seed
    leaf = name.rsplit(".", 1)[-1]
    parent = name.rsplit(".", 2)[-2] if name.count(".") >= 1 else ""
    is_norm = "norm" in parent
    std02 = 0.02 * np.sqrt(3.0)
    if is_norm and leaf == "weight":
        return (np.float32(1.0) + uniform_sym(seed, shape, 0.1)).astype(np.float32)
    if is_norm and leaf == "bias":
        return uniform_sym(seed, shape, 0.05)
    if leaf in ("relative_position_bias_table", "absolute_pos_embed", "pos_embed"):
        return uniform_sym(seed, shape, std02)
    if len(shape) == 4:  # Conv2d (out,in,kh,kw) / ConvTranspose2d (in,out,kh,kw)
        fan = shape[1] * shape[2] * shape[3]
        return uniform_sym(seed, shape, 1.0 / np.sqrt(fan))
    if leaf == "weight":
        return uniform_sym(seed, shape, std02)
    if leaf == "bias":
        return uniform_sym(seed, shape, 0.01)
    return uniform_sym(seed, shape, std02)


def smooth_field(seed: int, shape, sigma: float = 4.0, clip: float = 3.0) -> np.ndarray:
    """Gaussian-filtered white noise (periodic in longitude), unit std, clipped.

    SURVEY §8 d1: `s` is a smooth field, Gaussian-filtered white noise with
    sigma = 4 px, truncated to +-3.
    """
    from scipy.ndimage import gaussian_filter

    u = splitmix_uniform(seed, int(np.prod(shape))).astype(np.float64)
    white = (u - 0.5) * np.sqrt(12.0)
    white = white.reshape(shape)
    sig = [0.0] * (len(shape) - 2) + [sigma, sigma]
    f = gaussian_filter(white, sigma=sig, mode=["nearest"] * (len(shape) - 2) + ["nearest", "wrap"])
    axes = (-2, -1)
    f = (f - f.mean(axis=axes, keepdims=True)) / (f.std(axis=axes, keepdims=True) + 1e-12)
    return np.clip(f, -clip, clip).astype(np.float32)
