"""ORACLE harness (survey container only) — imports the real reference from
/root/reference so golden fixtures can be generated from it.

Never imported on the GPU box (the reference does not travel). Recipe per
SURVEY §8 c2: in-process stub modules for the absent third-party imports
(timm, fairscale, torchvision, turtle, petrel_client, torch_harmonics,
xarray, xspharm, tensorboard), sys.path + chdir to the reference (quirk Q8),
and no bytecode writes into the read-only tree.
"""
from __future__ import annotations

import importlib.machinery
import os
import sys
import types

REF = "/root/reference"


def _mod(name: str, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    m.__path__ = []  # allow submodules
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    import collections.abc
    import itertools

    import torch

    class DropPath(torch.nn.Module):  # drop_path = 0 everywhere on the DA path
        def __init__(self, *a, **k):
            super().__init__()

        def forward(self, x):
            return x

    def to_2tuple(x):  # timm semantics
        if isinstance(x, collections.abc.Iterable) and not isinstance(x, str):
            return tuple(x)
        return tuple(itertools.repeat(x, 2))

    _mod("timm")
    _mod("timm.models")
    _mod("timm.models.layers", DropPath=DropPath, to_2tuple=to_2tuple, trunc_normal_=torch.nn.init.trunc_normal_)
    _mod("fairscale")
    _mod("fairscale.nn")
    _mod("fairscale.nn.checkpoint")
    _mod("fairscale.nn.checkpoint.checkpoint_activations", checkpoint_wrapper=lambda m, *a, **k: m)
    _mod("torchvision")
    _mod("torchvision.utils")
    sys.modules["torchvision"].utils = sys.modules["torchvision.utils"]
    _mod("turtle", forward=None)
    _mod("petrel_client")
    _mod("petrel_client.client", Client=object)
    _mod("torch_harmonics", RealSHT=None, InverseRealSHT=None)
    sys.modules["torch_harmonics"].__all__ = []
    _mod("xarray")
    _mod("xspharm")
    _mod("xspharm.xspharm", xspharm=None)
    sys.modules["xspharm"].xspharm = sys.modules["xspharm.xspharm"]
    try:
        import torch.utils.tensorboard  # noqa: F401
    except Exception:
        _mod("torch.utils.tensorboard", SummaryWriter=object)


def import_reference():
    """Return (networks_old.transformer, networks_old.utils.swinblock) from /root/reference."""
    sys.dont_write_bytecode = True
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    os.chdir(REF)  # Q8: VAE_lr reads nf_model/<param>.yaml relative to cwd
    import importlib

    tr = importlib.import_module("networks_old.transformer")
    sb = importlib.import_module("networks_old.utils.swinblock")
    return tr, sb
