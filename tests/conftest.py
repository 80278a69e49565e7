import hashlib
import json
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vae-var_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvaevar on the GPU)")


def has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


# ---------------------------------------------------------------------------------------------------------------
# Parity margins: every tolerance check of a parity test goes through check(), which records the
# achieved error next to its bound; after each test one JSON line {test, outcome, checks: [...]} is appended to
# $VV_MARGINS (default gpurun_out/parity_margins.jsonl when a GPU is present), tagged with the library's sha256 and
# $VV_HEAD (the commit, passed in by the caller: the GPU box has no .git).
_CUR: list = []


def check(name: str, achieved, bound, op: str = "<"):
    """Assert `achieved op bound` (op "<", "<=" or "==") and record both numbers for the margins file."""
    a, b = float(achieved), float(bound)
    ok = {"<": a < b, "<=": a <= b, "==": a == b}[op]
    _CUR.append({"name": name, "achieved": a, "bound": b, "op": op, "ok": bool(ok),
                 "margin": (b / a if a > 0 and op != "==" else None)})
    assert ok, f"{name}: achieved {a:.3e} not {op} bound {b:.3e}"


def note(name: str, achieved):
    """Record a measured quantity that has no bound of its own (e.g. a free-running trajectory's per-pass J error,
    which a line-search branch may move; its final J and xa carry the bounds)."""
    _CUR.append({"name": name, "achieved": float(achieved), "bound": None, "op": None, "ok": True, "margin": None})


def check_bitwise(name: str, a, b):
    """Assert that a and b are identical (tensors, arrays or scalars) and record the largest difference (bound 0)."""
    import numpy as np

    try:
        import torch

        if isinstance(a, torch.Tensor):
            a = a.detach().cpu().double().numpy()
        if isinstance(b, torch.Tensor):
            b = b.detach().cpu().double().numpy()
    except ImportError:
        pass
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if a.shape != b.shape:
        check(name + " (shape)", 1.0, 0.0, "==")
    same = np.array_equal(a, b, equal_nan=True)
    d = 0.0 if same else float(np.nanmax(np.abs(a - b))) if a.size else 1.0
    check(name, d if not same and d > 0 else (0.0 if same else 1.0), 0.0, "==")


def _margins_path():
    p = os.environ.get("VV_MARGINS")
    if p:
        return p
    return os.path.join(ROOT, "gpurun_out", "parity_margins.jsonl") if has_gpu() else None


_LIB_SHA = None


def _lib_sha():
    global _LIB_SHA
    if _LIB_SHA is None:
        so = os.path.join(ROOT, "vae-var_amd", "vaevar", "libvaevar.so")
        try:
            with open(so, "rb") as f:
                _LIB_SHA = hashlib.sha256(f.read()).hexdigest()[:16]
        except OSError:
            _LIB_SHA = ""
    return _LIB_SHA


@pytest.fixture(autouse=True)
def _margin_scope():
    _CUR.clear()
    yield


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    out = yield
    rep = out.get_result()
    if rep.when != "call" or "gpu" not in item.keywords:
        return
    path = _margins_path()
    if not path:
        return
    os.makedirs(os.path.dirname(path), exist_ok=True)
    line = {"test": item.nodeid, "outcome": rep.outcome, "duration_s": round(rep.duration, 2),
            "checks": list(_CUR), "lib_sha16": _lib_sha(), "head": os.environ.get("VV_HEAD", ""),
            "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    with open(path, "a") as f:
        f.write(json.dumps(line) + "\n")
