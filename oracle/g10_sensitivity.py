"""ORACLE tool (survey container only): how far does the config-2 trajectory of G10 move when only the
floating-point summation order changes? The reference's own decoder modules (oracle/ref_harness.py) are run again
with a different torch thread count (so the CPU GEMMs block and sum differently), (a) free-running with
torch.optim.LBFGS and (b) as a fixed-step replay of G10's recorded line-search steps through the product's L-BFGS
mirror (vaevar.lbfgs.LBFGS with torch-CPU vector primitives). The relative J difference per outer pass against G10
is the intrinsic sensitivity of the problem; tests/test_gpu_parity.py::test_config2_trajectory_g10 takes its
tolerance from it (written to tests/golden/g10_sensitivity.npz). `--case g13` does the same for G13 (config 3:
T = 2 with the flow stand-in) into tests/golden/g13_sensitivity.npz (test_config3_trajectory_g13); `--case g15`
(config 5: 721x1440 state, T = 2, Nit 5, against the genuine one_step_DA of G15) and `--case g16` (config 4: T = 6,
Nit 3) likewise (test_gpu_config4.py).

Run:  PYTHONDONTWRITEBYTECODE=1 python -B oracle/g10_sensitivity.py [--threads 4] [--case g13]
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
from oracle.da_ref import RefProblem, one_step_da_ref  # noqa: E402
from oracle.make_golden import build_ref  # noqa: E402
from vaevar import config as C  # noqa: E402
from vaevar.lbfgs import LBFGS  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")


class CpuPrims:
    """The vector-primitive contract of vaevar.engine.Context on torch-CPU tensors (double-accumulated dots)."""

    def dot(self, a, b):
        return float((a.double() * b.double()).sum())

    def abssum(self, a):
        return float(a.double().abs().sum())

    def absmax(self, a):
        return float(a.abs().max())

    def reduce_batch(self, reqs, extra=None):
        out = [self.dot(a, b) if op == 0 else self.abssum(a) if op == 1 else self.absmax(a) for op, a, b in reqs]
        return out + (extra.tolist() if extra is not None else [])

    def axpy(self, y, x, alpha):
        y.add_(x, alpha=alpha)

    def axpby(self, out, x, a, y, b):
        out.copy_(a * x + (b * y if y is not None else 0))

    def scale(self, y, alpha):
        y.mul_(alpha)

    def copy(self, dst, src):
        dst.copy_(src)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--case", default="g10", choices=["g10", "g13", "g15", "g16"])
    ap.add_argument("--part", default="both", choices=["both", "free", "replay"],
                    help="free: run only the free-running trajectory and keep its J per pass in oracle/_ref/ (it needs "
                         "no golden, so it can run beside make_golden.py); replay: read that file, run the replay and "
                         "write the sensitivity fixture")
    a = ap.parse_args()
    T, Hs, Ws, nit, fx = {"g10": (1, 128, 256, 10, "g10_config2_trajectory.npz"),
                          "g13": (2, 128, 256, 10, "g13_config3_trajectory.npz"),
                          "g15": (2, 721, 1440, 5, "g15_config5_trajectory.npz"),
                          "g16": (6, 128, 256, 10, "g16_config4_trajectory.npz")}[a.case]
    raw = os.path.join(HERE, "_ref", f"{a.case}_free_J_t{a.threads}.npy")
    torch.set_num_threads(a.threads)
    cwd = os.getcwd()
    tr, _ = ref_harness.import_reference()
    os.chdir(cwd)
    m, _ = build_ref(tr, C.DECODER)
    fm = build_ref(tr, {k: v for k, v in C.FLOW.items() if k != "arch"})[0] if T > 1 else None
    for v in list(m.parameters()) + (list(fm.parameters()) if fm is not None else []):
        v.requires_grad_(False)
    prob = make_problem(nch=69, Hs=Hs, Ws=Ws, T=T, seed=20250620)
    rp = RefProblem(prob, m, C.DECODER["img_size"], fm) if fm is not None else RefProblem(prob, m, C.DECODER["img_size"])
    t0 = time.time()
    if a.part == "replay":
        jf = np.load(raw)
    else:
        _, _, js, _, _ = one_step_da_ref(rp, nit, (32, 128, 256))
        jf = np.array(js).sum(1)
        os.makedirs(os.path.dirname(raw), exist_ok=True)
        np.save(raw, jf)
        print(f"free-running, {a.threads} threads ({time.time() - t0:.0f}s): J per pass {jf.tolist()}", flush=True)
        if a.part == "free":
            return
    g = np.load(os.path.join(GOLD, fx))
    assert int(g["nit"]) == nit if "nit" in g else True, "golden and sensitivity budgets differ"
    Jr = g["J"].sum(1)
    free = np.abs(jf - Jr) / np.abs(Jr)
    print(f"free-running, {a.threads} threads: J rel per pass {free.tolist()}", flush=True)

    # fixed-step replay of G10's line searches through the product's L-BFGS mirror
    z = torch.zeros(1, 32, 128, 256)
    opt = LBFGS(CpuPrims(), z, history_size=10, max_iter=10, line_search_fn="strong_wolfe", device_two_loop=False)
    opt.replay = [(float(t), int(n)) for t, n in zip(g["ls_t"], g["ls_evals"])]

    def closure(zz, gr):
        x = zz.detach().clone().requires_grad_(True)
        r, o = rp.loss_terms(x)
        (r + o).backward()
        gr.copy_(x.grad)
        return float(np.float32(float(r)) + np.float32(float(o)))

    jr = []
    for kk in range(nit + 1):
        with torch.no_grad():
            r, o = rp.loss_terms(z)
        jr.append(float(r) + float(o))
        if kk < nit:
            opt.step(closure)
    rep = np.abs(np.array(jr) - Jr) / np.abs(Jr)
    print(f"replay, {a.threads} threads ({time.time() - t0:.0f}s): J rel per pass {rep.tolist()}", flush=True)
    np.savez(os.path.join(GOLD, f"{a.case}_sensitivity.npz"), threads=a.threads, free_rel=free, replay_rel=rep)


if __name__ == "__main__":
    main()
