"""Full CPU convergence of BASELINE config 2 (SURVEY §8 d: "Run a full CPU convergence for config 2"): the oracle
restatement of the reference path (torch-CPU fp32, weight gradients on as the reference computes them, quirk Q5)
driven by torch.optim.LBFGS(history 10, max_iter 10, strong Wolfe) for Nit = 10 outer passes on the same synthetic
problem and weights as bench.py's config 2 (make_problem seed 20250620). Without the per-pass logging evaluations.
Prints one JSON line with the wall clock, iterations, evaluations and the thread count. Runs on the GPU box's host
cores (the GPU is not used)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
sys.path.insert(0, ROOT)

import torch

from oracle.da_ref import oracle_problem
from oracle.lgunet_ref import synth_params
from vaevar import config as C
from vaevar.problem import make_problem

threads = int(os.environ.get("THREADS", os.environ.get("OMP_NUM_THREADS", "16")))
torch.set_num_threads(threads)
nit = int(os.environ.get("NIT", "10"))
p = make_problem(nch=69, Hs=128, Ws=256, T=1, seed=20250620)
params = synth_params(C.DECODER)
for v in params.values():
    v.requires_grad_(True)  # the reference's VAE keeps requires_grad=True (Q5)
rp = oracle_problem(p, params, C.DECODER)
z = torch.zeros(1, 32, 128, 256, requires_grad=True)
opt = torch.optim.LBFGS([z], history_size=10, max_iter=10, line_search_fn="strong_wolfe")
n_eval = [0]


def closure():
    opt.zero_grad()
    for v in params.values():
        v.grad = None
    obj = rp.loss(z)
    obj.backward()
    n_eval[0] += 1
    return obj


with torch.no_grad():
    j0 = float(rp.loss(z))
t0 = time.time()
for kk in range(nit):
    opt.step(closure)
    print(json.dumps({"pass": kk + 1, "elapsed_s": time.time() - t0, "evals": n_eval[0]}), flush=True)
with torch.no_grad():
    xa = rp.analysis(z)
wall = time.time() - t0
with torch.no_grad():
    j1 = float(rp.loss(z))
n_iter = opt.state[opt._params[0]]["n_iter"]
print(json.dumps({"cpu_convergence": True, "wall_clock_s": wall, "iters": n_iter, "evals": n_eval[0],
                  "iters_per_s": n_iter / wall, "threads": threads, "J_start": j0, "J_final": j1,
                  "workload": "config 2 (69ch 128x256, full decoder), Nit 10, torch.optim.LBFGS over the oracle "
                              "restatement, weight grads on"}), flush=True)
