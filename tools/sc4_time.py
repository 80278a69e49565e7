"""sc4dvar timing (development tool): HIP closure (J + dJ/dw) and transform per call at 128x256 and 721x1440, one
Nit = 10 analysis (LBFGS max_iter 5) on the GPU, and the float64 oracle closure on the host for scale."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
sys.path.insert(0, ROOT)
import torch
from vaevar.problem import make_problem
from vaevar.sc4dvar import BMatrix, Sc4dvarProblem, one_step_sc4dvar

bm = BMatrix.from_npz(os.path.join(ROOT, "tests", "golden", "bq_info_lr.npz"))
for grid in ((128, 256), (721, 1440)):
    p = make_problem(nch=69, Hs=grid[0], Ws=grid[1], T=1, seed=5)
    prob = Sc4dvarProblem(bm, p)
    w = torch.randn(69, 128, 256, device="cuda") * 0.1
    g = torch.empty_like(w)
    for _ in range(3):
        prob.closure(w, g)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        prob.closure(w, g)
    torch.cuda.synchronize()
    ev = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        prob.transform(w)
    torch.cuda.synchronize()
    tr = (time.perf_counter() - t0) / n
    one_step_sc4dvar(prob, nit=1, log_terms=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = one_step_sc4dvar(prob, nit=10, log_terms=False)
    an = time.perf_counter() - t0
    out = {"grid": list(grid), "closure_ms": ev * 1e3, "transform_ms": tr * 1e3, "analysis_s": an,
           "iters": res["n_iter"], "evals": res["n_eval"], "iters_per_s": res["n_iter"] / an}
    if grid == (128, 256) and os.environ.get("CPU", "1") == "1":
        from oracle.sc4dvar_ref import Sc4dvarRef, load_bq
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
        ref = Sc4dvarRef(load_bq(npz=os.path.join(ROOT, "tests", "golden", "bq_info_lr.npz")), p)
        u = (w.cpu().double()).requires_grad_(True)
        ref.loss(u).backward()
        t0 = time.perf_counter()
        for _ in range(3):
            u.grad = None
            ref.loss(u).backward()
        out["oracle_fp64_cpu_closure_ms"] = (time.perf_counter() - t0) / 3 * 1e3
        out["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(out), flush=True)
