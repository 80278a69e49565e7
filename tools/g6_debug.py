"""Config-5 one_step_DA on the HIP closure, driven by the L-BFGS mirror and by torch.optim.LBFGS (dev tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import numpy as np, torch
from vaevar import config as C
from vaevar.da import one_step_da
from vaevar.engine import DAProblem, LGUnet, loss
from vaevar.problem import make_problem

dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
flow = LGUnet(C.FLOW, 1, 1).load_synthetic()
T = int(os.environ.get("T", "2"))
Hs, Ws = (721, 1440) if not os.environ.get("SMALL") else (128, 256)
prob = DAProblem(dec, make_problem(nch=69, Hs=Hs, Ws=Ws, T=T, seed=20250620), flow=flow if T > 1 else None)

import vaevar.lbfgs as L
_de = L.LBFGS._directional_evaluate
def de(self, closure, x, t, d):
    loss, g = _de(self, closure, x, t, d)
    print("  mirror eval t", repr(t), type(t).__name__, "f", loss, "gtd_new", self._dot(g, d), flush=True)
    return loss, g
L.LBFGS._directional_evaluate = de
_dot = L.LBFGS._dot
def log(kk, jb, jo): print("mirror pass", kk, jb, jo, flush=True)
res = one_step_da(prob, nit=1, log=log)
print("mirror: n_eval", res["n_eval"], "n_iter", res["n_iter"], flush=True)

_tde = torch.optim.LBFGS._directional_evaluate
def tde(self, closure, x, t, d):
    loss, g = _tde(self, closure, x, t, d)
    print("  torch eval t", repr(float(t)), type(t).__name__, "f", loss, "gtd_new", float(g.dot(d)), flush=True)
    return loss, g
torch.optim.LBFGS._directional_evaluate = tde
z = torch.zeros(1, 32, 128, 256, device="cuda", requires_grad=True)
opt = torch.optim.LBFGS([z], history_size=10, max_iter=10, line_search_fn="strong_wolfe")
nev = [0]
def closure():
    opt.zero_grad()
    o = loss(prob, z)
    o.backward()
    nev[0] += 1
    print("  torch-lbfgs eval", nev[0], float(o.detach()), flush=True)
    return o
for kk in range(2):
    with torch.no_grad():
        jb, jo = prob.closure(z.detach(), None)
    print("torch pass", kk, jb, jo, flush=True)
    if kk < 1:
        opt.step(closure)
print("torch: n_eval", nev[0], "n_iter", opt.state[opt._params[0]]["n_iter"], flush=True)
