"""Closure J / dJ/dz of the config-3 problem under each bf16x6 short-K tile (tuning key bs_tile) against the default
(development tool, run on the GPU box): the tiles run the same per-element product order, so the results should be
bit-identical."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch  # noqa: E402

from vaevar import config as C  # noqa: E402
from vaevar.engine import DAProblem, LGUnet  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402
from vaevar.synth import smooth_field  # noqa: E402

dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
flow = LGUnet(C.FLOW, 1, 1).load_synthetic()
prob = DAProblem(dec, make_problem(T=2), flow=flow)
z = torch.from_numpy(0.3 * smooth_field(5, (1, 32, 128, 256))).cuda()
res = {}
for v in (0, 25, 26, 27):
    dec.ctx.set_tuning("bs_tile", v)
    flow.ctx.set_tuning("bs_tile", v)
    g = torch.empty_like(z)
    jb, jo = prob.closure(z, g)
    res[v] = (jb + jo, g.clone())
dec.ctx.set_tuning("bs_tile", 0)
j0, g0 = res[0]
for v in (25, 26, 27):
    j, g = res[v]
    print(f"bs_tile {v}: J rel {abs(j - j0) / abs(j0):.2e}, dJ/dz max rel {float((g - g0).abs().max() / g0.abs().max()):.2e}, "
          f"bitwise {torch.equal(g, g0) and j == j0}", flush=True)
