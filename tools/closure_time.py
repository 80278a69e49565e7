"""Config-3 closure time of the library this process loads (VAEVAR_LIB to pick another build): T = 2, graph-replayed
closures, the minimum and median of 5 repeats of 40 (development tool for same-box library A/Bs,
tools/gpu_ab_closure.sh)."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch  # noqa: E402

from vaevar import config as C  # noqa: E402
from vaevar.engine import DAProblem, LGUnet  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402

dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
flow = LGUnet(C.FLOW, 1, 1).load_synthetic()
prob = DAProblem(dec, make_problem(T=2), flow=flow)
z = torch.zeros(1, 32, 128, 256, device="cuda")
g = torch.empty_like(z)
for _ in range(5):
    prob.closure(z, g)
torch.cuda.synchronize()
ms = []
for _ in range(5):
    t0 = time.perf_counter()
    for _ in range(40):
        prob.closure(z, g)
    torch.cuda.synchronize()
    ms.append((time.perf_counter() - t0) / 40 * 1e3)
print(json.dumps({"lib": os.path.basename(os.environ.get("VAEVAR_LIB", "head")), "ms_min": min(ms),
                  "ms_median": statistics.median(ms)}))
