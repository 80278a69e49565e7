"""Run one GEMM shape/tile N times (for rocprofv3 PMC passes); PRE=1 registers B (split planes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context
M, N, K, t, n = (int(x) for x in sys.argv[1:6])
ctx = Context.get(0)
A = torch.rand(M, K, device="cuda") * 2 - 1
B = torch.rand(N, K, device="cuda") * 2 - 1
if os.environ.get("PRE"):
    ctx.gemm_register_weight(B)
for _ in range(n):
    ctx.gemm(A, B, tile=t)
torch.cuda.synchronize()
