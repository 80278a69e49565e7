"""Swin-tower GEMM shapes (bf16x6 class; dim 96 / 192 towers, 6 groups folded into M) at the engine's tile choice:
time per call and effective HBM rate of the algorithmic bytes (A + B + C once). Development tool."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
shapes = [(49152, 288, 96), (49152, 96, 96), (49152, 384, 96), (49152, 96, 384),
          (12288, 576, 192), (12288, 192, 192), (12288, 768, 192), (12288, 192, 768),
          (49152, 96, 288)]
tiles = [int(t) for t in os.environ.get("TILES", "-1").split(",")]
for (M, N, K) in shapes:
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * 0.05
    ctx.gemm_register_weight(B)
    row = {"M": M, "N": N, "K": K}
    for t in tiles:
        for _ in range(3):
            ctx.gemm(A, B, tile=t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 30
        e0.record()
        for _ in range(n):
            ctx.gemm(A, B, tile=t)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        byt = 4.0 * (M * K + N * K + M * N)
        row[f"t{t}"] = [round(us, 1), round(byt / us / 1e6, 2)]  # us, TB/s
    print(json.dumps(row), flush=True)
    del A, B
