"""GEMM microbenchmark over the decoder's GEMM shapes and tile variants (development tool)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
shapes = [(2048, 1024, 4608), (2048, 3456, 1152), (2048, 1152, 1152), (2048, 4608, 1152), (2048, 1152, 4608), (2048, 1152, 3456),
          (8192, 288, 96), (8192, 96, 384), (2048, 576, 192), (2048, 192, 768), (4096, 4608, 1152), (4096, 1152, 4608)]
tiles = [int(t) for t in os.environ.get("TILES", "2,16,4").split(",")]
res = []
for (M, N, K) in shapes:
    A = torch.rand(M, K, device="cuda") * 2 - 1
    B = torch.rand(N, K, device="cuda") * 2 - 1
    row = {"M": M, "N": N, "K": K}
    for t in tiles:
        try:
            for _ in range(3):
                ctx.gemm(A, B, tile=t)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                ctx.gemm(A, B, tile=t)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            row[f"t{t}"] = round(2 * M * N * K / us / 1e6, 1)
        except Exception as ex:
            row[f"t{t}"] = str(ex)[:40]
    print(json.dumps(row), flush=True)
